#!/bin/bash
# prof counters of single C3 pairs in member mode (scripts/onepass_phases.py --offset)
set -o pipefail
O=gpurun_out/one
mkdir -p $O
for i in "$@"; do
  DG_MEMBERS=1 DG_LIB_VARIANT=prof timeout -k 10 120 python scripts/onepass_phases.py --config c3 --pairs 1 --offset $i > $O/p$i.json 2>&1 || { echo "rc=$?"; tail -5 $O/p$i.json; exit 1; }
  echo "pair $i"; tail -1 $O/p$i.json
done
