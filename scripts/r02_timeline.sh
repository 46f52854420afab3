#!/bin/bash
# per-pair timeline of the onepass chain (prof build): when waves start and how long they run
set -o pipefail
O=gpurun_out/${1:-tl}
mkdir -p $O
for m in 1 0; do
  DG_MEMBERS=$m DG_NO_MEMBERS=$((1-m)) DG_LIB_VARIANT=prof timeout -k 10 120 python scripts/onepass_phases.py --config c3 > $O/c3.m$m.json 2>&1 || { echo "rc=$?"; tail -5 $O/c3.m$m.json; exit 1; }
  tail -1 $O/c3.m$m.json
done
