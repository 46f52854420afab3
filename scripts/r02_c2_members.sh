#!/bin/bash
# C2 in member mode vs the plain chain, with and without the CRC (A/B build).
set -o pipefail
O=gpurun_out/c2m
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, env...
  local t=$1; shift
  env DG_LIB_VARIANT=ab "$@" timeout -k 10 200 python scripts/ab_bench.py --config c2 --steps 50 --warmup 10 > $O/$t.json 2> $O/$t.err || { echo "$t rc=$?"; tail -5 $O/$t.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$t.json').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
}
run plain
run plain_nocrc DG_SKIP_CRC=1
run mem DG_MEMBERS=1
run mem_nocrc DG_MEMBERS=1 DG_SKIP_CRC=1
run mem_serial DG_MEMBERS=1 DG_SERIAL_CRC=1
