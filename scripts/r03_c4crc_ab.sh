#!/bin/bash
# C4 CRC placement A/B (ab build): wide pass before the build vs forked beside the V scan
set -o pipefail
mkdir -p gpurun_out/c4crc
export TMPDIR=/tmp
for r in 1 2; do
for m in wide widebeside fused; do
  DG_LIB_VARIANT=ab DG_CORR_CRC=$m timeout -k 10 200 python scripts/ab_bench.py --config c4 --steps 20 --warmup 5 > gpurun_out/c4crc/$m.$r.json 2> gpurun_out/c4crc/$m.$r.err || { echo "$m rc=$?"; tail -5 gpurun_out/c4crc/$m.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4crc/$m.$r.json').read().strip().splitlines()[-1]); print('$r $m', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline'].get('stage_ms_profile',{}).get('crc64'))"
done
done
