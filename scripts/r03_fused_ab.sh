#!/bin/bash
# C2: in-kernel serialisation behind a decoupled look-back (DG_FUSED=1, ab build) vs scan + serialise
set -o pipefail
mkdir -p gpurun_out/fz
export TMPDIR=/tmp
for r in 1 2 3; do
for m in 0 1; do
  DG_LIB_VARIANT=ab DG_FUSED=$m timeout -k 10 200 python scripts/ab_bench.py --config c2 --steps 100 --warmup 20 > gpurun_out/fz/$m.$r.json 2> gpurun_out/fz/$m.$r.err || { echo "$m rc=$?"; tail -5 gpurun_out/fz/$m.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/fz/$m.$r.json').read().strip().splitlines()[-1]); print('$r fused=$m', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline'].get('stage_ms_profile'))"
done
done
