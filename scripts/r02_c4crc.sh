#!/bin/bash
# C4: the CRC beside the correcting build/scan, after it, and skipped (A/B build)
set -o pipefail
O=gpurun_out/c4crc
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for m in default DG_SERIAL_CRC DG_SKIP_CRC DG_CRC_FIRST; do
  if [ $m = default ]; then E=""; else E="$m=1"; fi
  env $E DG_LIB_VARIANT=ab timeout -k 10 200 python scripts/ab_bench.py --config c4 --steps 20 --warmup 3 > $O/$m.$r.json 2> $O/$m.$r.err || { echo "$m rc=$?"; tail -5 $O/$m.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$m.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$m', d['value'], d['ms_per_step'], s)"
done; done
