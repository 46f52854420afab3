#!/bin/bash
# round 6 session p: the CRC rows pass beside onepass at C2: grid (blocks per
# CU), table type (byte / five-bit), pieces per batch (PF 2 / 4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p2
mkdir -p $O
run() {   # name variant env...
  local n=$1 v=$2; shift 2
  timeout -k 10 300 env DG_LIB_VARIANT=$v "$@" python scripts/ab_bench.py --config c2 --steps 30 --warmup 3 > $O/$n.json 2> $O/$n.err || { echo "$n fail"; tail -3 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n'.ljust(14), d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
}
for r in 1 2; do
  run vp.$r vp || exit 1
  run vp_b768.$r vp DG_CRC_BLOCKS=768 || exit 1
  run crc5_b512.$r crc5 || exit 1
  run crc5_b768.$r crc5 DG_CRC_BLOCKS=768 || exit 1
  run crc5_b1024.$r crc5 DG_CRC_BLOCKS=1024 || exit 1
  run pf4.$r crcpf4 || exit 1
done
