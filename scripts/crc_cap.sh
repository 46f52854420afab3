#!/bin/bash
# CRC grid cap A/B beside each differencing mode (the cap assumed 16 waves per CU)
set -o pipefail
O=gpurun_out/crccap
mkdir -p $O
for c in c3 c4 c2; do
  for b in default 512 1024 2048 4096 100000; do
    E=""; [ $b != default ] && E="DG_CRC_BLOCKS=$b"
    env DG_LIB_VARIANT=ab $E timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 10 --warmup 2 > $O/$c.$b.json 2> $O/$c.$b.err || { echo "$c $b rc=$?"; tail -3 $O/$c.$b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$c.$b.json').read().strip().splitlines()[-1]); print('$c $b', d['value'], d['ms_per_step'], d['roofline']['stage_ms'].get('crc64'))"
  done
done
