#!/bin/bash
# Kernel times in isolation (A/B build, CRC on the run stream): C2 and C3.
set -o pipefail
O=gpurun_out/${1:-iso}
mkdir -p $O
export TMPDIR=/tmp
for c in c2 c3; do
  DG_LIB_VARIANT=ab DG_SERIAL_CRC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- python3 scripts/ab_bench.py --config $c --steps 5 --warmup 1 > $O/$c.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $O/$c.log; exit 1; }
  echo "== $c"; tail -1 $O/$c.log | cut -c1-300
  find $O/$c -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-4 | grep -v "at::native\|rocclr" | head -12
done
