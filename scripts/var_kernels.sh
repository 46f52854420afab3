#!/bin/bash
# Kernel times of library variants on one config (rocprofv3 kernel stats).
# usage: scripts/var_kernels.sh OUT CONFIG KERNEL_REGEX VARIANT...
set -o pipefail
O=gpurun_out/$1; C=$2; K=$3; shift 3
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  DG_LIB_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/ab_bench.py --config $C --steps 3 --warmup 1 > $O/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.log; exit 1; }
  echo "$v $(find $O/$v -name '*kernel_stats.csv' -exec cat {} \; | grep -E "$K" | cut -d, -f1-4 | tr '\n' ' ')"
done
