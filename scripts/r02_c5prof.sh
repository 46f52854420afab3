#!/bin/bash
# rocprofv3 kernel stats of the C5 bench line (which kernels make the decode step)
set -o pipefail
O=gpurun_out/c5prof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config c5 --also none --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-160 | head -20
