#!/bin/bash
# round 6 session ad: kernel trace of C2 with the split serialiser
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_split2 -o run -- python3 scripts/ab_bench.py --config c2 --steps 10 --warmup 2 > $O/split2.json 2> $O/split2.err || { echo fail; tail -5 $O/split2.err; exit 1; }
find $O/ks_split2 -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-200
