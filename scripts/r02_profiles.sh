#!/bin/bash
# Round-2 evidence: PMC traffic of the dominant kernels (C2, C3, C5), rocprof
# kernel stats of the default bench, and the default bench line itself.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_r02
mkdir -p $O
bash scripts/pmc_traffic.sh r02 c3 member_chunk_kernel > $O/t_c3.log 2>&1 || { echo "c3 traffic failed"; tail -5 $O/t_c3.log; exit 1; }
tail -1 $O/t_c3.log | cut -c1-300
bash scripts/pmc_traffic.sh r02 c2 onepass16_kernel > $O/t_c2.log 2>&1 || { echo "c2 traffic failed"; tail -5 $O/t_c2.log; exit 1; }
tail -1 $O/t_c2.log | cut -c1-300
bash scripts/pmc_traffic.sh r02 c5 decode_kernel > $O/t_c5.log 2>&1 || { echo "c5 traffic failed"; tail -5 $O/t_c5.log; exit 1; }
tail -1 $O/t_c5.log | cut -c1-300
bash scripts/pmc_traffic.sh r02 c4 "correcting_build_lds_kernel|correcting_scan_kernel" "correcting_build_kernel + correcting_scan_kernel" > $O/t_c4.log 2>&1 || { echo "c4 traffic failed"; tail -5 $O/t_c4.log; exit 1; }
tail -1 $O/t_c4.log | cut -c1-300
cp profiles/r02_pmc_traffic_c*.json $O/ 2>/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 10 --warmup 2 > $O/bench_prof.log 2>&1 || { echo "stats failed"; tail -5 $O/bench_prof.log; exit 1; }
find $O/stats -name '*kernel_stats.csv' -exec cp {} $O/r02_default_kernel_stats.csv \;
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-600
