#!/bin/bash
# Round-3 profile session on one box: rocprofv3 kernel-trace stats of the
# default bench command, and PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
# of each config's dominant kernel(s); C4's build and scan also apart.
set -o pipefail
mkdir -p gpurun_out/r03prof
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03prof/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03prof/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/r03prof/trace.log; exit 1; }
tail -c 600 gpurun_out/r03prof/trace.log
bash scripts/pmc_traffic.sh r03 c2 onepass16_kernel > gpurun_out/r03prof/p2.log 2>&1 || { echo "pmc c2 failed"; tail -5 gpurun_out/r03prof/p2.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c3 member_chunk_kernel > gpurun_out/r03prof/p3.log 2>&1 || { echo "pmc c3 failed"; tail -5 gpurun_out/r03prof/p3.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4 "correcting_build_lds_kernel|correcting_build_kernel|correcting_scan_kernel" "correcting_build_kernel + correcting_scan_kernel" > gpurun_out/r03prof/p4.log 2>&1 || { echo "pmc c4 failed"; tail -5 gpurun_out/r03prof/p4.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4 "correcting_build_lds_kernel|correcting_build_kernel" "correcting_build (LDS and memory-atomic builds)" c4_build > gpurun_out/r03prof/p4b.log 2>&1 || { echo "pmc c4 build failed"; tail -5 gpurun_out/r03prof/p4b.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4 correcting_scan_kernel correcting_scan_kernel c4_scan > gpurun_out/r03prof/p4s.log 2>&1 || { echo "pmc c4 scan failed"; tail -5 gpurun_out/r03prof/p4s.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c3s_chain onepass16_kernel > gpurun_out/r03prof/p3s.log 2>&1 || { echo "pmc c3s failed"; tail -5 gpurun_out/r03prof/p3s.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4o_chain onepass16_kernel > gpurun_out/r03prof/p4o.log 2>&1 || { echo "pmc c4o failed"; tail -5 gpurun_out/r03prof/p4o.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c5 decode_kernel > gpurun_out/r03prof/p5.log 2>&1 || { echo "pmc c5 failed"; tail -5 gpurun_out/r03prof/p5.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c5o decode_kernel > gpurun_out/r03prof/p5o.log 2>&1 || { echo "pmc c5o failed"; tail -5 gpurun_out/r03prof/p5o.log; exit 1; }
echo profiles done
