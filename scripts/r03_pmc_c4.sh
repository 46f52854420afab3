set -o pipefail
export TMPDIR=/tmp
bash scripts/pmc_traffic.sh r03 c4 "correcting_build_lds_kernel|correcting_build_kernel|correcting_scan_kernel" "correcting_build_kernel + correcting_scan_kernel" > gpurun_out/p4.log 2>&1 || { echo "pmc c4 failed"; tail -5 gpurun_out/p4.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4 "correcting_build_lds_kernel|correcting_build_kernel" "correcting_build (LDS and memory-atomic builds)" c4_build > gpurun_out/p4b.log 2>&1 || { echo "pmc c4 build failed"; tail -5 gpurun_out/p4b.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4 correcting_scan_kernel correcting_scan_kernel c4_scan > gpurun_out/p4s.log 2>&1 || { echo "pmc c4 scan failed"; tail -5 gpurun_out/p4s.log; exit 1; }
echo ok
