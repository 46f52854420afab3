set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_TIMING=none AB_STEPS=100 AB_WARMUP=20 bash scripts/ab_multi.sh notime "v1938aff cur" "c2" 3 && AB_STEPS=100 AB_WARMUP=20 bash scripts/ab_multi.sh time "v1938aff cur" "c2" 2 && AB_TIMING=none AB_STEPS=20 AB_WARMUP=5 bash scripts/ab_multi.sh notime20 "v1938aff cur" "c2" 2
