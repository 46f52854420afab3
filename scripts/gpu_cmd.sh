set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in none dominant all none dominant all; do AB_TIMING=$t AB_STEPS=100 AB_WARMUP=20 bash scripts/ab_multi.sh ev_$t "ab" "c2 c3" 1; done
