set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash scripts/ab.sh ab35 "-- --config c4 --steps 5 --warmup 1" "-- --config c2"
