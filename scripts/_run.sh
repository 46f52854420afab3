set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
bash scripts/ab.sh ab25 "-- --config c5" && DG_LIB_VARIANT=prof timeout -k 10 120 python scripts/decode_phases.py > gpurun_out/dph.json 2> gpurun_out/dph.err; cat gpurun_out/dph.json
