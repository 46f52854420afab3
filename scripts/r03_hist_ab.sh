set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -v -x --timeout 200 --timeout-method thread -k "tag_wrap or contention" > gpurun_out/tw.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/tw.log; exit 1; }
tail -4 gpurun_out/tw.log
AB_STEPS=5 AB_WARMUP=1 bash scripts/ab_multi.sh hist "h4 h6 h8" "c2 c3s_chain c4o_chain" 1
