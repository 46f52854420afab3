set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shift.py > gpurun_out/t_shift.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/t_shift.log; exit 1; }
tail -3 gpurun_out/t_shift.log
timeout -k 10 600 python bench.py --config c3 --also c3s,c3s_chain,c4o,c4o_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/shift.json 2> gpurun_out/shift.err || { echo bench failed; tail -5 gpurun_out/shift.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/shift.json').read().strip().splitlines()[-1])
for k,v in [('c3',d)]+list(d['also'].items()): print(k, v['value'], v['ms_per_step'], v['config']['onepass_chain'], v['roofline']['stage_ms'])"
AB_TIMING=none AB_STEPS=100 AB_WARMUP=20 bash scripts/ab_multi.sh notime "v1938aff cur" "c2" 2 && AB_STEPS=100 AB_WARMUP=20 bash scripts/ab_multi.sh time "v1938aff cur" "c2" 2
