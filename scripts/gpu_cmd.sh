set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shift.py tests/test_gpu_members_adversarial.py tests/test_gpu_parity.py > gpurun_out/t_route.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/t_route.log; exit 1; }
tail -2 gpurun_out/t_route.log
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { echo "bench $* failed"; tail -5 gpurun_out/b.err; exit 1; }; python3 -c "
import json; d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1])
for k,v in [('head',d)]+list(d.get('also',{}).items()): print('$*', k, v['value'], v['ms_per_step'], v['roofline']['stage_ms'])"; }
run --steps 20 --warmup 5 --also none
run --steps 20 --warmup 5 --also none
run --steps 100 --warmup 20 --also none
run --steps 20 --warmup 5 --also c3,c3s,c4o
