set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
for r in 1 2; do
for v in "DG_CORR_CRC=wide" "DG_CORR_CRC=fused" "DG_CORR_CRC=beside"; do
  env DG_LIB_VARIANT=ab $v timeout -k 10 300 python scripts/ab_bench.py --config c4 --steps 20 --warmup 5 > gpurun_out/c4_ab.json 2> gpurun_out/c4_ab.err || { echo "c4 $v failed"; tail -5 gpurun_out/c4_ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4_ab.json').read().strip().splitlines()[-1]); print('c4 $v', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline']['stage_ms_profile'].get('crc64'))"
done
done
for c in c2 c3; do
  timeout -k 10 300 python scripts/ab_bench.py --config $c --steps 20 --warmup 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "$c failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline'].get('stage_ms_profile',{}).get('crc64'))"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo bench failed; tail -5 gpurun_out/bench_default.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/bench_default.json'):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l)
    print('HEAD', d['config'].get('workload'), d['value'], d['ms_per_step'], d['roofline']['frac'])
    for x in d.get('also',[]):
        print(' ', x['config'].get('workload'), x['value'], x['ms_per_step'], x['roofline']['frac'])
PY
