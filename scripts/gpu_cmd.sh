set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/default.json 2> gpurun_out/default.err || { echo bench failed; tail -5 gpurun_out/default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/default.json').read().strip().splitlines()[-1])
for k,v in [('c2',d)]+list(d['also'].items()): print(k, v['value'], v['ms_per_step'], v['roofline']['frac'], v['roofline']['path_frac'], v['roofline']['stage_ms'], (v.get('cpu_baseline') or {}).get('value'))"
