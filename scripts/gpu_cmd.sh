set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_correcting.py "tests/test_gpu_fullsize.py::test_c4_full_batch" tests/test_gpu_pipelined.py tests/test_gpu_verbose.py > gpurun_out/t_corr.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/t_corr.log; exit 1; }
tail -3 gpurun_out/t_corr.log
for v in "" "DG_CORR_CRC_SEPARATE=1" "" "DG_CORR_CRC_SEPARATE=1"; do
  env DG_LIB_VARIANT=ab $v timeout -k 10 300 python scripts/ab_bench.py --config c4 --steps 20 --warmup 5 > gpurun_out/c4_ab.json 2> gpurun_out/c4_ab.err || { echo "c4 $v failed"; tail -5 gpurun_out/c4_ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4_ab.json').read().strip().splitlines()[-1]); print('c4 $v', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline']['stage_ms_profile'])"
done
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/default.json 2> gpurun_out/default.err || { echo bench failed; tail -5 gpurun_out/default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/default.json').read().strip().splitlines()[-1])
for k,v in [('c2',d)]+list(d['also'].items()): print(k, v['value'], v['ms_per_step'], v['roofline']['frac'], v['roofline']['path_frac'], v['roofline']['stage_ms'])"
