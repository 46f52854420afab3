set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for v in ab pf8 pf16; do
  env DG_LIB_VARIANT=$v timeout -k 10 300 python scripts/ab_bench.py --config c4 --steps 20 --warmup 5 > gpurun_out/c4_ab.json 2> gpurun_out/c4_ab.err || { echo "c4 $v failed"; tail -5 gpurun_out/c4_ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4_ab.json').read().strip().splitlines()[-1]); print('c4 $v', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline']['stage_ms_profile'].get('crc64'))"
done
done
bash scripts/pmc_probe.sh gpurun_out/probe8 c4 crc_segments_wide TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,TCP_PENDING_STALL_CYCLES_sum,GRBM_GUI_ACTIVE
