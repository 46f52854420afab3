set -o pipefail
mkdir -p gpurun_out
for v in prof pc1 pc2 pc3; do
  DG_LIB_VARIANT=$v timeout -k 10 300 python3 scripts/onepass_phases.py --config c4o_chain --pairs 2048 > gpurun_out/pcexp_$v.json 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/pcexp_$v.json; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/pcexp_$v.json') if l.startswith('{')][-1]); print('$v', 't_c', d['t_c'], 'c_chunks', d['c_chunks'], 'diff', d['stage_ms']['diff'], 'epochs', d['epochs'])"
done
