#!/bin/bash
# Instruction-mix PMC passes over one bench config (no trace domains mixed in).
# usage: scripts/pmc_quick.sh OUTDIR "bench args"
set -o pipefail
OUT=${1:-gpurun_out/pmcq}
ARGS=${2:---steps 3 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "onepass|crc_|serialize|correcting|decode_kernel|member" \
      --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT
