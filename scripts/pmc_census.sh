#!/bin/bash
# Member-kernel census counters: the instruction-mix and
# LDS passes over one member-plan bench config, one rocprofv3 run per pass.
# usage: scripts/pmc_census.sh OUTDIR [config] [kernel regex]
set -o pipefail
OUT=${1:-gpurun_out/census}
CFG=${2:-c3}
RX=${3:-"member_chunk|crc_rows"}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_VSKIPPED SQ_INSTS_VALU_CVT" \
           "SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VALU2 SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RX" \
      --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --also "" --no-e2e > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt
