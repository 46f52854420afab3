#!/bin/bash
# PMC passes over a short bench run (one counter group per pass; no sys/runtime trace).
set -o pipefail
OUT=${1:-gpurun_out/pmc}
ARGS=${2:---steps 3 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "onepass|crc_seg|serialize|correcting|decode_kernel" \
      --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc done
