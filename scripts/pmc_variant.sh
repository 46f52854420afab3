#!/bin/bash
# SQ counters of one kernel for several library variants (2 passes each).
# usage: scripts/pmc_variant.sh OUT CONFIG KERNEL_REGEX VARIANT...
set -o pipefail
O=gpurun_out/$1; C=$2; K=$3; shift 3
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
             "SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    DG_LIB_VARIANT=$v timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $O/$v/p$i -o pmc -- python3 scripts/ab_bench.py --config $C --steps 2 --warmup 1 > $O/$v.p$i.log 2>&1 || { echo "$v pass $i rc=$?"; tail -3 $O/$v.p$i.log; exit 1; }
  done
  echo "== $v"; python3 scripts/pmc_summary.py $O/$v | tail -n +2
done
