#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters, one counter per pass
# (MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE in KiB, separate --pmc
# passes, no trace domains mixed in).  Summarised by scripts/pmc_traffic.py
# into profiles/<tag>_pmc_traffic_<config>.json, which bench.py reports as
# roofline.traffic.
# usage: scripts/pmc_traffic.sh TAG CONFIG KERNEL_REGEX [LABEL [OUTNAME]]
set -o pipefail
TAG=${1:-r01}
CFG=${2:-c2}
KRE=${3:-onepass16_kernel}
OUT=gpurun_out/pmct_${TAG}_${5:-$CFG}
export TMPDIR=/tmp
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/$c -o pmc -- python3 bench.py --config $CFG --also none --steps 5 --warmup 1 --no-cpu-baseline \
      > $OUT/$c.log 2>&1 || { echo "pass $c failed rc=$?"; tail -5 $OUT/$c.log; exit 1; }
done
python3 scripts/pmc_traffic.py $OUT $TAG $CFG "$KRE" "${4:-$KRE}" "${5:-$CFG}"
