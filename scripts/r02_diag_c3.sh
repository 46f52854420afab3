#!/bin/bash
# Round-2 C3 diagnosis: bench line, per-phase counters (prof build), rocprof
# kernel stats, SQ instruction mix and HBM traffic of onepass16_kernel at C3.
set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "bench c3 rc=$?"; tail $O/c3.err; exit 1; }
cat $O/c3.json
DG_LIB_VARIANT=prof timeout -k 10 300 python scripts/onepass_phases.py --config c3 > $O/c3.phases.json 2> $O/c3.phases.err || { echo "phases rc=$?"; tail $O/c3.phases.err; exit 1; }
cat $O/c3.phases.json
DG_LIB_VARIANT=prof timeout -k 10 300 python scripts/onepass_phases.py --config c2 > $O/c2.phases.json 2> $O/c2.phases.err || { echo "phases rc=$?"; tail $O/c2.phases.err; exit 1; }
cat $O/c2.phases.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- python3 bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline > $O/c3prof.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
find $O/c3prof -name '*kernel_stats.csv' -exec cat {} \;
bash scripts/pmc_kernel.sh $O/pmc_c3 onepass16_kernel "--config c3 --steps 3 --warmup 1 --no-cpu-baseline" > $O/pmc_c3.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc_c3.log; exit 1; }
cat $O/pmc_c3.log
bash scripts/pmc_traffic.sh r02 c3 onepass16_kernel > $O/pmct.log 2>&1 || { echo "pmc traffic rc=$?"; tail -5 $O/pmct.log; exit 1; }
tail -3 $O/pmct.log
echo done
