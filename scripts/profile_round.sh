#!/bin/bash
# One profile session on a GPU box (replaces the per-round wrappers):
#   ks    rocprofv3 --kernel-trace --stats of each config run alone
#         (bench.py --config C --also none), its bench line beside it
#   calib FETCH_SIZE / WRITE_SIZE of scripts/micro/pmc_calib per access class
#   pmc   FETCH_SIZE / WRITE_SIZE passes of each config's dominant kernel(s)
#   path  FETCH_SIZE / WRITE_SIZE passes of every kernel of a step (all dg::
#         kernels but the input synthesis), for the path-level traffic
# usage: scripts/profile_round.sh TAG [ks|calib|pmc|path|all] [CONFIGS...]
# Outputs under gpurun_out/TAG/; scripts/profile_collect.py TAG copies the
# summaries into profiles/.
set -o pipefail
TAG=${1:?tag}
WHAT=${2:-all}
shift 2 2>/dev/null
CFGS=${*:-c2 c3 c4 c5 c5o c6 c2_defq c3s c3s_chain c4o c4o_chain}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$WHAT" = ks ] || [ "$WHAT" = all ]; then
  for c in $CFGS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$c -o run -- \
        python3 bench.py --config $c --also none --steps 20 --warmup 5 --no-cpu-baseline --no-e2e \
        --full-out $O/ks_$c/bench_full.json > $O/ks_$c.log 2>&1 || { echo "ks $c rc=$?"; tail -5 $O/ks_$c.log; exit 1; }
    tail -1 $O/ks_$c.log | cut -c1-200
  done
fi
if [ "$WHAT" = calib ] || [ "$WHAT" = all ]; then
  for k in ${CALIB:-stream16 dma16 stream8 dma4 rand16 rand4 store16 store16r}; do
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 60 rocprofv3 --pmc $c --kernel-include-regex "^$k" --output-format csv -d $O/calib_${k}_$c -o pmc -- \
          scripts/micro/pmc_calib $k > $O/calib_${k}_$c.log 2>&1 || { echo "calib $k $c rc=$?"; tail -5 $O/calib_${k}_$c.log; exit 1; }
    done
  done
  echo calib done
fi
if [ "$WHAT" = pmc ] || [ "$WHAT" = all ]; then
  for c in $CFGS; do
    case $c in
      c2|c2_defq|c3s_chain|c4o_chain) K=onepass16_kernel ;;
      c3|c6) K=member_chunk_kernel ;;
      c3s|c4o) K="onepass16_kernel|member_chunk_kernel" ;;
      c4) K="correcting_build_lds_kernel|correcting_build_kernel|correcting_scan_kernel" ;;
      c5|c5o) K=decode_kernel ;;
      *) continue ;;
    esac
    for p in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "$K" --output-format csv -d $O/pmc_${c}_$p -o pmc -- \
          python3 bench.py --config $c --also none --steps 5 --warmup 1 --no-cpu-baseline --no-e2e \
          --full-out $O/pmc_${c}_$p.json > $O/pmc_${c}_$p.log 2>&1 || { echo "pmc $c $p rc=$?"; tail -5 $O/pmc_${c}_$p.log; exit 1; }
    done
    echo "pmc $c done"
  done
fi
if [ "$WHAT" = path ] || [ "$WHAT" = all ]; then
  for c in $CFGS; do
    case $c in c2|c3|c4|c6|c2_defq) ;; *) continue ;; esac
    for p in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $p --kernel-include-regex "dg::" --kernel-exclude-regex "synth" \
          --output-format csv -d $O/path_${c}_$p -o pmc -- \
          python3 bench.py --config $c --also none --steps 5 --warmup 1 --no-cpu-baseline --no-e2e \
          --full-out $O/path_${c}_$p.json > $O/path_${c}_$p.log 2>&1 || { echo "path $c $p rc=$?"; tail -5 $O/path_${c}_$p.log; exit 1; }
    done
    echo "path $c done"
  done
fi
echo profile_round done
