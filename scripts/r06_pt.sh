#!/bin/bash
# round 6 session pt: per-pair start / duration of the c3s chains: routed
# beside the CRC pass (base), routed after it (join), forced plain chain
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06pt
mkdir -p $O
timeout -k 10 200 env DG_LIB_VARIANT=pairtime python3 scripts/pair_time.py --config c3s > $O/base.json 2> $O/base.err || { echo base fail; tail -20 $O/base.err; exit 1; }
timeout -k 10 200 env DG_LIB_VARIANT=pairtime DG_CRC_FIRST=1 DG_CHAIN_JOIN=1 python3 scripts/pair_time.py --config c3s > $O/join.json 2> $O/join.err || { echo join fail; tail -20 $O/join.err; exit 1; }
timeout -k 10 200 env DG_LIB_VARIANT=pairtime python3 scripts/pair_time.py --config c3s_chain > $O/chain.json 2> $O/chain.err || { echo chain fail; tail -20 $O/chain.err; exit 1; }
for f in base join chain; do python3 -c "import json; r=json.load(open('$O/$f.json'))[-1]; print('$f', json.dumps(r))"; done
