#!/bin/bash
# round 6 session ah: onepass phase shares (profiling build) of the table-tier
# lines: how much of a chain's cycles the table tier (phase C) is
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ah
mkdir -p $O
for c in c3s_chain c4o_chain c2; do
  timeout -k 10 300 env DG_LIB_VARIANT=prof python3 scripts/onepass_phases.py --config $c > $O/phases_$c.json 2> $O/phases_$c.err || { echo "$c fail"; tail -5 $O/phases_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/phases_$c.json')); print('$c', {k: d.get(k) for k in ('epochs','b_chunks','c_chunks','t_total','t_bc','t_c','t_diag','t_refill','t_ext')})"
done
