#!/bin/bash
# GPU session: the -m gpu suite, then the default bench line (C2 + also C3/C4/C5).
set -o pipefail
O=gpurun_out/${1:-r02c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
cat $O/bench.json
