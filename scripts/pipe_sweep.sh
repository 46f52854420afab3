#!/bin/bash
# dg_encode_pipelined host-to-host rate (bin/pipe_bench, C only) over chunk sizes, pinned and pageable
set -o pipefail
O=gpurun_out/pipe
mkdir -p $O
for c in 512 1024 2048 4096; do
  timeout -k 10 200 delta-compression_amd/bin/pipe_bench 16384 65536 $c 5 1 > $O/pinned_$c.json || exit 1
  echo "pinned $c $(cut -c1-200 $O/pinned_$c.json | grep -o '"value": [0-9.]*')"
done
for c in 1024 2048; do
  timeout -k 10 300 delta-compression_amd/bin/pipe_bench 16384 65536 $c 5 0 > $O/pageable_$c.json || exit 1
  echo "pageable $c $(grep -o '"value": [0-9.]*' $O/pageable_$c.json)"
done
