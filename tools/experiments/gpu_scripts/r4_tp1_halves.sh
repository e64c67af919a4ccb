#!/bin/bash
# Round 4: TP=1 bench with the micro-batch as two staggered halves on two streams (no collectives:
# only kernel co-scheduling), alternating A/B on one box.
set -o pipefail
O=gpurun_out/r4tp1h; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 1; do
    NXD_SP_STREAMS_NO_SP=$v timeout -k 10 500 python bench.py --steps 6 --warmup 2 > $O/bench_${v}_${rep}.json 2> $O/bench_$v.err || exit $?
    echo "no_sp_halves=$v rep=$rep $(tail -1 $O/bench_${v}_${rep}.json)" >> $O/summary.txt
  done
done
