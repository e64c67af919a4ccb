#!/bin/bash
# Round 4: TP=1 halves -- stagger sweep on the 1-GPU bench (one box, alternating).
set -o pipefail
O=gpurun_out/r4tp1st; mkdir -p $O
export TMPDIR=/tmp
for st in 2 0 1 3 2; do
  NXD_SP_STAGGER=$st timeout -k 10 500 python bench.py --steps 6 --warmup 2 > $O/bench_$st.json 2> $O/bench.err || exit $?
  echo "stagger=$st $(tail -n 1 $O/bench_$st.json)" >> $O/summary.txt
done
