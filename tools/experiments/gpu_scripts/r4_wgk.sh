#!/bin/bash
# Round 4: TP=1 halves -- hand-written weight-gradient kernel for every shape (NXD_WGRAD_KERNEL=1) vs auto.
set -o pipefail
O=gpurun_out/r4wgk; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in auto 1; do
    NXD_WGRAD_KERNEL=$v timeout -k 10 500 python bench.py --steps 6 --warmup 2 > $O/bench_${v}_${rep}.json 2> $O/bench.err || exit $?
    echo "wgrad_kernel=$v rep=$rep $(tail -n 1 $O/bench_${v}_${rep}.json)" >> $O/summary.txt
  done
done
