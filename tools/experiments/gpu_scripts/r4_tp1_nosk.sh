#!/bin/bash
# Round 4: TP=1 halves with / without stream-K GEMMs (the halves' GEMMs run beside other kernels).
set -o pipefail
O=gpurun_out/r4tp1nosk; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 1; do
    NXD_GEMM_NO_STREAMK=$v timeout -k 10 500 python bench.py --steps 6 --warmup 2 > $O/bench_${v}_${rep}.json 2> $O/bench.err || exit $?
    echo "no_streamk=$v rep=$rep $(tail -n 1 $O/bench_${v}_${rep}.json)" >> $O/summary.txt
  done
done
