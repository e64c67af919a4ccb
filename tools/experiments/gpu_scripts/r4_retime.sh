#!/bin/bash
# Round 4: GEMM autotuner re-timing of the three leaders (NXD_GEMM_RETIME) A/B on the 1-GPU bench.
set -o pipefail
O=gpurun_out/r4retime; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 3; do
    NXD_GEMM_RETIME=$v timeout -k 10 500 python bench.py --steps 6 --warmup 2 > $O/bench_${v}_${rep}.json 2> $O/bench_${v}.err || exit $?
    echo "retime=$v rep=$rep $(tail -1 $O/bench_${v}_${rep}.json)" >> $O/summary.txt
  done
done
