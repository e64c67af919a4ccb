#!/bin/bash
# 256-tile grouped fwd/dgrad: L2 raster band sweep (NXD_GRG_BAND) on the Mixtral shapes.
set -o pipefail
O=gpurun_out/r3grg; mkdir -p $O
export TMPDIR=/tmp
for b in 2 8 16; do
  NXD_GRG_BAND=$b timeout -k 10 200 python -u tools/bench_grouped_gemm.py > $O/band$b.jsonl 2>&1 || exit $?
done
