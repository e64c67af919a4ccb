#!/bin/bash
# 256x256-tile grouped GEMM (NXD_GG_BIG=1): numerics, then kernel and layer timing vs the 128x128 kernel.
set -o pipefail
mkdir -p gpurun_out/ggbig
export TMPDIR=/tmp
NXD_GG_BIG=1 timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ggbig/pytest.log 2>&1 || exit $?
NXD_GG_BIG=1 timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/ggbig/bench_big.jsonl 2>&1 || exit $?
for b in 2 4; do
  NXD_GG_BIG=1 NXD_GG_BAND=$b timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/ggbig/bench_big_band$b.jsonl 2>&1 || exit $?
done
NXD_GG_BIG=1 MOE_BACKENDS=grouped,grouped timeout -k 10 300 python -u tools/bench_moe_layer.py > gpurun_out/ggbig/layer_big.jsonl 2>&1 || exit $?
