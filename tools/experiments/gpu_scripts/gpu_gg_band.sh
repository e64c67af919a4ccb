#!/bin/bash
# Grouped GEMM raster band sweep (NXD_GG_BAND row tiles per band).
set -o pipefail
mkdir -p gpurun_out/ggband
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ggband/pytest.log 2>&1 || exit $?
for b in 4 8 16 32; do
  NXD_GG_BAND=$b timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/ggband/band_$b.jsonl 2>&1 || exit $?
done
