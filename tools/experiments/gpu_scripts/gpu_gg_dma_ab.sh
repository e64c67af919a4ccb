#!/bin/bash
# Grouped GEMM: LDS-DMA staging vs VGPR staging (NXD_GG_DMA), numerics first.
set -o pipefail
mkdir -p gpurun_out/ggdma
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ggdma/pytest.log 2>&1 || exit $?
NXD_GG_DMA=1 timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/ggdma/bench_dma.jsonl 2>&1 || exit $?
NXD_GG_DMA=0 timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/ggdma/bench_vgpr.jsonl 2>&1 || exit $?
MOE_BACKENDS=grouped,grouped timeout -k 10 300 python -u tools/bench_moe_layer.py > gpurun_out/ggdma/layer_dma.jsonl 2>&1 || exit $?
