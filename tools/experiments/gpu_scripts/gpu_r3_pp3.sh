#!/bin/bash
# PP variant 2 (LDS-DMA inside the MFMA bursts): numerics tests forced on, 3-way A/B, then the TP compute floors.
set -o pipefail
O=gpurun_out/r3pp3; mkdir -p $O
NXD_GRG_PP=2 NXD_WG_PP=2 timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py tests/test_moe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pp2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_pp_ab.py > $O/pp_ab3.jsonl 2>&1 || exit $?
bash tools/gpu_r3_tpfloor.sh || exit $?
