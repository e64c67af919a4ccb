#!/bin/bash
# Ping-pong main loops of the grouped row GEMM and the wgrad kernel: numerics tests with the PP
# variants forced on, then an in-process A/B, then the SP chunk bench, smoke and the default bench.
set -o pipefail
O=gpurun_out/r3pp; mkdir -p $O
NXD_GRG_PP=1 NXD_WG_PP=1 timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py tests/test_moe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pp.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_pp_ab.py > $O/pp_ab.jsonl 2>&1 || exit $?
bash tools/gpu_r3_spchunks.sh || exit $?
bash tools/gpu_r3_final.sh || exit $?
