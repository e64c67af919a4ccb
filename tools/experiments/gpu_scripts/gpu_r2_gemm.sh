#!/bin/bash
# GEMM layout A/B + per-TP-degree compute floor (one GPU)
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 400 python tools/bench_gemm_layouts.py > gpurun_out/r2/gemm_layouts.jsonl 2> gpurun_out/r2/gemm_layouts.err || exit $?
timeout -k 10 500 python tools/profile_tp_shapes.py --tp 1 2 4 8 > gpurun_out/r2/tp_shapes.jsonl 2> gpurun_out/r2/tp_shapes.err
