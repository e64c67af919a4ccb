#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "transpose or dgrad" --timeout 120 --timeout-method thread > gpurun_out/r2/dgrad_tests.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_gemm_layouts.py > gpurun_out/r2/gemm_layouts2.jsonl 2> gpurun_out/r2/gemm_layouts2.err || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r2/bench_dgradwt.log 2>&1 || exit $?
NXD_DGRAD_WT=0 timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r2/bench_nodgradwt.log 2>&1
