#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "transpose or dgrad or wgrad" --timeout 120 --timeout-method thread > gpurun_out/r2/wgrad_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r2/bench_wgradt.log 2>&1 || exit $?
NXD_WGRAD_T=0 timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r2/bench_nowgradt.log 2>&1
