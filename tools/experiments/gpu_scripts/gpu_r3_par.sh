#!/bin/bash
set -o pipefail
D=gpurun_out/r3par; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_parallel_gpu.py tests/test_bench_gpu.py tests/test_wgrad_gemm_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit $?
