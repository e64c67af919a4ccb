#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3wg
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3wg/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_wgrad.py "$@" > gpurun_out/r3wg/bench.jsonl 2>&1 || exit $?
