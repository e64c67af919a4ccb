#!/bin/bash
# FA forward after the variant cleanup: numerics tests + TF/s on the bench shapes.
set -o pipefail
mkdir -p gpurun_out/r3fa
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_attention_gpu.py -m gpu -x -q -k "flash or attn or long" --timeout 300 --timeout-method thread > gpurun_out/r3fa/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_fa_shapes.py > gpurun_out/r3fa/fa_shapes.jsonl 2>&1 || exit $?
