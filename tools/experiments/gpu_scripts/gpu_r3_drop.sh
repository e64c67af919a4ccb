#!/bin/bash
# In-kernel attention dropout: numerics vs the fp32 host path, FA regression tests, TF/s with / without.
set -o pipefail
mkdir -p gpurun_out/r3drop
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_attention_dropout_gpu.py tests/test_kernels_gpu.py -m gpu -x -v -k "dropout or flash or attn" --timeout 300 --timeout-method thread > gpurun_out/r3drop/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_fa_dropout.py > gpurun_out/r3drop/fa_dropout.jsonl 2>&1 || exit $?
