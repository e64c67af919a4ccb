#!/bin/bash
# FA backward: numerics (incl. dropout) + drain-schedule A/B and ablations.
set -o pipefail
D=gpurun_out/r3fab; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_attention_dropout_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -k "dropout or flash_bwd" --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/fab_drain_ab.py > $D/drain_ab.jsonl 2>&1 || exit $?
