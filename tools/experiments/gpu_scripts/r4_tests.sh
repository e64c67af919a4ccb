#!/bin/bash
# Round 4 (3): per-shard gradient parity, TP=2 serving rehearsal, exhaustive-GEMM TP=4 rehearsal,
# bench through the public training API (1 GPU).
set -o pipefail
O=gpurun_out/r4tests; mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_shard_grad_parity_gpu.py > $O/shard_grad_parity.log 2>&1 || exit $?
timeout -k 10 600 $PT -s tests/test_spmd_inference_gpu.py > $O/spmd_inference.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_mode_rehearsal.py 2>/dev/null | grep '^{' > $O/gemm_mode_default.jsonl || exit $?
NXD_GEMM_TUNE=2 NXD_GEMM_NO_STREAMK=1 timeout -k 10 400 python -u tools/gemm_mode_rehearsal.py 2>/dev/null | grep '^{' > $O/gemm_mode_exhaustive_nosk.jsonl || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
