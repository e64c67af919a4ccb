#!/bin/bash
# 1-GPU bench A/B of the hipBLASLt in-process tuner knobs (top-N candidates, workspace).
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/ab/base.log 2>&1 || exit $?
NXD_GEMM_TUNE_CANDIDATES=64 timeout -k 10 500 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/ab/cand64.log 2>&1 || exit $?
NXD_GEMM_WORKSPACE_MB=512 timeout -k 10 400 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/ab/ws512.log 2>&1 || exit $?
