#!/bin/bash
# PP=2 x TP=2 gloo-gpu rehearsal: loss with the dual-layout SwiGLU on and off, then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/pp
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
for d in 1 0; do
  NXD_SWIGLU_DUAL=$d NXD_SWIGLU_DUAL_FWD=$d timeout -k 10 240 python bench.py --gpus 4 --model tiny --seq 512 --gbs 8 --steps 2 --warmup 1 --gloo-gpu --pp 2 > gpurun_out/pp/pp_dual$d.log 2>&1
  rc=$?; echo "dual=$d rc=$rc $(grep -o '"loss": [^,]*' gpurun_out/pp/pp_dual$d.log)" >> gpurun_out/pp/summary.txt; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pp/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pp/pytest_gpu.log
cat gpurun_out/pp/summary.txt
exit $rc
