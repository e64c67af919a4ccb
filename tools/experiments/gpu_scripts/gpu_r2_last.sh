#!/bin/bash
# Final check of the tree: SwiGLU kernel tests + tile A/B (fwd and bwd), full GPU suite, smoke, 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out/last
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "swiglu" --timeout 120 --timeout-method thread > gpurun_out/last/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/last/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
for r in 64 128; do
  NXD_SWIGLU_DUAL_ROWS=$r timeout -k 10 120 python tools/bench_swiglu_dual.py >> gpurun_out/last/kernel_ab.jsonl 2>> gpurun_out/last/kernel_ab.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench rows=$r rc=$rc"; exit $rc; }
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/last/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/last/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/last/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 5 --warmup 1 > gpurun_out/last/bench1.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/last/bench1.log
cat gpurun_out/last/kernel_ab.jsonl
exit $rc
