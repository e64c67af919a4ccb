#!/bin/bash
# Dual SwiGLU tile-height A/B (kernel timing), then the full GPU suite + smoke on the final tree.
set -o pipefail
mkdir -p gpurun_out/dual2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "swiglu" --timeout 120 --timeout-method thread > gpurun_out/dual2/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/dual2/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
for r in 64 128 128; do
  NXD_SWIGLU_DUAL_ROWS=$r timeout -k 10 120 python tools/bench_swiglu_dual.py >> gpurun_out/dual2/kernel_ab.jsonl 2>> gpurun_out/dual2/kernel_ab.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench rows=$r rc=$rc"; exit $rc; }
done
for d in 1 0 1 0; do
  NXD_SWIGLU_DUAL_FWD=$d timeout -k 10 400 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/dual2/bench_fwd$d.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench fwd=$d rc=$rc"; exit $rc; }
  grep '"metric"' gpurun_out/dual2/bench_fwd$d.log | python -c "import sys,json;r=json.loads(sys.stdin.read());print('dual_fwd=$d', r['value'], r['ms_per_step'], r['loss'], r['peak_mem_gib'])" >> gpurun_out/dual2/ab.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dual2/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/dual2/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/dual2/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/dual2/smoke.log
cat gpurun_out/dual2/kernel_ab.jsonl gpurun_out/dual2/ab.txt
exit $rc
