#!/bin/bash
# Dual-layout SwiGLU backward: kernel + plumbing tests, training-path GPU tests, then the 1-GPU bench
# A/B (NXD_SWIGLU_DUAL=1 vs 0, alternating) and a rocprof step breakdown with it on.
set -o pipefail
mkdir -p gpurun_out/dual
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "swiglu" --timeout 120 --timeout-method thread > gpurun_out/dual/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/dual/pytest_kernels.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "llama or train or bench or smoke or parallel" --timeout 200 --timeout-method thread > gpurun_out/dual/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/dual/pytest_train.log; [ $rc -ne 0 ] && exit $rc
for d in 1 0 1 0; do
  NXD_SWIGLU_DUAL=$d timeout -k 10 400 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/dual/bench_dual$d.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench dual=$d rc=$rc"; exit $rc; }
  grep '"metric"' gpurun_out/dual/bench_dual$d.log | python -c "import sys,json;r=json.loads(sys.stdin.read());print('dual=$d', r['value'], r['ms_per_step'], r['loss'])" >> gpurun_out/dual/ab.txt
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/dual/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > gpurun_out/dual/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/dual/prof.log
cat gpurun_out/dual/ab.txt
exit $rc
