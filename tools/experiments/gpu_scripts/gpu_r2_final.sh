#!/bin/bash
# Inference GPU tests (incl. the decode prefetch exactness test) + rocprof kernel stats of a 2-micro-batch bench step.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_inference_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_infer.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/final/pytest_infer.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > gpurun_out/final/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/final/prof.log
exit $rc
