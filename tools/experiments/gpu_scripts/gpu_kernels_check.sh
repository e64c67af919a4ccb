#!/bin/bash
# First GPU bring-up: kernel numerics + micro-benchmarks. Each GPU step has its own time limit;
# a crash/timeout (rc >= 124 or signal) stops the script before any further GPU work.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/kt.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/kt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bk.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bk.log
exit $rc
