#!/bin/bash
mkdir -p gpurun_out/gemm
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gemm > gpurun_out/gemm/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gemm/pytest.log; [ $rc -ne 0 ] && exit $rc
export NXD_GEMM_TUNE_FILE=gpurun_out/gemm/tuned.txt
timeout -k 10 600 python tools/bench_gemm.py > gpurun_out/gemm/bench_gemm.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/gemm/bench_gemm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/gemm/bench1.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/gemm/bench1.log
exit $rc
