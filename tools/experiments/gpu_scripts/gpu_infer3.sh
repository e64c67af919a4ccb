#!/bin/bash
mkdir -p gpurun_out/infer3
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_inference_gpu.py -x -q > gpurun_out/infer3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/infer3/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench_inference.py --prompt 2048 --new 256 --runs 5 --report gpurun_out/infer3/report_bf16.json > gpurun_out/infer3/bench_bf16.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/infer3/bench_bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/infer3/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --runs 1 --report gpurun_out/infer3/prof_report.json > gpurun_out/infer3/prof.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/infer3/prof.log
exit $rc
