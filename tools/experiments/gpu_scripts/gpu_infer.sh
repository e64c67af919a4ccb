#!/bin/bash
# Inference GPU tests + Llama-3.2-1B benchmark (+ kernel stats of one e2e generate).
mkdir -p gpurun_out/infer
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_inference_gpu.py -x -q > gpurun_out/infer/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/infer/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench_inference.py --prompt 2048 --new 256 --runs 5 --report gpurun_out/infer/benchmark_report.json > gpurun_out/infer/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/infer/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench_inference.py --prompt 128 --new 256 --runs 5 --report gpurun_out/infer/benchmark_report_p128.json > gpurun_out/infer/bench_p128.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/infer/bench_p128.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/infer/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --runs 1 --report gpurun_out/infer/prof_report.json > gpurun_out/infer/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/infer/prof.log
exit $rc
