#!/bin/bash
O=gpurun_out/stp; mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u -m pytest tests/test_parallel_gpu.py tests/test_bench_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_$i.log 2>&1
  tail -3 $O/tests_$i.log
done
