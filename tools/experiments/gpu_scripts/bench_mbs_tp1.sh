#!/bin/bash
# TP=1 micro-batch 1 vs 2 on one box (alternating), with peak allocated / reserved memory.
mkdir -p gpurun_out; out=gpurun_out/mbs_tp1_ab.txt; : > $out
timeout -k 10 400 python -u -m pytest tests/test_bench_gpu.py tests/test_emulate_tp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bench_gpu_tests.log 2>&1 || { tail -30 gpurun_out/bench_gpu_tests.log; exit 1; }
tail -1 gpurun_out/bench_gpu_tests.log
for m in 1 2 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --mbs $m > gpurun_out/ab_tmp.log 2>&1 || { tail -5 gpurun_out/ab_tmp.log; exit 1; }
  echo "mbs=$m $(tail -1 gpurun_out/ab_tmp.log)" | tee -a $out
done
