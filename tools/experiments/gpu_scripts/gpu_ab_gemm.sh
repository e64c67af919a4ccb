#!/bin/bash
# A/B: shipped exhaustive GEMM table vs runtime top-24 heuristic tuning, full 1-GPU bench each
mkdir -p gpurun_out/ab
NXD_GEMM_TABLE="" timeout -k 10 500 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/ab/bench_notable.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/ab/bench_table.log 2>&1
