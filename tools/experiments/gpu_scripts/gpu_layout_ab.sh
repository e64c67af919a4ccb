#!/bin/bash
# Prefill latency with / without the measured weight-layout pass (Llama-3.2-1B, bs 1)
set -o pipefail
mkdir -p gpurun_out/layout
for P in 128 2048; do
  timeout -k 10 300 python bench_inference.py --prompt $P --new 16 --runs 10 --report gpurun_out/layout/base_p$P.json > gpurun_out/layout/base_p$P.log 2>&1 || exit $?
  timeout -k 10 300 python bench_inference.py --prompt $P --new 16 --runs 10 --weight-layout --report gpurun_out/layout/wl_p$P.json > gpurun_out/layout/wl_p$P.log 2>&1 || exit $?
done
