#!/bin/bash
# rocprofv3 kernel stats of one MoE layer fwd+bwd (Mixtral shapes, 16384 tokens), per expert-GEMM backend.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/moeprof
for b in grouped loop; do
  MOE_TOKENS=16384 MOE_BACKENDS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/moeprof/$b -o run -- python3 tools/bench_moe_layer.py > gpurun_out/moeprof/$b.log 2>&1 || exit $?
done
find gpurun_out/moeprof -name '*kernel_trace*' -delete
find gpurun_out/moeprof -type f -size +2M -delete; du -sh gpurun_out/moeprof
