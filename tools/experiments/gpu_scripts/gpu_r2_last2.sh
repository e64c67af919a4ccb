#!/bin/bash
# SwiGLU token-major copies restricted to the dense MLP: kernel/plumbing tests, Llama HF parity, MoE GPU tests, bench.
set -o pipefail
mkdir -p gpurun_out/last2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_hf_parity_gpu.py tests/test_moe_gpu.py tests/test_graph_step_gpu.py tests/test_bench_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/last2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/last2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/last2/bench1.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/last2/bench1.log
exit $rc
