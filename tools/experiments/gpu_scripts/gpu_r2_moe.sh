#!/bin/bash
# MoE grouped GEMM: numerics tests + microbench.
set -o pipefail
mkdir -p gpurun_out/moe
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/moe/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/moe/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/moe/bench.jsonl 2> gpurun_out/moe/bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/moe/bench.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_moe_layer.py > gpurun_out/moe/layer.jsonl 2> gpurun_out/moe/layer.err
rc=$?; echo "layer rc=$rc" >> gpurun_out/moe/layer.err
exit $rc
