#!/bin/bash
# MoE expert weight gradients on the token-major wgrad kernel: numerics, GEMM TF/s, layer, Mixtral 4L.
set -o pipefail
O=gpurun_out/r3moe; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_moe_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_grouped_gemm.py > $O/grouped_gemm.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_moe_layer.py > $O/moe_layer.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_mixtral_train.py --layers 4 --seq 4096 --mbs 2 --accum 4 --steps 3 > $O/mixtral_train.jsonl 2> $O/mixtral_train.err || exit $?
