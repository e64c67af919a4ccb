#!/bin/bash
# FA numerics tests + FA timing at the Llama-3-8B TP1 / TP8 head shapes.
set -o pipefail
mkdir -p gpurun_out/fa
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or rope_attention" > gpurun_out/fa/tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/fa/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_kernels.py --only fa > gpurun_out/fa/times.jsonl 2>&1
