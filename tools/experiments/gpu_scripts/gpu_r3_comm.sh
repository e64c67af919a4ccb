#!/bin/bash
set -o pipefail
D=gpurun_out/r3comm; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_comm_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_cu_interference.py > $D/interference.jsonl 2>&1 || exit $?
