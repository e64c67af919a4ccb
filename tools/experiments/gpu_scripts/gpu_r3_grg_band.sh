#!/bin/bash
# 256-tile grouped fwd/dgrad: L2 raster band (NXD_GRG_BAND) and ring depth (NXD_GRG_STAGES) sweep.
set -o pipefail
O=gpurun_out/r3grg; mkdir -p $O
export TMPDIR=/tmp
NXD_GRG_STAGES=5 timeout -k 10 200 python -u -m pytest tests/test_moe_gpu.py -m gpu -x -q -k grouped_gemm --timeout 120 --timeout-method thread > $O/pytest_s5.log 2>&1 || exit $?
for cfg in "4 4" "5 4" "4 8" "5 8" "4 16"; do
  set -- $cfg
  NXD_GRG_STAGES=$1 NXD_GRG_BAND=$2 timeout -k 10 200 python -u tools/bench_grouped_gemm.py > $O/s$1_b$2.jsonl 2>&1 || exit $?
done
