#!/bin/bash
# GEMV early epilogue / prologue reads (NXD_DECODE_EPI_PF) A/B on Llama-3.2-1B bs=1 decode + the decode GPU tests.
set -o pipefail
O=gpurun_out/r3dec4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for v in 0 1 0 1; do
  NXD_DECODE_EPI_PF=$v timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_pf$v.json > $O/bench_pf$v.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/report_pf$v.json'));print('pf=$v', d['token_generation'])" >> $O/summary.txt
done
