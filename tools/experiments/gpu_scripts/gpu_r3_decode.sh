#!/bin/bash
# Fused decode attention + o_proj: GPU tests, then Llama-3.2-1B bs=1 decode (prompt 128, 256 new) on / off.
set -o pipefail
O=gpurun_out/r3dec; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_inference_gpu.py -m gpu -x -v -k "fused or graph_decode or greedy" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for v in 1 0 1 0; do
  NXD_DECODE_ATTN_OPROJ=$v timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_oproj$v.json > $O/bench_oproj$v.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/report_oproj$v.json'));print('oproj=$v', d['token_generation'])" >> $O/summary.txt
done
