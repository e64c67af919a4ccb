#!/bin/bash
# Round 4: decode GEMV non-temporal weight loads (NXD_DECODE_NT) and per-wave register RMSNorm
# prologue (NXD_DECODE_FN), alternating A/B on Llama-3.2-1B bs=1, + the decode GPU tests + kernel stats.
set -o pipefail
O=gpurun_out/r4dec; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_inference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    NXD_DECODE_NT=$1 NXD_DECODE_FN=$2 timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_nt$1_fn$2_$rep.json > $O/bench_nt$1_fn$2_$rep.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('$O/report_nt$1_fn$2_$rep.json'));print('nt=$1 fn=$2 rep=$rep', d['token_generation'])" >> $O/summary.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 2 > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \; ; find $O/prof -name "*.csv" -delete
