#!/bin/bash
# Fused decode attention + o_proj: workgroup-count sweep and kernel stats (Llama-3.2-1B bs=1, prompt 128).
set -o pipefail
O=gpurun_out/r3dec2; mkdir -p $O
export TMPDIR=/tmp
for w in 64 128 256 64 128 256; do
  NXD_DECODE_OPROJ_WGS=$w timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_w$w.json > $O/bench_w$w.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/report_w$w.json'));print('wgs=$w', d['token_generation'])" >> $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 1 --report $O/prof_report.json > $O/prof.log 2>&1 || exit $?
find $O/prof -name '*kernel_trace*' -delete
