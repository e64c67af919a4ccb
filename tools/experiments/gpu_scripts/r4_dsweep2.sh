#!/bin/bash
# Round 4: fused attention + o_proj vs separate attention and o_proj GEMV launches on the round-4
# GEMVs (nt weight stream, operands ahead of the weights), alternating; kernel stats of the split path.
set -o pipefail
O=gpurun_out/r4dsw2; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in 1 0; do
    NXD_DECODE_ATTN_OPROJ=$v timeout -k 10 120 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/r.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
    python -c "import json;d=json.load(open('$O/r.json'));print('attn_oproj=$v rep=$rep', round(d['token_generation']['ms_per_token_p50'],4))" >> $O/summary.txt
  done
done
NXD_DECODE_ATTN_OPROJ=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 2 > $O/prof.log 2>&1 || exit $?
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats_split.csv
find $O/prof -name "*.csv" -delete
cat $O/summary.txt
