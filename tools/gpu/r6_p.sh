#!/bin/bash
# SYNC v2 (one merger per head hands the merged rows to the head's other workgroups): test, A/B, stats
O=gpurun_out/r6p; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_inference_gpu.py -k "long_context" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
for rep in 1 2; do
  for sy in 1 0; do
    NXD_DECODE_ATTN_SYNC=$sy timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 4 --report $O/r_${sy}_$rep.json > $O/b_${sy}_$rep.log 2>&1 || { tail -30 $O/b_${sy}_$rep.log; exit 1; }
    python -c "import json; r=json.load(open('$O/r_${sy}_$rep.json')); print('sync $sy rep $rep', round(r['token_generation']['ms_per_token_p50'],4))"
  done
done
rm -rf $O/prof
NXD_DECODE_ATTN_SYNC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 2 --report $O/report_prof.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $S $O/kernel_stats_sync.csv; rm -rf $O/prof
head -4 $O/kernel_stats_sync.csv | cut -c1-140
