#!/bin/bash
# Llama-3.2-1B bs=1 decode at the fork's notebook config (context 2048 -> 256 new tokens) and at the
# prompt-128 point, then a kernel trace of the notebook config.
O=gpurun_out/r6inf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 6 --report $O/report_p2048.json > $O/p2048.log 2>&1 || { tail -30 $O/p2048.log; exit 1; }
tail -3 $O/p2048.log
timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --batch 1 --runs 6 --report $O/report_p128.json > $O/p128.log 2>&1 || { tail -30 $O/p128.log; exit 1; }
tail -3 $O/p128.log
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 2 --report $O/report_prof.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $S $O/kernel_stats_p2048.csv
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1); gzip -c $T > $O/kernel_trace_p2048.csv.gz; rm -rf $O/prof
head -12 $O/kernel_stats_p2048.csv | cut -c1-200
