#!/bin/bash
# round 5 K: per-kernel split of Llama-3.2-1B decode at batch 8 vs batch 1 (rocprofv3 kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5k
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for bs in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bs$bs -o run -- python3 -u bench_inference.py --prompt 128 --new 128 --batch $bs --runs 2 --report $O/report_bs$bs.json > $O/bs$bs.log 2>&1 || { tail -20 $O/bs$bs.log; exit 1; }
  f=$(find /tmp/prof_bs$bs -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { ls -R /tmp/prof_bs$bs | head; tail -5 $O/bs$bs.log; exit 1; }
  cp "$f" $O/kernel_stats_bs$bs.csv
  head -12 $O/kernel_stats_bs$bs.csv | cut -c1-160
done
