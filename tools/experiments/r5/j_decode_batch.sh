#!/bin/bash
# round 5 J: Llama-3.2-1B decode throughput vs batch size (fused decode + hipGraphs), prompt 128, 256 new tokens
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5j
mkdir -p $O
export PYTHONUNBUFFERED=1
for bs in 1 2 4 8; do
  timeout -k 10 240 python -u bench_inference.py --prompt 128 --new 256 --batch $bs --runs 5 --report $O/report_bs$bs.json > $O/bs$bs.log 2>&1 || { tail -20 $O/bs$bs.log; exit 1; }
  tail -1 $O/bs$bs.log
done
