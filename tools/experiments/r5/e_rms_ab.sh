#!/bin/bash
# round 5 E: step-level A/B of the RMSNorm kernels (row-per-wave vs one row per workgroup), alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5e
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for r in 1 0; do
    NXD_RMS_ROWS=$r timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > $O/b_rows${r}_$i.json 2> $O/b_rows${r}_$i.err || { tail -20 $O/b_rows${r}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/b_rows${r}_$i.json')); print('rows=$r run $i', d['ms_per_step'], d['value'])"
  done
done
