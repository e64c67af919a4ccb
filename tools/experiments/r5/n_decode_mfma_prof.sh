#!/bin/bash
# round 5 N: per-kernel split of decode on the MFMA GEMVs (batch 2 and 8; k-slice wave targets 2048 / 8192)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5n
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
prof() {  # tag bs env...
  local tag=$1 bs=$2; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$tag -o run -- python3 -u bench_inference.py --prompt 128 --new 128 --batch $bs --runs 2 --report $O/report_$tag.json > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  f=$(find /tmp/prof_$tag -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { tail -5 $O/$tag.log; exit 1; }
  cp "$f" $O/kernel_stats_$tag.csv
  echo "== $tag"; head -9 $O/kernel_stats_$tag.csv | cut -d, -f1-4 | cut -c1-120
}
prof mfma2048_bs8 8 NXD_DECODE_MFMA_WAVES=2048
prof mfma8192_bs8 8 NXD_DECODE_MFMA_WAVES=8192
prof mfma2048_bs2 2 NXD_DECODE_MFMA_WAVES=2048
prof valu_bs2 2 NXD_DECODE_MFMA=0
