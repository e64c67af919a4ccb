#!/bin/bash
# round 5 P: per-kernel split of the final decode path (batch 1: VALU dot2 GEMVs; batch 8: MFMA rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5p
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for bs in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bs$bs -o run -- python3 -u bench_inference.py --prompt 128 --new 128 --batch $bs --runs 2 --report $O/report_bs$bs.json > $O/bs$bs.log 2>&1 || { tail -20 $O/bs$bs.log; exit 1; }
  f=$(find /tmp/prof_bs$bs -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] || { tail -5 $O/bs$bs.log; exit 1; }
  cp "$f" $O/kernel_stats_bs$bs.csv
done
python3 - <<'PY'
import csv
for bs in (1, 8):
    rows = list(csv.DictReader(open(f"gpurun_out/r5p/kernel_stats_bs{bs}.csv")))
    print(f"== batch {bs}")
    for r in rows[:8]:
        n = r["Name"].replace("void nxd::", "").replace("(nxd::dfused::Params)", "").replace("(nxd::dattn::Params)", "")[:64]
        print(f"  {n:64s} calls {r['Calls']:>6} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
