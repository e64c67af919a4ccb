#!/bin/bash
# Round 4: per-stream kernel trace of the emulated TP=8 / TP=4 rank with the link model (8 layers):
# where the step loses time against max(compute, link).
set -o pipefail
O=gpurun_out/r4trace; mkdir -p $O
export TMPDIR=/tmp
for cfg in "8 400 2" "8 400 1" "4 200 2"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$1_$3 -o run --output-format csv -- python -u tools/emulate_tp_rank.py --tp $1 --layers 8 --steps 2 --warmup 1 --link-gbps $2 --sp-streams $3 > $O/emu_$1_$3.log 2>&1 || exit $?
  T=$(find $O/prof_$1_$3 -name "run_kernel_trace.csv" | head -1)
  python tools/stream_timeline.py $T --json >> $O/timeline.jsonl || exit $?
  head -1 $T > $O/trace_head.csv
  python - "$T" "$O/trace_tp$1_s$3_laststep.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
lo = ad[-3] if len(ad) >= 3 else 0
keep = ["Kernel_Name", "Start_Timestamp", "End_Timestamp"] + [k for k in ("Stream_Id", "Queue_Id") if k in rows[0]]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=keep, extrasaction="ignore")
    w.writeheader()
    for r in rows[lo:]:
        r["Kernel_Name"] = r["Kernel_Name"][:80]
        w.writerow(r)
PY
  find $O/prof_$1_$3 -name "*.csv" -delete
done
