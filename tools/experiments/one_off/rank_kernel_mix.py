"""Kernel mix of each rank's LAST optimizer step from a multi-process rocprofv3 kernel trace (one
run_kernel_trace.csv per process, e.g. tools/gpu_r3_tp8rehearsal.sh: 8 gloo-gpu ranks of bench.py
sharing one GPU).  Per rank: kernel launches and busy time per category (tools/step_breakdown.py
categories), so the real TP + SP code path can be checked for stray copies / transposes /
element-wise kernels that the single-process TP-shape profile does not exercise.  Times are
inflated by the ranks sharing the GPU; counts are exact.

    python tools/rank_kernel_mix.py gpurun_out/r3tp8gg/prof
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_breakdown import cat  # noqa: E402


def last_step(rows):
    adam = [i for i, r in enumerate(rows) if "adamw_kernel" in r[2]]
    if len(adam) < 2:
        return rows
    groups = []
    for i in adam:
        if groups and i - groups[-1][-1] < 50:
            groups[-1].append(i)
        else:
            groups.append([i])
    start = groups[-2][-1] + 1 if len(groups) >= 2 else 0
    return rows[start:groups[-1][-1] + 1]


def main(root):
    files = sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True))
    out = []
    for fn in files:
        rows = []
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
        rows.sort()
        step = last_step(rows)
        n = defaultdict(int)
        t = defaultdict(float)
        for s, e, name in step:
            c = cat(name)
            n[c] += 1
            t[c] += (e - s) / 1e6
        rec = {"trace": os.path.relpath(fn, root), "kernels": len(step),
               "by_category": {c: {"n": n[c], "ms": round(t[c], 2)} for c in sorted(n, key=lambda c: -t[c])}}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r3tp8gg/prof")
