"""Per-category GPU time of the LAST optimizer step in a rocprofv3 kernel trace.

The last step is located as everything after the second-to-last AdamW launch group (the bench
runs warmup steps first, which include GEMM autotuning).  Usage:
    python tools/step_breakdown.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def cat(name: str) -> str:
    n = name
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "gemm(hipBLASLt)"
    for key, c in (("fab::", "flash_attn_bwd"), ("fa::fwd", "flash_attn_fwd"), ("optim::", "adamw/norm"),
                   ("swiglu", "swiglu"), ("rms::", "rmsnorm"), ("rope", "rope"), ("xent", "cross_entropy"),
                   ("emb", "embedding"), ("rccl", "rccl"), ("nccl", "rccl"), ("Fill", "torch fill"),
                   ("copy", "copies"), ("Copy", "copies"), ("rocclr", "copies")):
        if key in n:
            return c
    return "other:" + n[:60]


def main(path, split="adamw_kernel", by_kernel=False):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if split in r[2]]
    # group adam launches into steps (consecutive launches within a short index distance)
    groups = []
    for i in adam:
        if groups and i - groups[-1][-1] < 50:
            groups[-1].append(i)
        else:
            groups.append([i])
    if split == "adamw_kernel":
        start = groups[-2][-1] + 1 if len(groups) >= 2 else 0
        end = groups[-1][-1] + 1
    else:   # e.g. "emb": from the last forward's first kernel group to the end of the trace
        start, end = groups[-1][0], len(rows)
    sel = rows[start:end]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in sel:
        k = n[:110] if by_kernel else cat(n)
        tot[k] += (e - s) / 1e6
        cnt[k] += 1
    wall = (sel[-1][1] - sel[0][0]) / 1e6
    busy = sum(tot.values())
    print(f"last step: {len(sel)} kernels, wall {wall:.1f} ms, kernel-busy {busy:.1f} ms")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:25]:
        print(f"  {k:40s} {v:9.2f} ms  {100 * v / busy:5.1f}%  n={cnt[k]}")


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split", default="adamw_kernel", help="kernel-name marker of a step boundary ('emb' for a"
                    " forward+backward micro-batch trace without optimizer)")
    ap.add_argument("--by-kernel", action="store_true")
    a = ap.parse_args()
    main(a.trace, a.split, a.by_kernel)
