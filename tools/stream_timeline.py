"""Overlap accounting of one training step from a rocprofv3 kernel trace (emulated TP rank with
the link model: the link is the `cu_stream_kernel` spin on its own stream).

For the last optimizer step (between the last two AdamW launch groups) it reports wall time and
the union-of-intervals time of: compute kernels (every stream but the link's), link work (the spin
and the receiving-side copies on the link stream), both at once, neither (GPU idle), and
compute-idle-while-link-busy (exposed link time), split into the forward half (up to the first
flash-attention backward launch) and the backward + optimizer half.

    python tools/stream_timeline.py gpurun_out/<dir>/run_kernel_trace.csv [--json]
"""
import csv
import json
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def clip(iv, lo, hi):
    return [[max(s, lo), min(e, hi)] for s, e in iv if e > lo and s < hi]


def main(path, as_json=False):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], q))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adamw_kernel" in r[2]]
    groups = []
    for i in adam:
        if groups and i - groups[-1][-1] < 50:
            groups[-1].append(i)
        else:
            groups.append([i])
    start = groups[-2][-1] + 1 if len(groups) >= 2 else 0
    end = groups[-1][-1] + 1
    sel = rows[start:end]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    # link work = everything on the link model's streams: the spin's stream and a stream that runs
    # nothing but copies (the receiving-side writes, on their own side stream since round 4)
    copyish = ("cu_stream_kernel", "copyBuffer", "elementwise_kernel", "CatArray")
    per = {}
    for s_, e_, n, q in sel:
        c = per.setdefault(q, [0, 0])
        c[0] += 1
        c[1] += any(k in n for k in copyish)
    lq = {q for s_, e_, n, q in sel if "cu_stream_kernel" in n}
    lq |= {q for q, (tot, cp) in per.items() if lq and cp >= 0.95 * tot}
    link = union([[s, e] for s, e, n, q in sel if q in lq])
    comp = union([[s, e] for s, e, n, q in sel if q not in lq])
    fab = [s for s, e, n, q in sel if "fab::" in n]
    tb = min(fab) if fab else t1
    res = {"trace": path, "kernels": len(sel), "streams": sorted({q for *_, q in sel})}
    for name, lo, hi in (("step", t0, t1), ("forward", t0, tb), ("backward+opt", tb, t1)):
        c, l = clip(comp, lo, hi), clip(link, lo, hi)
        both = length(intersect(c, l))
        busy = length(union(c + l))
        res[name] = {"wall_ms": round((hi - lo) / 1e6, 2), "compute_ms": round(length(c) / 1e6, 2),
                     "link_ms": round(length(l) / 1e6, 2), "overlap_ms": round(both / 1e6, 2),
                     "idle_ms": round((hi - lo - busy) / 1e6, 2),
                     "exposed_link_ms": round((length(l) - both) / 1e6, 2)}
    if as_json:
        print(json.dumps(res))
    else:
        for k, v in res.items():
            print(f"{k}: {v}")


if __name__ == "__main__":
    main(sys.argv[1], "--json" in sys.argv)
