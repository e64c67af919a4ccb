"""Summarise rocprofv3 --pmc CSVs (one or more passes) + a --kernel-trace CSV per hand-written kernel:
MFMA busy %, LDS bank-conflict rate, HBM bytes and achieved bandwidth.

MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs) / (1024 SIMDs x 2.4 GHz x kernel duration):
the fraction of the chip's matrix-core cycles that were busy.  FETCH_SIZE / WRITE_SIZE are in KiB.

    python tools/pmc_summary.py OUT.md trace.csv pass1.csv [pass2.csv ...]
"""
import csv
import sys
from collections import defaultdict

KEYS = ("fa::fwd_kernel", "fab::bwd_kernel", "fab::", "rms::", "rmsnorm", "swiglu", "xent", "adamw", "rope", "embedding",
        "gg::grouped_gemm", "dfused::", "dattn::")


def short(name):
    for k in KEYS:
        if k in name:
            return name.split("(")[0].replace("void ", "")[:60]
    return None


def main(out, trace, *passes):
    dur = defaultdict(list)
    for r in csv.DictReader(open(trace)):
        s = short(r["Kernel_Name"])
        if s:
            dur[s].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cnt = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in passes:
        for r in csv.DictReader(open(p)):
            s = short(r["Kernel_Name"])
            if s:
                cnt[s][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(s, r["Counter_Name"])].add(r["Dispatch_Id"])
    lines = ["| kernel | calls | avg us | MFMA busy % | LDS bank-conflict / LDS inst | HBM read GB/s | HBM write GB/s |",
             "|---|---|---|---|---|---|---|"]
    for s in sorted(cnt):
        c = cnt[s]
        n = max(len(disp[(s, k)]) for k in c) or 1
        avg = sum(dur[s]) / len(dur[s]) if dur[s] else float("nan")

        def per(k):
            return c[k] / max(1, len(disp[(s, k)])) if k in c else None

        busy, mfma = per("SQ_BUSY_CYCLES"), per("SQ_VALU_MFMA_BUSY_CYCLES")
        lds, conf = per("SQ_INSTS_LDS"), per("SQ_LDS_BANK_CONFLICT")
        fetch, write = per("FETCH_SIZE"), per("WRITE_SIZE")
        f = lambda x: "-" if x is None else f"{x:.1f}"  # noqa: E731
        mf = None if (mfma is None or avg != avg) else 100.0 * mfma / (1024 * 2.4e9 * avg * 1e-6)
        lc = None if not (lds and conf is not None) else conf / lds
        rd = None if fetch is None or avg != avg else fetch * 1024 / (avg * 1e-6) / 1e9
        wr = None if write is None or avg != avg else write * 1024 / (avg * 1e-6) / 1e9
        lines.append(f"| {s} | {n} | {f(avg)} | {f(mf)} | {'-' if lc is None else f'{lc:.3f}'} | {f(rd)} | {f(wr)} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
