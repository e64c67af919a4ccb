"""Per-kernel average of every PMC counter over the dispatches of rocprofv3 --pmc output dirs, plus
derived ratios (MFMA busy of the CU cycles, wait shares, LDS conflicts).
Usage: python tools/pmc_avg.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, cn), v in per.items():
            vals[names[disp][:100]][cn].append(v)
for k, c in vals.items():
    print(k)
    avg = {cn: sum(v) / len(v) for cn, v in c.items()}
    for cn in sorted(avg):
        print(f"  {cn:28s} {avg[cn]:18.1f}  (n={len(c[cn])})")
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for cn in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if cn in avg:
                print(f"  {cn}/WAVE_CYCLES = {avg[cn] / wc:.3f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        # MFMA busy cycles summed over 1024 SIMDs vs GRBM_GUI_ACTIVE (summed over 8 XCDs)
        print(f"  MFMA busy = {100 * avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * avg['GRBM_GUI_ACTIVE'] / 8):.1f} %")
    if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
        print(f"  LDS conflict cycles / LDS active = {avg['SQ_LDS_BANK_CONFLICT'] / max(1, avg['SQ_LDS_IDX_ACTIVE']):.3f}")
