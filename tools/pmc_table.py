"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel name, the mean of each counter
over dispatches (and derived ratios when present).  python tools/pmc_table.py <csv> [kernel-substring]"""
import csv
import sys
from collections import defaultdict


SIMDS = 256 * 4   # MI355X: 256 CUs x 4 SIMDs


def mfma_busy_fraction(mfma_busy_cycles: float, grbm_gui_active: float) -> float:
    """Share of the chip's SIMD-cycles in which a matrix instruction executed.

    SQ_VALU_MFMA_BUSY_CYCLES sums the matrix-pipe cycles of every MFMA on the chip (32 per
    v_mfma_f32_32x32x16_bf16, 16 per 16x16x32: MI355X_MICROARCH.md, cycle constants);
    GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs, so / 8 is the dispatch's length in cycles.
    """
    return mfma_busy_cycles / (SIMDS * grbm_gui_active / 8.0)


def main(path, pat=""):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        if pat and pat not in name:
            continue
        key = (name[:70], r.get("Dispatch_Id"))
        vals[name[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c, v in sorted(m.items()):
            print(f"  {c:32s} {v:16.1f}")
        if "SQ_WAVE_CYCLES" in m:
            w = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_BUSY_CYCLES"):
                if c in m:
                    print(f"  {c}/WAVE_CYCLES = {m[c] / w:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            print(f"  MFMA busy = {100 * mfma_busy_fraction(m['SQ_VALU_MFMA_BUSY_CYCLES'], m['GRBM_GUI_ACTIVE']):.1f} %")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
            print(f"  LDS conflict share = {m['SQ_LDS_BANK_CONFLICT'] / max(m['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
        if "TCC_HIT_sum" in m:
            print(f"  L2 hit = {m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
