"""Summarise rocprofv3 --pmc counter_collection.csv files: per counter, the mean
over dispatches of the per-dispatch sum (over the XCD/SE dimensions), plus the
kernel duration from the matching kernel_trace.csv.
usage: python tools/pmc_summary.py <dir with p*/ subdirs> [kernel substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, sub=""):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if sub not in row.get("Kernel_Name", ""):
                continue
            vals[row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
    durs = []
    for f in glob.glob(os.path.join(d, "*", "*_kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            if sub in row.get("Kernel_Name", ""):
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    out = {k: sum(v.values()) / len(v) for k, v in sorted(vals.items())}
    for k, v in out.items():
        print(f"{k:28s} {v:16.4g}")
    if durs:
        print(f"{'duration_ms (profiled)':28s} {sum(durs) / len(durs):16.4g}  (n={len(durs)})")
    g = out.get("GRBM_GUI_ACTIVE")
    # MI355X: GRBM_GUI_ACTIVE is counted once per XCD (8), the SQ MFMA-busy cycles per
    # SIMD over 256 CUs x 4 SIMDs; the sums above run over those instances
    if g and durs:
        cyc = g / 8
        print(f"{'clock_GHz':28s} {cyc / (sum(durs) / len(durs) * 1e6):16.4g}  (GRBM_GUI_ACTIVE / 8 XCDs / duration)")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in out:
            print(f"{'mfma_busy_frac':28s} {out['SQ_VALU_MFMA_BUSY_CYCLES'] / (256 * 4 * cyc):16.4g}"
                  "  (MFMA busy cycles / (256 CUs x 4 SIMDs x GPU cycles))")
    return out


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
