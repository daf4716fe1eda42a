#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc pass (counter_collection.csv, one row
per dispatch and counter): kernels whose name contains SUBSTR, every counter
averaged over their dispatches, plus the derived shares the SQ counters give
(MI355X_MICROARCH.md 'rocprofv3 PMC slots': WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~ WAVE_CYCLES) and, with GRBM_GUI_ACTIVE and a kernel trace,
the effective clock.  Usage: sq_summary.py PASS_DIR SUBSTR [LABEL]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d, sub = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else d
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        if sub.replace(" ", "") in r["Kernel_Name"].replace(" ", ""):
            vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    dur = {}
    for p in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    ids = sorted(vals)
    if not ids:
        print(json.dumps({"label": label, "error": "no dispatch of " + sub}))
        return
    mean = {c: sum(vals[i][c] for i in ids) / len(ids) for c in vals[ids[0]]}
    out = {"label": label, "kernel": names[ids[0]][:90], "dispatches": len(ids), "mean": {k: float(f"{v:.4g}") for k, v in mean.items()}}
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in mean:
                out[k + "_share"] = round(mean[k] / wc, 4)
    ms = [dur[i] for i in ids if i in dur]
    if ms:
        out["ms"] = round(sum(ms) / len(ms), 4)
        if "GRBM_GUI_ACTIVE" in mean:  # summed over the 8 XCDs
            out["eff_clock_ghz"] = round(mean["GRBM_GUI_ACTIVE"] / 8 / (out["ms"] * 1e-3) / 1e9, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
