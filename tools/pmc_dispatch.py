#!/usr/bin/env python3
"""Per-dispatch HBM traffic from two rocprofv3 passes (--pmc FETCH_SIZE and
--pmc WRITE_SIZE, each with --kernel-trace) of the same command.

Prints one JSON object per dispatch of kernels whose name contains SUBSTR, in
dispatch order: read bytes (gfx950: 2 x FETCH_SIZE x 1024, MI355X_MICROARCH.md
HBM section), write bytes (WRITE_SIZE x 1024), and the dispatch's duration in
the FETCH pass.  Usage: pmc_dispatch.py FETCH_DIR WRITE_DIR SUBSTR"""
import csv
import glob
import json
import sys


def rows(d, sub):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(path)):
        if sub.replace(" ", "") in r["Kernel_Name"].replace(" ", ""):  # spacing of template arguments varies
            out[int(r["Dispatch_Id"])] = (float(r["Counter_Value"]), r["Kernel_Name"])
    return out


def durations(d):
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not paths:
        return {}
    return {int(r["Dispatch_Id"]): (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in csv.DictReader(open(paths[0]))}


def main():
    fdir, wdir, sub = sys.argv[1], sys.argv[2], sys.argv[3]
    f, w, dur = rows(fdir, sub), rows(wdir, sub), durations(fdir)
    # dispatch ids differ between the two runs; pair them by order
    for i, (fd, wd) in enumerate(zip(sorted(f), sorted(w))):
        rd, wr = int(2 * f[fd][0] * 1024), int(w[wd][0] * 1024)
        print(json.dumps({"i": i, "kernel": f[fd][1][:80], "read_bytes": rd, "write_bytes": wr,
                          "hbm_bytes": rd + wr, "ms_fetch_pass": round(dur.get(fd, 0.0), 4)}))


if __name__ == "__main__":
    main()
