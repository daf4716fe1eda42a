#!/usr/bin/env python3
"""Summarise per-L2-channel request counters (tools/tcc_instances.yaml passes
over tools/tcc_channels.py) into one JSON line per (label, direction).

  tcc_summary.py LABEL DIR [DIR ...]
  tcc_summary.py --lat LABEL ROOT     (the `lat5` passes: one directory per pass under ROOT)

Each DIR is one rocprofv3 output directory; the counters of all DIRs are
merged per dispatch order (the passes run the same program).  For every
coding dispatch (k_mul_* kernels) it reports the 16 instance counts summed
over the XCDs, their share of the total, max/mean and the coefficient of
variation -- an even spread (max/mean ~1) says the requests are balanced over
the L2 channels; a skew names the channels the layout piles onto."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    if sys.argv[1] == "--lat":
        return lat_main(sys.argv[2], sys.argv[3])
    label, dirs = sys.argv[1], sys.argv[2:]
    per = {}  # (dispatch order, counter) -> value
    for d in dirs:
        paths = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        if not paths:
            continue
        rows = [r for r in csv.DictReader(open(paths[0])) if "k_mul" in r["Kernel_Name"]]
        order = {did: i for i, did in enumerate(sorted({int(r["Dispatch_Id"]) for r in rows}))}
        for r in rows:
            per[(order[int(r["Dispatch_Id"])], r["Counter_Name"])] = float(r["Counter_Value"])
    for tag in ("RD", "WR"):
        for i in sorted({i for i, _ in per}):
            v = [per.get((i, f"NXEC_TCC_{tag}_I{c}")) for c in range(16)]
            if any(x is None for x in v) or sum(v) == 0:
                continue
            mean = sum(v) / 16
            print(json.dumps({"label": label, "dir": tag, "dispatch": i, "total_req": int(sum(v)),
                              "share": [round(x / sum(v), 4) for x in v],
                              "max_over_mean": round(max(v) / mean, 4), "min_over_mean": round(min(v) / mean, 4),
                              "cv": round(statistics.pstdev(v) / mean, 4)}))


# --lat: per-dispatch L2 -> fabric request latency and credit stalls: the mean
# cycles a read / write request spends in flight (TCC_EA0_{RD,WR}REQ_LEVEL_sum
# / *_sum, per the counters' own description) and the DRAM-credit stalls.
def lat_main(label, root):
    per = {}
    dur = {}
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        paths = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        if not paths:
            continue
        rows = [r for r in csv.DictReader(open(paths[0])) if "k_mul" in r["Kernel_Name"]]
        order = {did: i for i, did in enumerate(sorted({int(r["Dispatch_Id"]) for r in rows}))}
        for r in rows:
            per[(order[int(r["Dispatch_Id"])], r["Counter_Name"])] = float(r["Counter_Value"])
        kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
        if kt:
            ks = [r for r in csv.DictReader(open(kt[0])) if "k_mul" in r["Kernel_Name"]]
            for i, r in enumerate(sorted(ks, key=lambda r: int(r["Dispatch_Id"]))):
                dur.setdefault(i, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for i in sorted({i for i, _ in per}):
        g = lambda c: per.get((i, c))  # noqa: E731
        out = {"label": label, "dispatch": i}
        if g("TCC_EA0_RDREQ_sum"):
            out["rd_req"] = int(g("TCC_EA0_RDREQ_sum"))
            out["rd_cycles_in_flight"] = round(g("TCC_EA0_RDREQ_LEVEL_sum") / g("TCC_EA0_RDREQ_sum"), 1)
            out["rd_dram_credit_stall"] = int(g("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"))
        if g("TCC_EA0_WRREQ_sum"):
            out["wr_req"] = int(g("TCC_EA0_WRREQ_sum"))
            out["wr_cycles_in_flight"] = round(g("TCC_EA0_WRREQ_LEVEL_sum") / g("TCC_EA0_WRREQ_sum"), 1)
            out["wr_dram_credit_stall"] = int(g("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"))
            out["too_many_wrreq_stall"] = int(g("TCC_TOO_MANY_EA_WRREQS_STALL_sum"))
        if g("TCC_BUSY_avr") is not None:
            out["tcc_busy_avr"] = int(g("TCC_BUSY_avr"))
            out["tag_stall"] = int(g("TCC_TAG_STALL_sum"))
        if i in dur:
            out["ms_per_pass"] = [round(x, 4) for x in dur[i]]
        print(json.dumps(out))



if __name__ == "__main__":
    main()
