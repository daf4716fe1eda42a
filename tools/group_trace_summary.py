"""Summarise a rocprofv3 --kernel-trace of `bench.py --gpus 8 --group` on one
GPU (per-process CSVs, `-o run_%pid%`): for the ranks' timed k_mul_vec
launches and the group's, the wall span, the union of kernel intervals (is
the GPU ever idle?), the effective time per launch and how many launches run
at once.  Usage: python tools/group_trace_summary.py gpurun_out/gtrace"""
import csv
import glob
import json
import sys


def load(d):
    out = {}
    for f in sorted(glob.glob(f"{d}/*kernel_trace.csv")):
        rows = [r for r in csv.DictReader(open(f)) if "k_mul_vec" in r["Kernel_Name"]]
        out[f] = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows)
    return out


def summary(ks):
    ks = sorted(ks)
    span = max(e for _, e, _ in ks) - ks[0][0]
    busy, cs, ce = 0, None, None
    for s, e, _ in ks:
        if ce is None or s > ce:
            busy += 0 if ce is None else ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    ev = sorted([(s, 1) for s, _, _ in ks] + [(e, -1) for _, e, _ in ks])
    hist, cur, last = {}, 0, ev[0][0]
    for t, d in ev:
        hist[cur] = hist.get(cur, 0) + t - last
        cur, last = cur + d, t
    tot = sum(hist.values())
    return {"launches": len(ks), "span_ms": round(span / 1e6, 3), "busy_ms": round(busy / 1e6, 3),
            "ms_per_launch_effective": round(busy / 1e6 / len(ks), 4),
            "mean_launch_ms": round(sum(e - s for s, e, _ in ks) / len(ks) / 1e6, 4),
            "queues": len({q for _, _, q in ks}),
            "time_share_by_launches_running": {k: round(v / tot, 3) for k, v in sorted(hist.items()) if v}}


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gtrace"
    per = load(d)
    group_file = max(per, key=lambda f: len(per[f]))
    gk = per[group_file]  # rank 0: its own 28 launches, then the group's
    # each rank: 2 warm-up steps x 2 ops, then the 10 timed steps x 2 ops
    ranks = [k for f, ks in per.items() for k in (gk[:28] if f == group_file else ks)[4:24]]
    # the group: the initial encode (8) and 2 warm-up steps (32), then 160 timed
    group = gk[28 + 8 + 32:28 + 8 + 32 + 160]
    print(json.dumps({"ranks_timed": summary(ranks), "group_timed": summary(group)}, indent=1))


if __name__ == "__main__":
    main()
