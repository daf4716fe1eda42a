#!/usr/bin/env python3
"""Summarise separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
bench.py into profiles/rNN_pmc_traffic.json (HBM bytes per launch of the
headline kernel), applying the gfx950 FETCH_SIZE x2 correction of
MI355X_MICROARCH.md.  Usage: pmc_summary.py OUT_DIR ALGORITHMIC_BYTES [KERNEL_SUBSTRING] > json"""
import csv
import json
import sys


def per_launch_kb(path, kernel_sub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel_sub in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main():
    out, alg = sys.argv[1], int(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else "k_mul_vec<10, 8, false, false, true>"
    f, nf = per_launch_kb(f"{out}/pmc_FETCH_SIZE/run_counter_collection.csv", sub)
    w, nw = per_launch_kb(f"{out}/pmc_WRITE_SIZE/run_counter_collection.csv", sub)
    rd, wr = int(2 * f * 1024), int(w * 1024)
    print(json.dumps({
        "kernel": f"{sub} (RS(10,4) encode/recover, 4096 stripes x 1 MiB)",
        "source": "rocprofv3 --pmc FETCH_SIZE --kernel-trace and --pmc WRITE_SIZE --kernel-trace, separate passes, "
                  "python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-host-inclusive (tools/gpu_check.sh PMC=1)",
        "launches": [nf, nw],
        "fetch_size_kb_per_launch": round(f, 2), "write_size_kb_per_launch": round(w, 2),
        "gfx950_correction": "FETCH_SIZE reports half the bytes of a wide coalesced streaming read "
                             "(MI355X_MICROARCH.md, HBM): read_bytes = 2 * FETCH_SIZE * 1024; "
                             "write_bytes = WRITE_SIZE * 1024",
        "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round((rd + wr) / alg, 5)}, indent=2))


if __name__ == "__main__":
    main()
