"""Print the kernel + memory-copy timeline of the last N events of a
rocprofv3 --kernel-trace --memory-copy-trace --output-format csv run.
usage: python tools/copy_timeline.py <dir with run_*_trace.csv> [N]"""
import csv
import os
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
ev = []
for r in csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"].replace("MEMORY_COPY_", ""),
               r["Stream_Id"]))
kt = os.path.join(d, "run_kernel_trace.csv")
if os.path.exists(kt):
    for r in csv.DictReader(open(kt)):
        name = r["Kernel_Name"].replace("void nxec::(anonymous namespace)::", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name[:40], r["Stream_Id"]))
ev.sort()
t0 = ev[-last][0]
print(f"{'start ms':>9} {'end ms':>9} {'dur ms':>8}  stream  op")
for s, e, name, st in ev[-last:]:
    print(f"{(s - t0) / 1e6:9.2f} {(e - t0) / 1e6:9.2f} {(e - s) / 1e6:8.2f}  st{st:<5} {name}")
