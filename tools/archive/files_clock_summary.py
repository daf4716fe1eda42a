#!/usr/bin/env python3
"""Summarise tools/files_clock_probe.py's per-workgroup log: per batch, the
workgroups with only whole-stripe requests against those with last stripes
(duration, steps, us per step)."""
import re
import statistics as st
import sys

txt = open(sys.argv[1]).read()
sec = re.split(r"== (\S+) (warm-up|timed)\n", txt)
for i in range(1, len(sec), 3):
    name, kind, body = sec[i], sec[i + 1], sec[i + 2]
    if kind != "timed":
        continue
    rows = []
    for l in body.strip().split("\n"):
        m = re.match(r"wg (\d+) steps (\d+) full (\d+) tail (\d+) start ([\d.]+) code_end ([\d.]+) hash_end ([\d.]+)", l)
        if m:
            rows.append(tuple(float(x) for x in m.groups()))
    print(f"{name}: {len(rows)} workgroups, kernel span {max(max(r[5], r[6]) for r in rows):.1f} us")
    for label, sel in (("whole stripes only", lambda r: r[3] == 0), ("with last stripes", lambda r: r[3] > 0)):
        rr = [r for r in rows if sel(r)]
        if rr:
            dur = [max(r[5], r[6]) - r[4] for r in rr]
            print(f"  {label}: {len(rr)} wgs, duration mean {st.mean(dur):.1f} max {max(dur):.1f} us, "
                  f"steps mean {st.mean(r[1] for r in rr):.0f}, us/step {st.mean(d / r[1] for d, r in zip(dur, rr)):.3f}")
