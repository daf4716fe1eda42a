#!/usr/bin/env python3
"""Per-erasure-pattern timing of the RS(10,4) recover launch (4096 x 1 MiB),
event-timed on the context stream; encode for reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, cs, ns = 14, 10, 1 << 20, 4096
ctx = nxec.Context(0)
st = ctx.stream
buf = nxec.DeviceBuffer(ns * n * cs)
buf.fill_random(5)
ctx.rs_encode(n, k, buf.ptr, cs, n * cs, cs, ns, st)
ctx.sync()
pats = {"encode": None, "data0-3": [0, 1, 2, 3], "parity10-13": [10, 11, 12, 13], "mixed1,4,11,13": [1, 4, 11, 13],
        "data6-9": [6, 7, 8, 9], "one0": [0], "two0,13": [0, 13],
        "0,2,4,6": [0, 2, 4, 6], "1,2,3,4": [1, 2, 3, 4], "0,1,12,13": [0, 1, 12, 13], "4,5,6,7": [4, 5, 6, 7],
        "1,4,11,13 again": [1, 4, 11, 13], "0,5,10,13": [0, 5, 10, 13], "2,3,11,12": [2, 3, 11, 12]}
for name, f in pats.items():
    def go():
        if f is None:
            ctx.rs_encode(n, k, buf.ptr, cs, n * cs, cs, ns, st)
        else:
            ctx.rs_recover(n, k, f, buf.ptr, cs, n * cs, cs, ns, st)
    go()
    e0, e1 = nxec.Event(), nxec.Event()
    e0.record(st)
    for _ in range(5):
        go()
    e1.record(st)
    ctx.sync()
    ms = e0.elapsed_ms(e1) / 5
    e = k + (n - k if f is None else len(f))
    b = ns * e * cs
    print(f"{name:16s} {ms:7.3f} ms  {b / ms / 1e6:8.1f} GB/s  frac8T {b / ms / 1e6 / 8e3:.3f}", flush=True)
buf.free()
ctx.close()
