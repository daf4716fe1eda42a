#!/usr/bin/env python3
"""Probe: does the position of the 4 written chunks (and of the 10 read ones)
inside a stripe change the RS(10,4)-shaped multiply rate?  Stripes of 20 x 1 MiB
chunks (2867 stripes, ~56 GiB); 10 sources and 4 destinations chosen per row."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, cs = 20, 1 << 20
ns = (56 << 30) // (n * cs)
ctx = nxec.Context(0)
st = ctx.stream
buf = nxec.DeviceBuffer(ns * n * cs)
buf.fill_random(3)
coef = nxec.gen_rs_matrix(14, 10)[10:]
cases = [
    ("src 0-9 dst 10-13", list(range(10)), [10, 11, 12, 13]),
    ("src 0-9 dst 11-14", list(range(10)), [11, 12, 13, 14]),
    ("src 0-9 dst 10,12,14,16", list(range(10)), [10, 12, 14, 16]),
    ("src 0-9 dst 10,13,16,19", list(range(10)), [10, 13, 16, 19]),
    ("src 0-9 dst 16-19", list(range(10)), [16, 17, 18, 19]),
    ("src even 0-18 dst 1,3,5,7", list(range(0, 20, 2)), [1, 3, 5, 7]),
    ("src even 0-18 dst 1,9,11,13", list(range(0, 20, 2)), [1, 9, 11, 13]),
    ("src 0,2,3,5-10,12 dst 1,4,11,13", [0, 2, 3, 5, 6, 7, 8, 9, 10, 12], [1, 4, 11, 13]),
    ("src 4-13 dst 0-3", list(range(4, 14)), [0, 1, 2, 3]),
]
for name, src, dst in cases:
    def go():
        ctx.stripes_mul(coef, buf.ptr, buf.ptr, src_idx=src, dst_idx=dst, src_chunk_stride=cs,
                        src_stripe_stride=n * cs, dst_chunk_stride=cs, dst_stripe_stride=n * cs, length=cs,
                        nstripes=ns, stream=st)
    go()
    e0, e1 = nxec.Event(), nxec.Event()
    e0.record(st)
    for _ in range(5):
        go()
    e1.record(st)
    ctx.sync()
    ms = e0.elapsed_ms(e1) / 5
    b = ns * 14 * cs
    print(f"{name:34s} {ms:7.3f} ms  frac8T {b / (ms * 1e-3) / 8e12:.3f}", flush=True)
buf.free()
ctx.close()
