#!/usr/bin/env python3
"""Probe: is the scattered-erasure slowdown tied to the addresses
the writes share with the reads?  Same RS(10,4)-shaped multiply as
tools/dst_spacing.py (20 x 1 MiB chunk stripes), with the written chunks
shifted by a sub-chunk byte offset, or written to a separate buffer."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, cs = 20, 1 << 20
ns = (52 << 30) // (n * cs)
ctx = nxec.Context(0)
st = ctx.stream
slack = 1 << 20
buf = nxec.DeviceBuffer(ns * n * cs + slack)
buf.fill_random(3)
side = nxec.DeviceBuffer(ns * 4 * cs + slack)
coef = nxec.gen_rs_matrix(14, 10)[10:]
even = list(range(0, 20, 2))
cases = []
for d in (0, 256, 2048, 4096, 16384, 65536, 262144, 524288):
    cases.append((f"src even dst 1,3,5,7 +{d}", even, [1, 3, 5, 7], d, False))
for d in (0, 4096, 524288):
    cases.append((f"src 0-9 dst 10-13 +{d}", list(range(10)), [10, 11, 12, 13], d, False))
for d in (0, 4096):
    cases.append((f"src even dst side buffer +{d}", even, [0, 1, 2, 3], d, True))
    cases.append((f"src 0-9 dst side buffer +{d}", list(range(10)), [0, 1, 2, 3], d, True))
for name, src, dst, off, sep in cases:
    dptr = (side.ptr if sep else buf.ptr) + off
    dss = 4 * cs if sep else n * cs

    def go():
        ctx.stripes_mul(coef, buf.ptr, dptr, src_idx=src, dst_idx=dst, src_chunk_stride=cs,
                        src_stripe_stride=n * cs, dst_chunk_stride=cs, dst_stripe_stride=dss, length=cs,
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
side.free()
ctx.close()
