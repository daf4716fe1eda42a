#!/usr/bin/env python3
"""Probe: RS(10,4)-shaped multiply rate vs the stripe stride (in MiB) of a
[stripe][chunk][byte] batch with 1 MiB chunks.  If the scattered-erasure
slowdown comes from address bit 20 being fixed per chunk position (even
stripe strides), odd strides should remove it."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

cs = 1 << 20
total = 54 << 30
ctx = nxec.Context(0)
st = ctx.stream
buf = nxec.DeviceBuffer(total)
buf.fill_random(5)
coef = nxec.gen_rs_matrix(14, 10)[10:]
pat = {"contig src0-9 dst10-13": (list(range(10)), [10, 11, 12, 13]),
       "mixed src..dst1,4,11,13": ([0, 2, 3, 5, 6, 7, 8, 9, 10, 12], [1, 4, 11, 13]),
       "even src dst odd": ([0, 2, 4, 6, 8, 10, 12, 14, 16, 18], [1, 3, 5, 7])}
for stride_mib in (14, 15, 20, 21, 16, 17):
    for name, (src, dst) in pat.items():
        if max(src + dst) >= stride_mib:
            continue
        ss = stride_mib * cs
        ns = total // ss

        def go():
            ctx.stripes_mul(coef, buf.ptr, buf.ptr, src_idx=src, dst_idx=dst, src_chunk_stride=cs,
                            src_stripe_stride=ss, dst_chunk_stride=cs, dst_stripe_stride=ss, length=cs,
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
        print(f"stride {stride_mib:2d} MiB {name:26s} {ns:5d} stripes {ms:7.3f} ms  frac8T {b / (ms * 1e-3) / 8e12:.3f}",
              flush=True)
buf.free()
ctx.close()
