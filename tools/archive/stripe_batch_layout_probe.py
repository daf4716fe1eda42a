#!/usr/bin/env python3
"""Probe: the degraded read of StripeBatch::decodeFile (nxec_decode_object_ex,
full-output decode of every stripe into the object, chunk_manager.cc:738-800)
on the packed [s][n][M] layout it used to stage fetched chunks at and on the
recover-heavy layout it stages them at now (nxec_batch_layout), for the
bench's three erasure patterns.  4096 RS(10,4) 1 MiB stripes, HIP events on
the launch stream; bytes = 2k*cs per stripe (k survivors in, k data chunks out).
Usage: stripe_batch_layout_probe.py [pattern index ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, M, ns = 14, 10, 1 << 20, 4096
PATS = ([0, 1, 2, 3], [10, 11, 12, 13], [1, 4, 11, 13])
ctx = nxec.Context(0)
st = ctx.stream
L = ns * k * M
out = nxec.DeviceBuffer(L)
which = [int(a) for a in sys.argv[1:]] or [0, 1, 2]
for name, flags in (("packed", None), ("recover_heavy", nxec.LAYOUT_RECOVER_HEAVY)):
    cst, sst = (M, n * M) if flags is None else nxec.batch_layout(n, M, flags)
    buf = nxec.DeviceBuffer(ns * sst)
    buf.fill_random(11)
    ctx.rs_encode(n, k, buf.ptr, cst, sst, M, ns, st)
    for pi in which:
        pat = PATS[pi]
        ctx.decode_object_ex(n, k, pat, buf.ptr, cst, sst, L, M, out.ptr, None, st)  # warm
        e0, e1 = nxec.Event(), nxec.Event()
        reps = 5
        e0.record(st)
        for _ in range(reps):
            ctx.decode_object_ex(n, k, pat, buf.ptr, cst, sst, L, M, out.ptr, None, st)
        e1.record(st)
        ctx.sync()
        ms = e0.elapsed_ms(e1) / reps
        b = ns * 2 * k * M
        print(f"{name:14s} stride {sst >> 20} MiB lost {pat}: {ms:.3f} ms, {b / ms / 1e6:.0f} GB/s, "
              f"{b / ms / 1e6 / 8000:.4f} of 8 TB/s", flush=True)
    buf.free()
