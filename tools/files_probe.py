#!/usr/bin/env python3
"""Probe: the one-launch multi-file write (k_files_md5) against the
single-object fused write (k_mul_md5) on the SAME bytes -- one object of
`ns` full RS(n,k) stripes through nxec_encode_objects and nxec_encode_object
-- and the multi-file batch with requests sorted longest first vs as given."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, M, ns = 14, 10, 1 << 20, 4096
p = n - k
ctx = nxec.Context(0)
L = ns * k * M
obj = nxec.DeviceBuffer(L)
obj.fill_random(3)
par = nxec.DeviceBuffer(ns * p * M)
tail = nxec.DeviceBuffer(16)
dig = nxec.DeviceBuffer(ns * n * 16)


def timed(fn, reps=5):
    fn()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    return (time.perf_counter() - t0) / reps * 1e3


a = timed(lambda: ctx.encode_object(n, k, obj.ptr, L, M, par.ptr, None, dig.ptr))
b = timed(lambda: ctx.encode_objects(n, k, [obj.ptr], [L], M, par.ptr, tail.ptr, dig.ptr))
print(f"one object of {ns} RS({n},{k}) 1 MiB stripes: encode_object (k_mul_md5) {a:.3f} ms, "
      f"encode_objects (k_files_md5) {b:.3f} ms", flush=True)
