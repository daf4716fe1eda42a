#!/usr/bin/env python3
"""The write path's fused kernel alone (nxec_encode_object: encode + MD5 of
every chunk of 4096 RS(10,4) 1 MiB stripes), REPS launches, for rocprofv3
passes of k_mul_md5 with a barrier per step (NXEC_EM_RING=0, the probe
build) and the ring hand-off (NXEC_EM_RING=1).  Prints the mean wall time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, cs, ns = 14, 10, 1 << 20, 4096
reps = int(os.environ.get("REPS", "6"))
ctx = nxec.Context(0)
obj = nxec.DeviceBuffer(ns * k * cs)
obj.fill_random(11)
par = nxec.DeviceBuffer(ns * (n - k) * cs)
dig = nxec.DeviceBuffer(ns * n * 16)
ctx.encode_object(n, k, obj.ptr, ns * k * cs, cs, par.ptr, None, dig.ptr)
ctx.sync()
t0 = time.perf_counter()
for _ in range(reps):
    ctx.encode_object(n, k, obj.ptr, ns * k * cs, cs, par.ptr, None, dig.ptr)
ctx.sync()
print(f"em_ring={os.environ.get('NXEC_EM_RING', 'default')} {1e3 * (time.perf_counter() - t0) / reps:.3f} ms per write",
      flush=True)
for b in (obj, par, dig):
    b.free()
ctx.close()
