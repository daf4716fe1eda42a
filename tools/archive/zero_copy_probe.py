#!/usr/bin/env python3
"""Probe: host-resident RS(10,4) encode, DMA staging (nxec_rs_encode_host_batch:
pinned H2D -> kernel -> D2H) vs zero-copy (the kernel reads the pinned data and
writes the pinned parity directly over PCIe)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nexoedge_amd import nxec  # noqa: E402

n, k, cs, ns = 14, 10, 1 << 20, 512
p = n - k
ctx = nxec.Context(0)
hd = nxec.PinnedBuffer(ns * k * cs)
hp = nxec.PinnedBuffer(ns * p * cs)
hd.array[:] = np.random.default_rng(1).integers(0, 256, size=hd.nbytes, dtype=np.uint8)
enc = nxec.gen_rs_matrix(n, k)[k:]
b = ns * n * cs


def timed(fn, reps=3):
    fn()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    return (time.perf_counter() - t0) / reps


os.environ["NXEC_HOST_DIRECT"] = "0"
t = timed(lambda: ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64))
ref = hp.array.copy()
print(f"rs_encode_host_batch, DMA staging (NXEC_HOST_DIRECT=0), 64-stripe batches: {b / t / 2**30:7.2f} GiB/s", flush=True)
del os.environ["NXEC_HOST_DIRECT"]
hp.array[:] = 0
t = timed(lambda: ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64))
print(f"rs_encode_host_batch, default (zero copy for pinned):            {b / t / 2**30:7.2f} GiB/s  "
      f"match={np.array_equal(hp.array, ref)}", flush=True)
hp.array[:] = 0
for batch in (ns, 64):
    def zc():
        for s0 in range(0, ns, batch):
            m = min(batch, ns - s0)
            ctx.stripes_mul(enc, hd.ptr + s0 * k * cs, hp.ptr + s0 * p * cs, src_chunk_stride=cs,
                            src_stripe_stride=k * cs, dst_chunk_stride=cs, dst_stripe_stride=p * cs, length=cs,
                            nstripes=m)
    t = timed(zc)
    ok = np.array_equal(hp.array, ref)
    print(f"zero-copy kernel on pinned memory, {batch}-stripe launches:  {b / t / 2**30:7.2f} GiB/s  match={ok}",
          flush=True)
hd.free()
hp.free()
ctx.close()
