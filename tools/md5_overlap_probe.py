#!/usr/bin/env python3
"""Probe: the object write (RS(10,4) encode + MD5 of all 14 chunks of 4096
1 MiB stripes) scheduled three ways, wall time per write:

  serial   encode -> MD5(14 chunks)                     (nxec_encode_object today)
  fork     MD5(10 data chunks) on a 2nd stream || encode -> MD5(4 parity chunks)
  md5only  MD5(14 chunks) alone, and encode alone, for reference

Run with NXEC_MD5_CFG=D,G,NT to try smaller-footprint MD5 variants (so the
MD5 waves can share CUs with the encode's 1024-thread workgroups)."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402
from nexoedge_amd._lib import lib  # noqa: E402

n, k, cs, ns = 14, 10, 1 << 20, 4096
stripe = n * cs
ctx = nxec.Context(0)
sa = ctx.stream
sb_ = C.c_void_p()
nxec.check(lib.nxec_stream_create(C.byref(sb_)), "stream")
sb = sb_
buf = nxec.DeviceBuffer(ns * stripe)
buf.fill_random(11)
dig = nxec.DeviceBuffer(ns * n * 16)


def sync():
    ctx.sync()
    nxec.check(lib.nxec_stream_sync(sb), "sync")


def encode(st):
    ctx.rs_encode(n, k, buf.ptr, cs, stripe, cs, ns, st)


def md5(first, count, st):
    ctx.md5_chunks(buf.ptr + first * cs, cs, stripe, count, cs, ns, dig.ptr + first * 16, st)


def serial():
    encode(sa)
    md5(0, n, sa)


def fork():
    md5(0, k, sb)  # data chunks do not depend on the parity
    encode(sa)
    md5(k, n - k, sa)


def fork_encode_first():
    encode(sa)
    md5(0, k, sb)
    md5(k, n - k, sa)


def timed(fn, reps=4):
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
        sync()
    return (time.perf_counter() - t0) / reps * 1e3


cfg = os.environ.get("NXEC_MD5_CFG", "2,8,0")
for name, fn in [("encode only", lambda: encode(sa)), ("md5 14 chunks only", lambda: md5(0, n, sa)),
                 ("md5 10 data chunks only", lambda: md5(0, k, sa)), ("serial", serial), ("fork (md5 first)", fork),
                 ("fork (encode first)", fork_encode_first)]:
    print(f"md5 cfg {cfg:8s} {name:26s} {timed(fn):8.2f} ms", flush=True)
buf.free()
dig.free()
lib.nxec_stream_destroy(sb)
ctx.close()
