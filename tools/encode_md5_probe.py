#!/usr/bin/env python3
"""Probe: the object write (RS encode + MD5 of every chunk) through
nxec_encode_object, fused kernel vs the two kernels (NXEC_FUSED_MD5=0),
device-resident, wall time per write.

  python3 tools/encode_md5_probe.py [n k chunk_bytes nstripes]
Environment knobs passed through: NXEC_EM_PRIO (hash waves' s_setprio)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

args = [int(a) for a in sys.argv[1:]]
n, k, cs, ns = args if len(args) == 4 else (14, 10, 1 << 20, 4096)
p = n - k
ctx = nxec.Context(0)
obj = nxec.DeviceBuffer(ns * k * cs)
obj.fill_random(11)
par = nxec.DeviceBuffer(ns * p * cs)
dig = nxec.DeviceBuffer(ns * n * 16)


def write():
    ctx.encode_object(n, k, obj.ptr, ns * k * cs, cs, par.ptr, None, dig.ptr)


def timed(reps=6):
    write()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        write()
    ctx.sync()
    return (time.perf_counter() - t0) / reps * 1e3


alg = ns * n * cs  # every chunk hashed once; the encode moves the same bytes
for mode in ("1", "0", "1", "0"):
    os.environ["NXEC_FUSED_MD5"] = mode
    ms = timed()
    print(f"RS({n},{k}) {cs >> 10} KiB x {ns}: {'fused' if mode == '1' else 'two kernels'} "
          f"prio={os.environ.get('NXEC_EM_PRIO', '1')} {ms:8.3f} ms  {alg / ms / 1e6:8.1f} GB/s "
          f"({alg / ms / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)
for b in (obj, par, dig):
    b.free()
ctx.close()
