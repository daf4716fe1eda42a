#!/usr/bin/env python3
"""Per-workgroup timing of k_files_md5 (NXEC_FILES_CLOCK=1 prints, per
workgroup, its slots' full-stripe / last-stripe request counts and the
s_memrealtime of its start, code-wave-0 end and hash-wave-0 end): which
workgroups set a batch's time.  Batches: `mix` (bench.py's files, in-place
tails) then `full10` (4096 whole stripes as files), one warm call each first."""
import os
import sys

import numpy as np

os.environ["NXEC_FILES_CLOCK"] = "1"  # read once by the library
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, M = 14, 10, 1 << 20
p = n - k
ctx = nxec.Context(0)
sets = {"mix": [int(x) for x in np.random.default_rng(1234).integers(1, 2 * k * M + 1, size=4096)],
        "full10": [k * M] * 4096}
for name, lengths in sets.items():
    offs = np.concatenate([[0], np.cumsum([(L + 15) // 16 * 16 for L in lengths])])
    arena = nxec.DeviceBuffer(int(offs[-1]))
    arena.fill_random(77)
    total, tail_bytes = nxec.objects_layout(n, k, lengths, M)
    par, tail, md5 = nxec.DeviceBuffer(total * p * M), nxec.DeviceBuffer(max(tail_bytes, 16)), nxec.DeviceBuffer(total * n * 16)
    ptrs = [arena.ptr + int(o) for o in offs[:-1]]
    for warm in (True, False):
        print(f"== {name} {'warm-up' if warm else 'timed'}", file=sys.stderr, flush=True)
        ctx.encode_objects(n, k, ptrs, lengths, M, par.ptr, tail.ptr, md5.ptr, flags=nxec.OBJECTS_TAIL_INPLACE)
        ctx.sync()
    for b in (arena, par, tail, md5):
        b.free()
