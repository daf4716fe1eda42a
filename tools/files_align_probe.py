#!/usr/bin/env python3
"""Probe: where the multi-file write's fold costs.  The
bench's files workload (4096 files, sizes uniform in [1 B, 2*k*M]) against
two variants of the same sizes: `a16` rounds each last stripe up to chunks
that are multiples of 16 bytes and fill the stripe (every in-place read is
16-byte aligned, no chunk is masked), `a16m` is that minus 8 bytes (aligned
reads, one masked chunk per last stripe).  Prints k_files_md5's time per
launch (library HIP events) and its rate over (k + p) x chunk length per
request.  Run once per library: the product build and, with
NXEC_LIB=build/ab/probes/libnxec.so NXEC_FILES_FOLD=0, round 4's pad copy."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, M = 14, 10, 1 << 20
p = n - k
reps = int(os.environ.get("PROBE_REPS", "10"))
ctx = nxec.Context(0)
raw = [int(x) for x in np.random.default_rng(1234).integers(1, 2 * k * M + 1, size=4096)]


def aligned(L, minus, a=16):
    ns, nf, cl = nxec.object_layout(n, k, L, M)
    if ns == nf:
        return L
    c = min((cl + a - 1) // a * a, M)
    if a < 16 and c % 16 == 0 and c + a <= M:
        c += a  # a-byte aligned, not 16
    return nf * k * M + k * c - minus


variants = {"raw": raw, "a16": [aligned(L, 0) for L in raw], "a16m": [aligned(L, 8) for L in raw],
            "a4m": [aligned(L, 8, 4) for L in raw], "a8m": [aligned(L, 8, 8) for L in raw]}
for name, lengths in variants.items():
    offs = np.concatenate([[0], np.cumsum([(L + 15) // 16 * 16 for L in lengths])])
    arena = nxec.DeviceBuffer(int(offs[-1]))
    arena.fill_random(77)
    total, tail_bytes = nxec.objects_layout(n, k, lengths, M)
    par = nxec.DeviceBuffer(total * p * M)
    tail = nxec.DeviceBuffer(max(tail_bytes, 16))
    md5 = nxec.DeviceBuffer(total * n * 16)
    ptrs = [arena.ptr + int(o) for o in offs[:-1]]
    layouts = [nxec.object_layout(n, k, L, M) for L in lengths]
    kernel_bytes = sum((nf * M + (ns - nf) * cl) * n for ns, nf, cl in layouts)
    masked = sum(1 for (ns, nf, cl), L in zip(layouts, lengths) if ns > nf and (L - nf * k * M) % cl)
    unaligned = sum(1 for ns, nf, cl in layouts if ns > nf and cl % 16)

    def op():
        ctx.encode_objects(n, k, ptrs, lengths, M, par.ptr, tail.ptr, md5.ptr, None,
                           flags=nxec.OBJECTS_TAIL_INPLACE | nxec.OBJECTS_ASYNC)

    op()
    ctx.sync()
    ctx.kernel_timing(True)
    for _ in range(reps):
        op()
    ctx.sync()
    ms, launches = ctx.kernel_time()
    ctx.kernel_timing(False)

    print(f"{name:5s} kernel {ms / reps:.3f} ms/call ({launches // reps} launches/call) "
          f"{kernel_bytes / (ms / reps) / 1e6:.1f} GB/s over {kernel_bytes / 2**30:.2f} GiB; "
          f"last stripes unaligned {unaligned}, masked {masked}", flush=True)
    del arena, par, tail, md5
