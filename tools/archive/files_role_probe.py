#!/usr/bin/env python3
"""Role probes of the one-launch multi-file write (k_files_md5<10>, as
k_mul_md5's NXEC_EM_PROBE): NXEC_FM_PROBE bit 0 = no MD5 rounds, bit 1 = no
table lookups, bit 2 = no global loads/stores (outputs invalid).  For each
probe 0..7 the batches `full10` (4096 full RS(10,4) stripes as files) and
`mix` (bench.py's 4096 files of 1 B - 20 MiB, in-place tails) run 3 times;
run under rocprofv3 --kernel-trace for kernel-only durations (the launches
come in this order: probe-major, then set, then repetition)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

if not nxec.design_probes():
    sys.exit("libnxec was built without the design-probe kernels: make clean && make PROBES=1")
n, k, M = 14, 10, 1 << 20
p = n - k
ctx = nxec.Context(0)
sets = {"full10": [k * M] * 4096,
        "mix": [int(x) for x in np.random.default_rng(1234).integers(1, 2 * k * M + 1, size=4096)]}
bufs = {}
for name, lengths in sets.items():
    offs = np.concatenate([[0], np.cumsum([(L + 15) // 16 * 16 for L in lengths])])
    arena = nxec.DeviceBuffer(int(offs[-1]))
    arena.fill_random(77)
    total, tail_bytes = nxec.objects_layout(n, k, lengths, M)
    bufs[name] = (lengths, [arena.ptr + int(o) for o in offs[:-1]], nxec.DeviceBuffer(total * p * M),
                  nxec.DeviceBuffer(max(tail_bytes, 16)), nxec.DeviceBuffer(total * n * 16), arena)
for probe in range(8):
    os.environ["NXEC_FM_PROBE"] = str(probe)
    for name in sets:
        lengths, ptrs, par, tail, md5, _ = bufs[name]
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.encode_objects(n, k, ptrs, lengths, M, par.ptr, tail.ptr, md5.ptr, flags=nxec.OBJECTS_TAIL_INPLACE)
            ctx.sync()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(f"probe {probe} {name:6s} wall ms {' '.join(f'{t:.3f}' for t in ts)}", flush=True)
