#!/usr/bin/env python3
"""Probe: one nxec_agent_encode_batch call of 64 ENC_CHUNK_REQ-shaped
requests (4 pageable 1 MiB inputs -> 1 output + MD5), timed per call; run
under rocprofv3 --kernel-trace --memory-copy-trace to see where a call's
~30 ms go (tools/copy_timeline.py)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

cs, nreq, g = 1 << 20, 64, 4
ctx = nxec.Context(0)
rng = np.random.default_rng(1)
m = rng.integers(1, 256, size=(1, g), dtype=np.uint8)
reqs = []
for _ in range(nreq):
    ins = [rng.integers(0, 256, size=cs, dtype=np.uint8) for _ in range(g)]
    reqs.append((m, ins, [np.zeros(cs, dtype=np.uint8)], np.zeros((1, 16), dtype=np.uint8)))
for it in range(4):
    t0 = time.perf_counter()
    ctx.agent_encode_batch(reqs, cs)
    print(f"call {it}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
ctx.close()
