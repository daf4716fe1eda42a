"""nxec_encode_object_host timeline probe: RS(10,4), 1 MiB chunks, pinned
object / parity / digests, a few calls.  Run under
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d <dir> -- python3 tools/object_host_probe.py
to see whether H2D, the encode, MD5 and D2H of consecutive batches overlap."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, cs = 14, 10, 1 << 20
ns = int(os.environ.get("PROBE_STRIPES", "512"))
batch = int(os.environ.get("PROBE_BATCH", "0"))
p = n - k
ctx = nxec.Context(0)
hd = nxec.PinnedBuffer(ns * k * cs)
hp = nxec.PinnedBuffer(ns * p * cs)
hm = nxec.PinnedBuffer(ns * n * 16)
hd.array[:] = np.random.default_rng(1).integers(0, 256, size=hd.nbytes, dtype=np.uint8)
length = ns * k * cs
if os.environ.get("PROBE_PRE"):  # the bench's order: zero-copy and staged batch encodes first
    ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
    if os.environ["PROBE_PRE"] == "2":
        os.environ["NXEC_HOST_DIRECT"] = "0"
        ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
        del os.environ["NXEC_HOST_DIRECT"]
ctx.encode_object_host(n, k, hd.ptr, length, cs, hp.ptr, hm.ptr, batch)
for _ in range(3):
    t0 = time.perf_counter()
    ctx.encode_object_host(n, k, hd.ptr, length, cs, hp.ptr, hm.ptr, batch)
    dt = time.perf_counter() - t0
    print(f"encode_object_host {length / dt / (1 << 30):.2f} GiB/s user data ({dt * 1e3:.1f} ms)", flush=True)
