#!/usr/bin/env python3
"""Probe for the per-L2-channel counter passes: runs ONE
coding op of one geometry and batch layout a few times, so that a
`rocprofv3 -E tools/tcc_instances.yaml --pmc NXEC_TCC_RD_I0 ...` pass sees
only those dispatches.  tools/tcc_summary.py turns the passes into the
per-instance request shares.

  tcc_channels.py N K CS_KIB CHUNK_PAD STRIPE_PAD_CHUNKS OP [REPS]
  OP = enc | comma-separated erased chunk ids (recover)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, cs_kib, cpad, spad = (int(x) for x in sys.argv[1:6])
op = sys.argv[6]
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 3
cs = cs_kib << 10
cst = cs + cpad
sst = n * cst + spad * cst
total = int(float(os.environ.get("PROBE_GIB", "8")) * (1 << 30))
ns = total // sst
ctx = nxec.Context(0)
buf = nxec.DeviceBuffer(ns * sst)
buf.fill_random(11)
ctx.rs_encode(n, k, buf.ptr, cst, sst, cs, ns, ctx.stream)
ctx.sync()
for _ in range(reps):
    if op == "enc":
        ctx.rs_encode(n, k, buf.ptr, cst, sst, cs, ns, ctx.stream)
    else:
        ctx.rs_recover(n, k, [int(c) for c in op.split(",")], buf.ptr, cst, sst, cs, ns, ctx.stream)
ctx.sync()
e = len(op.split(",")) if op != "enc" else n - k
print(f"({n},{k}) cs {cs_kib} KiB chunk stride {cst} stripe stride {sst} op {op}: {ns} stripes, "
      f"{reps + 1} launches, {ns * (k + e) * cs} algorithmic bytes per launch", flush=True)
buf.free()
ctx.close()
