#!/usr/bin/env python3
"""Probe: coding rate vs the batch layout (chunk-stride and stripe-stride
padding) and the stripe-group tile order, for encode and the bench's recover
patterns.  One line per (geometry, layout, op): fraction of 8 TB/s by
algorithmic bytes ((k+rows)*cs per stripe).

  layout_probe.py [GEOM ...]   GEOM = n,k,cs_kib  (default 14,10,1024 20,16,4096)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

TOTAL = int(float(os.environ.get("PROBE_GIB", "48")) * (1 << 30))
ctx = nxec.Context(0)
st = ctx.stream
buf = nxec.DeviceBuffer(TOTAL)
buf.fill_random(5)


def rate(n, k, cs, cstride, sstride, op):
    ns = TOTAL // sstride
    if op == "encode":
        coef, src, dst = nxec.gen_rs_matrix(n, k)[k:], list(range(k)), list(range(k, n))
    else:
        ids, _, rm = nxec.rs_plan(n, k, op, True)
        coef, src, dst = rm, ids[:k], list(op)

    def go():
        ctx.stripes_mul(coef, buf.ptr, buf.ptr, src_idx=src, dst_idx=dst, src_chunk_stride=cstride,
                        src_stripe_stride=sstride, dst_chunk_stride=cstride, dst_stripe_stride=sstride, length=cs,
                        nstripes=ns, stream=st)
    go()
    e0, e1 = nxec.Event(), nxec.Event()
    e0.record(st)
    for _ in range(4):
        go()
    e1.record(st)
    ctx.sync()
    ms = e0.elapsed_ms(e1) / 4
    return ms, ns * (k + len(dst)) * cs / (ms * 1e-3) / 8e12


geoms = [tuple(int(x) for x in g.split(",")) for g in sys.argv[1:]] or [(14, 10, 1024), (20, 16, 4096)]
# PROBE_REPEAT=R walks the whole sweep R times (alternating A/B on one box)
for n, k, cs_kib in geoms * int(os.environ.get("PROBE_REPEAT", "1")):
    cs = cs_kib << 10
    p = n - k
    pats = ["encode", list(range(p)), list(range(k, n)), [1, 4, n - 3, n - 1][:p]]
    if os.environ.get("PROBE_PATS"):  # e.g. "enc;0;15"
        pats = ["encode" if x == "enc" else [int(c) for c in x.split(",")] for x in os.environ["PROBE_PATS"].split(";")]
    cpads = [int(x) for x in os.environ.get("PROBE_CPADS", "0,4096,65536").split(",")]
    spads = [float(x) for x in os.environ.get("PROBE_SPADS", "0,1").split(",")]  # in chunk strides
    sgs = os.environ.get("PROBE_SG", "1,8").split(",")
    for cpad in cpads:
        cstride = cs + cpad
        for spad_chunks in spads:
            # whole chunks of stripe padding exactly (an odd stripe stride in
            # units of the chunk stride); fractions rounded down to 4 KiB
            extra = int(spad_chunks) * cstride if spad_chunks == int(spad_chunks) else \
                int(spad_chunks * cstride) // 4096 * 4096
            sstride = n * cstride + extra
            for sg in (sgs if cs >= (2 << 20) or os.environ.get("PROBE_SG_ALL") else ["1"]):
                os.environ["NXEC_STRIPE_GROUP"] = sg
                res = [rate(n, k, cs, cstride, sstride, op) for op in pats]
                fr = [f for _, f in res]
                print(f"({n},{k}) cs {cs_kib:5d} KiB chunk_pad {cpad:6d} stripe_pad {spad_chunks:g} chunk sg {sg}: "
                      + " ".join(f"{('enc' if op == 'encode' else ','.join(map(str, op))):>12s} {f:.3f}"
                                 for op, f in zip(pats, fr))
                      + f"  mean {sum(fr) / len(fr):.3f} min {min(fr):.3f}", flush=True)
os.environ.pop("NXEC_STRIPE_GROUP", None)
buf.free()
ctx.close()
