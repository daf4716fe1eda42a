"""Same-box A/B of the pageable-frames read pipeline:
bench.py's read_from_frames (nxec_decode_frames pipelined, the sequential
calls, the gather and scatter legs alone, each with its process CPU seconds
and cgroup throttling) under the library / knobs the environment names.
usage: [NXEC_LIB=...] [NXEC_HOST_LANES=1] [NXEC_HOST_THREADS=N] [FRAMES_BIND=1] python tools/read_frames_ab.py LABEL"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from nexoedge_amd import nxec  # noqa: E402

bench.nxec = nxec
node = -1
if os.environ.get("FRAMES_BIND") == "1":  # this thread and the pools it starts on the GPU's NUMA node
    node = nxec.bind_thread_numa(0)
ctx = nxec.Context(0)
rf = bench.read_from_frames(ctx, 14, 10, 1 << 20, 256)
# the link alone: pinned host <-> HBM DMA, each direction by itself and both
# at once on two streams (no host copies): if the pipeline's both-directions
# rate is the link's duplex rate, the link -- not the host -- bounds it
if os.environ.get("FRAMES_DMA") == "1":
    import ctypes as C
    import time
    L = nxec._lib.lib
    nb = 2560 << 20
    hin, hout = nxec.PinnedBuffer(nb), nxec.PinnedBuffer(nb)
    din, dout = nxec.DeviceBuffer(nb), nxec.DeviceBuffer(nb)
    s1, s2 = C.c_void_p(), C.c_void_p()
    L.nxec_stream_create(C.byref(s1))
    L.nxec_stream_create(C.byref(s2))

    def dma(h2d, d2h, reps=3):
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                L.nxec_memcpy_h2d(C.c_void_p(din.ptr), C.c_void_p(hin.ptr), nb, s1)
            if d2h:
                L.nxec_memcpy_d2h(C.c_void_p(hout.ptr), C.c_void_p(dout.ptr), nb, s2)
        L.nxec_stream_sync(s1)
        L.nxec_stream_sync(s2)
        return round(reps * nb / (time.perf_counter() - t0) / (1 << 30), 2)

    dma(True, True, 1)
    rf["dma_GiB_s"] = {"h2d_alone": dma(True, False), "d2h_alone": dma(False, True),
                       "both_at_once_per_direction": dma(True, True)}
    for b in (hin, hout, din, dout):
        b.free()
rf["label"] = sys.argv[1] if len(sys.argv) > 1 else ""
rf["lib"] = os.environ.get("NXEC_LIB", "product")
rf["lanes"] = os.environ.get("NXEC_HOST_LANES", "")
rf["numa_node"] = node
print(json.dumps(rf), flush=True)
ctx.close()
