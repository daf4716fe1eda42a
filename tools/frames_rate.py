"""Chunk-frame gather / scatter rates (nxec_gather_chunks / nxec_scatter_chunks):
pageable and pinned frames, 1 MiB chunks, alone and with concurrent callers.
FRAMES_READ=1: the bench's read path (nxec_decode_frames vs the sequential
calls) under the pool size NXEC_HOST_THREADS gives.
Run on the GPU box: python tools/frames_rate.py"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

GIB = float(1 << 30)
cs, nchunks, reps = 1 << 20, 1280, 3


def run(ctx, frames, dev, op):
    for _ in range(reps):
        if op == "gather":
            ctx.gather_chunks(frames, cs, dev.ptr, cs)
        else:
            ctx.scatter_chunks(dev.ptr, cs, frames, cs)


def timed(jobs):
    ths = [threading.Thread(target=run, args=j) for j in jobs]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return len(jobs) * reps * nchunks * cs / (time.perf_counter() - t0) / GIB


def setup(callers, pinned):
    ctxs, devs, bufs, frames = [], [], [], []
    for _ in range(callers):
        ctxs.append(nxec.Context(0))
        devs.append(nxec.DeviceBuffer(nchunks * cs))
        if pinned:
            b = nxec.PinnedBuffer(nchunks * cs)
            base = b.ptr
        else:
            b = np.ones(nchunks * cs, dtype=np.uint8)
            base = b.ctypes.data
        bufs.append(b)
        frames.append([base + i * cs for i in range(nchunks)])
    return ctxs, devs, bufs, frames


def teardown(ctxs, devs, bufs, pinned):
    for d in devs:
        d.free()
    if pinned:
        for b in bufs:
            b.free()
    for c in ctxs:
        c.close()


def rate(callers, op, pinned):
    ctxs, devs, bufs, frames = setup(callers, pinned)
    jobs = [(ctxs[i], frames[i], devs[i], op) for i in range(callers)]
    for j in jobs:
        run(*j)
    r = timed(jobs)
    teardown(ctxs, devs, bufs, pinned)
    return r


def duplex():
    """one caller gathers while another scatters (both PCIe directions)"""
    ctxs, devs, bufs, frames = setup(2, False)
    jobs = [(ctxs[0], frames[0], devs[0], "gather"), (ctxs[1], frames[1], devs[1], "scatter")]
    for j in jobs:
        run(*j)
    r = timed(jobs)
    teardown(ctxs, devs, bufs, False)
    return r


def one_caller_duplex(use_async, pinned=False):
    """ONE caller moving request i out (scatter) and request i+1 in (gather):
    sequential synchronous calls vs both async requests in flight on two streams"""
    from ctypes import byref, c_void_p

    from nexoedge_amd._lib import lib
    ctxs, devs, bufs, frames = setup(1, pinned)
    ctx, dev_in, fin = ctxs[0], devs[0], frames[0]
    dev_out = nxec.DeviceBuffer(nchunks * cs)
    fout = (np.zeros(nchunks * cs, dtype=np.uint8), )
    fo = [fout[0].ctypes.data + i * cs for i in range(nchunks)]
    s1, s2 = c_void_p(), c_void_p()
    lib.nxec_stream_create(byref(s1))
    lib.nxec_stream_create(byref(s2))

    def step():
        if use_async:
            rg = ctx.gather_chunks_async(fin, cs, dev_in.ptr, cs, stream=s1)
            rs = ctx.scatter_chunks_async(dev_out.ptr, cs, fo, cs, stream=s2)
            rg.wait()
            rs.wait()
        else:
            ctx.gather_chunks(fin, cs, dev_in.ptr, cs)
            ctx.scatter_chunks(dev_out.ptr, cs, fo, cs)
    step()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    r = 2 * reps * nchunks * cs / (time.perf_counter() - t0) / GIB
    lib.nxec_stream_destroy(s1)
    lib.nxec_stream_destroy(s2)
    dev_out.free()
    teardown(ctxs, devs, bufs, pinned)
    return r


if os.environ.get("FRAMES_ASYNC"):  # only the one-caller duplex legs
    for pinned in (False, True):
        for a in (False, True, False, True):
            print(f"one caller gather+scatter pinned-in={pinned!s:5s} {'async' if a else 'sync '}: "
                  f"{one_caller_duplex(a, pinned):6.2f} GiB/s", flush=True)
    sys.exit(0)

if os.environ.get("FRAMES_READ"):  # the bench's read path (nxec_decode_frames) under this pool size
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: E402
    bench.nxec = nxec
    ctx = nxec.Context(0)
    r = bench.read_from_frames(ctx, 14, 10, cs, 256)
    print(f"read path NXEC_HOST_THREADS={os.environ.get('NXEC_HOST_THREADS', '8')}: {r}", flush=True)
    sys.exit(0)

if os.environ.get("FRAMES_QUICK"):  # one pageable gather pass (for a profiler timeline)
    print(f"gather   pinned=False callers=1: {rate(1, 'gather', False):6.2f} GiB/s", flush=True)
    sys.exit(0)
for pinned in (False, True):
    for op in ("gather", "scatter"):
        for callers in (1, 2, 4):
            print(f"{op:8s} pinned={pinned!s:5s} callers={callers}: {rate(callers, op, pinned):6.2f} GiB/s", flush=True)
print(f"duplex gather+scatter pageable: {duplex():6.2f} GiB/s", flush=True)
