"""Host-memory paths of the drop-in boundary on the GPU: the pinned chunk
arena (Chunk::allocateData, reference chunk.hh:55-66), the zero-copy
eligibility test on whole ranges (a buffer registered only in part takes the
staged path), and recovery of a work-queue slot left dirty by an unfinished
launch.  Parity bar: bit-exact vs the oracle."""
import ctypes as C
import threading

import numpy as np
import pytest

import oracle
from helpers import fill_bytes
from nexoedge_amd import _lib, nxec

lib = _lib.lib


def arena_alloc(nbytes):
    p = C.c_void_p()
    nxec.check(lib.nxec_host_alloc(nbytes, C.byref(p)), "nxec_host_alloc")
    return p.value


def as_array(ptr, nbytes):
    return np.ctypeslib.as_array((C.c_ubyte * nbytes).from_address(ptr))


def encode_ptrs(coeffs, src_ptrs, dst_ptrs, length):
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape
    rc = lib.nxec_encode_host(length, k, rows, C.c_void_p(c.ctypes.data), (C.c_void_p * k)(*src_ptrs),
                              (C.c_void_p * rows)(*dst_ptrs))
    nxec.check(rc, "nxec_encode_host")


@pytest.mark.gpu
def test_arena_blocks_pinned_recycled_and_owned(gpu_ctx):
    p = arena_alloc(1 << 20)
    assert p % 4096 == 0
    assert lib.nxec_host_arena_owns(C.c_void_p(p)) == 1
    assert lib.nxec_host_arena_owns(C.c_void_p(p + 16)) == 0  # only block starts
    assert lib.nxec_host_range_mapped(C.c_void_p(p), 1 << 20) == 1
    pinned, used = C.c_size_t(), C.c_size_t()
    lib.nxec_host_arena_stats(C.byref(pinned), C.byref(used))
    assert used.value >= 1 << 20 and pinned.value >= used.value
    nxec.check(lib.nxec_host_free(C.c_void_p(p)), "free")
    assert arena_alloc((1 << 20) - 100) == p  # same size class: the block is reused
    nxec.check(lib.nxec_host_free(C.c_void_p(p)), "free")
    assert lib.nxec_host_free(C.c_void_p(p + 64)) == _lib.NXEC_ERR_INVALID
    # pageable memory is never reported mapped
    a = np.zeros(1 << 16, dtype=np.uint8)
    assert lib.nxec_host_range_mapped(C.c_void_p(a.ctypes.data), a.nbytes) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("outputs", ["pinned", "pageable"])
@pytest.mark.parametrize("threads,cs", [(1, 1 << 20), (1, 65536 + 3), (6, 1 << 20), (6, 300001)])
def test_arena_chunks_encode_without_staging(gpu_ctx, threads, cs, outputs):
    """RS(10,4) encode of arena chunk buffers through nxec_encode_host (the call
    under RSCode::encode / RSCode::decode): one caller runs the zero-copy kernel
    on the chunks themselves, many callers DMA them; pageable outputs (decode's
    malloc'd result) come back through the staging slot.  Bit-exact vs the oracle."""
    n, k = 14, 10
    enc = nxec.gen_rs_matrix(n, k)[k:]
    blocks = [[arena_alloc(cs) for _ in range(n)] for _ in range(threads)]
    host_out = [[np.full(cs, 0xEE, dtype=np.uint8) for _ in range(n - k)] for _ in range(threads)]
    want, errors = [], []
    for t in range(threads):
        data = fill_bytes(k * cs, 9100 + t).reshape(k, cs)
        for j in range(k):
            as_array(blocks[t][j], cs)[:] = data[j]
        for r in range(n - k):
            as_array(blocks[t][k + r], cs)[:] = 0xEE
        want.append(np.stack(oracle.matmul(enc, list(data))))

    def outs(t):
        return blocks[t][k:] if outputs == "pinned" else [o.ctypes.data for o in host_out[t]]

    def work(t):
        try:
            for _ in range(3):
                encode_ptrs(enc, blocks[t][:k], outs(t), cs)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    [x.start() for x in th]
    [x.join() for x in th]
    assert not errors, errors
    for t in range(threads):
        if outputs == "pinned":
            got = np.stack([as_array(blocks[t][k + r], cs).copy() for r in range(n - k)])
        else:
            got = np.stack(host_out[t])
        assert np.array_equal(got, want[t]), t
        for b in blocks[t]:
            lib.nxec_host_free(C.c_void_p(b))


@pytest.mark.gpu
def test_arena_misaligned_and_mixed_buffers_take_staged_path(gpu_ctx):
    n, k, cs = 9, 6, 65536 + 5
    enc = nxec.gen_rs_matrix(n, k)[k:]
    data = fill_bytes(k * cs, 4321).reshape(k, cs)
    blk = [arena_alloc(cs + 64) for _ in range(n)]
    src = [blk[j] + 1 for j in range(k)]  # misaligned inside pinned blocks
    for j in range(k):
        as_array(src[j], cs)[:] = data[j]
    pageable_out = [np.zeros(cs, dtype=np.uint8) for _ in range(n - k)]  # pageable outputs
    encode_ptrs(enc, src, [o.ctypes.data for o in pageable_out], cs)
    want = oracle.matmul(enc, list(data))
    assert all(np.array_equal(pageable_out[r], want[r]) for r in range(n - k))
    for b in blk:
        lib.nxec_host_free(C.c_void_p(b))


def _page_aligned(nbytes, extra_pages=2):
    raw = np.zeros(nbytes + (extra_pages + 1) * 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw, raw[off:off + nbytes + extra_pages * 4096]


@pytest.mark.gpu
def test_partly_registered_batch_takes_staged_path(gpu_ctx):
    """A buffer registered only in part is never handed to a zero-copy kernel
    (ADVICE r1): the whole-range test sees the unregistered part whichever end
    it is on, and the batch is staged with bit-exact parity."""
    n, k, cs, ns = 14, 10, 65536, 6
    keep_raw, data = _page_aligned(ns * k * cs)
    data = data[:ns * k * cs]
    data[:] = fill_bytes(ns * k * cs, 555)
    half = (ns * k * cs // 2) // 4096 * 4096
    base = data.ctypes.data
    nxec.check(lib.nxec_host_register(C.c_void_p(base + half), data.nbytes - half), "register")
    try:
        assert lib.nxec_host_range_mapped(C.c_void_p(base + half), data.nbytes - half) == 1
        # checked on the host, before any kernel may run: registered start, unregistered end ...
        assert lib.nxec_host_range_mapped(C.c_void_p(base + half), data.nbytes - half + 4096) == 0
        # ... and unregistered start, registered end
        assert lib.nxec_host_range_mapped(C.c_void_p(base), data.nbytes) == 0
        parity = nxec.PinnedBuffer(ns * (n - k) * cs)
        gpu_ctx.rs_encode_host_batch(n, k, base, parity.ptr, cs, ns, 2)
        enc = nxec.gen_rs_matrix(n, k)[k:]
        d = data.reshape(ns, k, cs)
        got = parity.array.reshape(ns, n - k, cs)
        for s in range(ns):
            assert np.array_equal(got[s], np.stack(oracle.matmul(enc, list(d[s])))), s
        parity.free()
    finally:
        nxec.check(lib.nxec_host_unregister(C.c_void_p(base + half)), "unregister")
    del keep_raw


@pytest.mark.gpu
def test_recover_frames_straddling_registration_is_staged(gpu_ctx):
    """One frame runs past the end of the registered receive pool: the frames
    are staged (no zero-copy kernel over the unmapped tail), result bit-exact."""
    n, k, cs, ns = 9, 6, 65536, 2
    failed = [0, 8]  # the last frame (stripe 1, chunk 8) is written and straddles the registration end
    enc = nxec.gen_rs_matrix(n, k)
    stripes = [np.concatenate([d, np.stack(oracle.matmul(enc[k:], list(d)))])
               for d in (fill_bytes(k * cs, 880 + s).reshape(k, cs) for s in range(ns))]
    keep_raw, pool = _page_aligned(ns * n * cs)
    pool = pool[:ns * n * cs + 4096]
    reg = ns * n * cs - 4096  # the last frame's final page is outside the registration
    for s in range(ns):
        for c in range(n):
            o = (s * n + c) * cs
            pool[o:o + cs] = 0 if c in failed else stripes[s][c]
    frames = [pool.ctypes.data + (s * n + c) * cs for s in range(ns) for c in range(n)]
    nxec.check(lib.nxec_host_register(C.c_void_p(pool.ctypes.data), reg), "register")
    try:
        assert lib.nxec_host_range_mapped(C.c_void_p(frames[-1]), cs) == 0
        assert lib.nxec_host_range_mapped(C.c_void_p(frames[0]), cs) == 1
        gpu_ctx.rs_recover_frames(n, k, failed, frames, cs, ns)
        for s in range(ns):
            for c in range(n):
                o = (s * n + c) * cs
                assert np.array_equal(pool[o:o + cs], stripes[s][c]), (s, c)
    finally:
        nxec.check(lib.nxec_host_unregister(C.c_void_p(pool.ctypes.data)), "unregister")
    del keep_raw


@pytest.mark.gpu
def test_dirty_queue_slot_skips_tiles_until_reset(gpu_ctx):
    """A work-queue slot left non-zero by a launch that never finished makes the
    launch drawing it skip tiles (negative control); nxec_reset_work_queues
    clears every slot and the next encode is bit-exact again."""
    n, k, cs, ns = 14, 10, 1 << 20, 8
    stripe = n * cs
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(2468)
    gpu_ctx.rs_encode(n, k, buf.ptr, cs, stripe, cs, ns)
    gpu_ctx.sync()
    good = buf.checksum()
    host = buf.download().reshape(ns, n, cs)
    want = np.stack(oracle.matmul(nxec.gen_rs_matrix(n, k)[k:], list(host[0, :k])))
    assert np.array_equal(host[0, k:], want)

    zero = np.zeros((n - k, 1), dtype=np.uint8)  # wipe the parity
    gpu_ctx.stripes_mul(zero, buf.ptr, buf.ptr, src_idx=[0], dst_idx=list(range(k, n)), src_chunk_stride=cs,
                        src_stripe_stride=stripe, dst_chunk_stride=cs, dst_stripe_stride=stripe, length=cs,
                        nstripes=ns)
    gpu_ctx.sync()
    nxec.check(lib.nxec_debug_poison_next_queue_slot(5), "poison")
    gpu_ctx.rs_encode(n, k, buf.ptr, cs, stripe, cs, ns)
    gpu_ctx.sync()
    assert buf.checksum() != good  # tiles 0..4 were skipped
    nxec.check(lib.nxec_debug_poison_next_queue_slot(5), "poison")
    nxec.check(lib.nxec_reset_work_queues(), "reset")
    gpu_ctx.rs_encode(n, k, buf.ptr, cs, stripe, cs, ns)
    gpu_ctx.sync()
    assert buf.checksum() == good
    buf.free()
