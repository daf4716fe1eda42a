"""Agent service, fused form (k_gather_md5): nxec_agent_encode_batch codes and
hashes each batch in one kernel straight from and into pinned host memory.
Inputs / outputs that are arena (pinned, device-mapped) buffers are used in
place; pageable or misaligned ones go through the staging slot.  Every shape
the agent sends (container_manager.cc:221-258 partial encodes, agent.cc:240-415
CAR / non-CAR repairs) and every buffer mix is checked bit-exactly against the
oracle's CodingUtils::encode and hashlib MD5 (agent.cc:342)."""
import ctypes as C
import hashlib
import zlib

import numpy as np
import pytest

import oracle
from nexoedge_amd import _lib, nxec

lib = _lib.lib


class Arena:
    """nxec_host_alloc blocks viewed as numpy arrays (the agent's Chunk buffers)."""

    def __init__(self):
        self.blocks = []

    def array(self, nbytes, offset=0):
        p = C.c_void_p()
        nxec.check(lib.nxec_host_alloc(nbytes + offset, C.byref(p)), "nxec_host_alloc")
        self.blocks.append(p.value)
        return np.ctypeslib.as_array((C.c_ubyte * nbytes).from_address(p.value + offset))

    def free(self):
        for b in self.blocks:
            lib.nxec_host_free(C.c_void_p(b))
        self.blocks = []


def make_buf(arena, kind, cs, i):
    if kind == "pageable":
        return np.zeros(cs, dtype=np.uint8)
    if kind == "arena":
        return arena.array(cs)
    if kind == "misaligned":  # inside a pinned block but not 16-byte aligned: staged
        return arena.array(cs, offset=8)
    return make_buf(arena, ("arena", "pageable", "misaligned")[i % 3], cs, i)  # mixed


def run_batch(gpu_ctx, shapes, cs, in_kind, out_kind, nreq, seed, with_md5=lambda r: True, batch_bytes=0):
    rng = np.random.default_rng(seed)
    arena = Arena()
    reqs, want = [], []
    try:
        for r in range(nreq):
            ni, no = shapes[r % len(shapes)]
            m = rng.integers(0, 256, size=(no, ni), dtype=np.uint8)
            ins = []
            for j in range(ni):
                a = make_buf(arena, in_kind, cs, r * 7 + j)
                a[:] = rng.integers(0, 256, size=cs, dtype=np.uint8)
                ins.append(a)
            outs = [make_buf(arena, out_kind, cs, r * 5 + o) for o in range(no)]
            for o in outs:
                o[:] = 0xEE
            md5 = np.zeros((no, 16), dtype=np.uint8) if with_md5(r) else None
            reqs.append((m, ins, outs, md5))
            want.append(oracle.matmul(m, [x.copy() for x in ins]))
        gpu_ctx.agent_encode_batch(reqs, cs, batch_bytes)
        for r, ((m, ins, outs, md5), w) in enumerate(zip(reqs, want)):
            for o in range(m.shape[0]):
                assert np.array_equal(outs[o], w[o]), (r, o)
                if md5 is not None:
                    assert md5[o].tobytes().hex() == hashlib.md5(w[o].tobytes()).hexdigest(), (r, o)
    finally:
        arena.free()


# (ninputs, noutputs): ENC partial encodes of racks of 1-4 chunks, CAR XOR of
# G partials, non-CAR repairs of 1-4 lost chunks from k = 10 / 12 / 16 inputs
SHAPES = [(4, 1), (3, 1), (1, 1), (2, 1), (12, 2), (10, 4), (16, 4), (16, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("in_kind,out_kind", [("pageable", "pageable"), ("arena", "arena"), ("arena", "pageable"),
                                              ("mixed", "mixed"), ("misaligned", "arena")])
def test_agent_fused_buffer_kinds(gpu_ctx, in_kind, out_kind):
    for ni_no in SHAPES:
        run_batch(gpu_ctx, [ni_no], 65536, in_kind, out_kind, nreq=5, seed=zlib.crc32(repr((in_kind, out_kind, ni_no)).encode()))


@pytest.mark.gpu
@pytest.mark.parametrize("cs", [256, 4096, 1 << 20])
def test_agent_fused_chunk_sizes_and_grouping(gpu_ctx, cs):
    """Interleaved shapes (one launch per matrix group), the smallest step
    (256 B), 1 MiB chunks; requests without a digest pointer in a hashed group."""
    nreq = 24 if cs == 1 << 20 else 60
    run_batch(gpu_ctx, SHAPES[:4], cs, "mixed", "mixed", nreq=nreq, seed=cs, with_md5=lambda r: r % 5 != 3)


@pytest.mark.gpu
def test_agent_fused_many_requests_packed_per_workgroup(gpu_ctx):
    """More requests than CUs: several per workgroup (S > 1) and a partial last
    workgroup; a small batch_bytes splits them over rotating staging slots."""
    run_batch(gpu_ctx, [(4, 1)], 4096, "arena", "arena", nreq=1100, seed=17)
    run_batch(gpu_ctx, [(3, 1), (12, 2)], 8192, "pageable", "arena", nreq=700, seed=18, batch_bytes=3 << 20)


@pytest.mark.gpu
@pytest.mark.parametrize("cs", [1, 15, 16, 17, 100, 255, 257, 319, 5000, 65536 + 16, (1 << 20) - 3])
def test_agent_fused_any_chunk_size(gpu_ctx, cs):
    """Chunk sizes that are not a multiple of the 256-byte step (a file's last
    stripe, ceil(rem/k) bytes): the partial last step reads and writes nothing
    past a chunk's end -- every output sits in a larger buffer whose bytes past
    cs must keep their sentinel -- and the MD5 padding is built in registers."""
    rng = np.random.default_rng(cs)
    arena = Arena()
    try:
        reqs, want, guards = [], [], []
        for r in range(6):
            ni, no = [(4, 1), (12, 2), (3, 1)][r % 3]
            m = rng.integers(0, 256, size=(no, ni), dtype=np.uint8)
            ins = []
            for j in range(ni):
                a = make_buf(arena, ("arena", "pageable")[(r + j) % 2], cs, r)
                a[:] = rng.integers(0, 256, size=cs, dtype=np.uint8)
                ins.append(a)
            outs, g = [], []
            for o in range(no):
                big = arena.array(cs + 64) if (r + o) % 2 == 0 else np.zeros(cs + 64, dtype=np.uint8)
                big[:] = 0xEE
                outs.append(big[:cs])
                g.append(big)
            md5 = np.zeros((no, 16), dtype=np.uint8)
            reqs.append((m, ins, outs, md5))
            want.append(oracle.matmul(m, [x.copy() for x in ins]))
            guards.append(g)
        gpu_ctx.agent_encode_batch(reqs, cs)
        for r, ((m, ins, outs, md5), w, g) in enumerate(zip(reqs, want, guards)):
            for o in range(m.shape[0]):
                assert np.array_equal(outs[o], w[o]), (r, o)
                assert md5[o].tobytes().hex() == hashlib.md5(w[o].tobytes()).hexdigest(), (r, o)
                assert (g[o][cs:] == 0xEE).all(), (r, o)  # nothing written past the chunk
    finally:
        arena.free()


@pytest.mark.gpu
@pytest.mark.parametrize("in_kind,out_kind", [("arena", "arena"), ("pageable", "pageable"), ("mixed", "mixed"),
                                              ("misaligned", "arena")])
@pytest.mark.parametrize("cs", [65536, 65536 + 16, 5000, 1])
def test_agent_without_digests_zero_copy(gpu_ctx, in_kind, out_kind, cs):
    """Groups that want no digest (ENC_CHUNK_REQ: getEncodedChunks computes
    none) run the gather form of the multiply kernel over the same pointer
    tables -- mapped buffers in place, the others through the slot."""
    run_batch(gpu_ctx, SHAPES, cs, in_kind, out_kind, nreq=10, seed=cs + 7, with_md5=lambda r: False)
