"""The unmodified write path's MD5 on the GPU (call sites
chunk_manager.cc:175, :1173, agent.cc:342): nxec_encode_host_md5 codes a stripe
and hashes its chunks in the same k_gather_md5 pass (inputs hashed too for
RSCode::encode), concurrent callers aggregated into one launch.  Bit-exact
against the oracle's encode and hashlib MD5, for arena (zero copy), pageable
and misaligned buffers, every shape RSCode / the agent sends, chunk sizes off
the 256-byte step.  Plus the round-2 advisor's items on the same runtime:
exception-safe aggregation rounds, the arena trim, the verified read's tail
stripe, and the void drop-in's retry."""
import ctypes as C
import hashlib
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import oracle
from nexoedge_amd import _lib, nxec
from test_gpu_agent_fused import Arena, make_buf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = _lib.lib


def md5(a):
    return np.frombuffer(hashlib.md5(np.ascontiguousarray(a).tobytes()).digest(), dtype=np.uint8)


PLACES = {"auto": 0, "gpu": 1, "host": 2}


@pytest.fixture
def placement(request):
    """nxec_encode_host_md5's digest placement for the test (include/nxec.h §2)."""
    prev = lib.nxec_set_digest_placement(PLACES[request.param])
    assert prev >= 0
    yield request.param
    lib.nxec_set_digest_placement(prev)


def place_stats():
    h, g, t = C.c_ulonglong(), C.c_ulonglong(), C.c_int()
    lib.nxec_digest_place_stats(C.byref(h), C.byref(g), C.byref(t))
    return h.value, g.value


@pytest.mark.gpu
@pytest.mark.parametrize("placement", ["gpu", "host"], indirect=True)
@pytest.mark.parametrize("n,k", [(14, 10), (6, 4), (4, 2), (16, 12), (20, 16), (5, 1)])
@pytest.mark.parametrize("cs", [1 << 20, 65537, 4096, 1000, 31])
@pytest.mark.parametrize("kind", ["arena", "pageable", "mixed"])
def test_encode_host_md5_rs_stripe(gpu_ctx, placement, n, k, cs, kind):
    """RSCode::encode's call: parity + the digests of all n chunks, hashed in
    the coding kernel (gpu) or on the host digest pool (host)."""
    h0, g0 = place_stats()
    rng = np.random.default_rng(n * 1000 + k + cs)
    arena = Arena()
    try:
        data = [make_buf(arena, kind, cs, j) for j in range(k)]
        for d in data:
            d[:] = rng.integers(0, 256, size=cs, dtype=np.uint8)
        outs = [make_buf(arena, kind, cs, k + r) for r in range(n - k)]
        enc = nxec.gen_rs_matrix(n, k)[k:]
        _, md_in, md_out = nxec.encode_host_md5(enc, data, outs)
        want = oracle.rs_encode(n, k, np.concatenate(data), cs)
        for r in range(n - k):
            assert np.array_equal(outs[r], want[k + r]), f"parity {r}"
            assert np.array_equal(md_out[r], md5(outs[r])), f"parity digest {r}"
        for j in range(k):
            assert np.array_equal(md_in[j], md5(data[j])), f"data digest {j}"
        h1, g1 = place_stats()
        assert (h1 - h0, g1 - g0) == ((1, 0) if placement == "host" else (0, 1))
    finally:
        arena.free()


@pytest.mark.gpu
@pytest.mark.parametrize("placement", ["gpu", "host"], indirect=True)
def test_encode_host_md5_outputs_only_and_empty(gpu_ctx, placement):
    """RSCode::decode(isRepair) / CodingUtils::encode: only the outputs hashed;
    a zero-length call gives the empty message's digest."""
    rng = np.random.default_rng(5)
    for ni, no, cs in [(10, 1, 1 << 20), (12, 4, 300000), (3, 1, 17), (16, 4, 4096)]:
        m = rng.integers(0, 256, size=(no, ni), dtype=np.uint8)
        data = [rng.integers(0, 256, size=cs, dtype=np.uint8) for _ in range(ni)]
        outs, md_in, md_out = nxec.encode_host_md5(m, data, hash_inputs=False)
        assert md_in is None
        want = oracle.matmul(m, data)
        for r in range(no):
            assert np.array_equal(outs[r], want[r]) and np.array_equal(md_out[r], md5(want[r]))
    z = [np.zeros(0, dtype=np.uint8)] * 2
    _, mi, mo = nxec.encode_host_md5(np.ones((1, 2), dtype=np.uint8), z, [np.zeros(0, dtype=np.uint8)])
    assert bytes(mo[0]).hex() == "d41d8cd98f00b204e9800998ecf8427e" and bytes(mi[1]).hex() == bytes(mo[0]).hex()


@pytest.mark.gpu
@pytest.mark.parametrize("placement", ["gpu", "auto"], indirect=True)
def test_encode_host_md5_concurrent_callers_share_rounds(gpu_ctx, placement):
    """16 threads each encoding RS(10,4) stripes with digests at once (the
    proxy's workers): every stripe's parity and 14 digests are right whatever
    round it joined -- or, under auto placement, wherever each call hashed."""
    n, k, cs = 14, 10, 256 << 10
    h0, g0 = place_stats()
    enc = nxec.gen_rs_matrix(n, k)[k:]
    errors = []

    def worker(t):
        try:
            arena = Arena()
            rng = np.random.default_rng(100 + t)
            for it in range(4):
                data = [arena.array(cs) for _ in range(k)]
                for d in data:
                    d[:] = rng.integers(0, 256, size=cs, dtype=np.uint8)
                outs = [arena.array(cs) for _ in range(n - k)]
                _, mi, mo = nxec.encode_host_md5(enc, data, outs)
                want = oracle.rs_encode(n, k, np.concatenate(data), cs)
                for r in range(n - k):
                    if not (np.array_equal(outs[r], want[k + r]) and np.array_equal(mo[r], md5(want[k + r]))):
                        errors.append((t, it, r))
                for j in range(k):
                    if not np.array_equal(mi[j], md5(data[j])):
                        errors.append((t, it, "d", j))
            arena.free()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:10]
    h1, g1 = place_stats()
    assert (h1 - h0) + (g1 - g0) == 64
    if placement == "gpu":
        assert h1 == h0
    print(f"placement {placement}: host calls {h1 - h0}, gpu calls {g1 - g0}")


def _run(code, env_extra, timeout=300):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=env)


LEADER_THROWS = r"""
import sys, threading
sys.path.insert(0, {root!r})
import numpy as np
from nexoedge_amd import nxec
ctx = nxec.Context(0)
res = []
def call():
    try:
        m = np.ones((1, 2), dtype=np.uint8)
        ins = [np.zeros(4096, np.uint8), np.zeros(4096, np.uint8)]
        ctx.agent_encode_batch([(m, ins, [np.zeros(4096, np.uint8)], np.zeros((1, 16), np.uint8))], 4096)
        res.append("ok")
    except nxec.NxecError as e:
        res.append(e.code)
th = [threading.Thread(target=call) for _ in range(8)]
[t.start() for t in th]
[t.join(timeout=60) for t in th]
print("RESULTS", sorted(map(str, res)), "ALIVE", sum(t.is_alive() for t in th), flush=True)
"""


@pytest.mark.gpu
def test_agent_round_leader_exception_releases_everyone():
    """a leader that throws while building a round must still
    finish the round's jobs with an error and hand leadership on -- no caller
    may block forever (NXEC_TEST_FAULT=agent_round makes every leader throw)."""
    r = _run(LEADER_THROWS.format(root=ROOT), {"NXEC_TEST_FAULT": "agent_round"}, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULTS")][0]
    assert "ALIVE 0" in line and line.count(str(_lib.NXEC_ERR_NOMEM)) == 8, line


@pytest.mark.gpu
def test_arena_trim_returns_free_blocks(gpu_ctx):
    p = C.c_void_p()
    assert lib.nxec_host_alloc(8 << 20, C.byref(p)) == 0
    assert lib.nxec_host_free(p) == 0
    pinned, used = C.c_size_t(), C.c_size_t()
    lib.nxec_host_arena_stats(C.byref(pinned), C.byref(used))
    assert pinned.value >= 8 << 20
    assert lib.nxec_host_arena_trim(used.value) == 0
    lib.nxec_host_arena_stats(C.byref(pinned), C.byref(used))
    assert pinned.value == used.value  # every free block unpinned
    assert lib.nxec_host_arena_owns(p) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["tail", "full"])
def test_decode_object_verify_flags_a_corrupt_chunk(gpu_ctx, where):
    """Chunk::verifyMD5 of the fetched chunks (chunk_manager.cc:
    1548-1556) on the object read path -- a corrupted input chunk of the
    ragged tail stripe (or of a full stripe) is flagged, its stripe only, and
    counted; every other chunk reads ok."""
    n, k, M = 14, 10, 64 << 10
    length = 3 * k * M + 5 * 1000 + 7  # 3 full stripes + a ragged tail stripe
    ns, nf, cl = nxec.object_layout(n, k, length, M)
    assert (ns, nf) == (4, 3)
    obj = oracle.fill_bytes(length, 77)
    # the stored chunks [s][n][M] as the write path made them (the tail stripe zero-padded at cl)
    chunks = np.zeros((ns, n, M), dtype=np.uint8)
    digests = np.zeros((ns, n, 16), dtype=np.uint8)
    for s in range(ns):
        cs = M if s < nf else cl
        blob = np.zeros(k * cs, dtype=np.uint8)
        part = obj[s * k * M: s * k * M + k * cs]
        blob[:len(part)] = part
        st = oracle.rs_encode(n, k, blob, cs)
        for c in range(n):
            chunks[s, c, :cs] = st[c]
            digests[s, c] = md5(st[c])
    bad_s = ns - 1 if where == "tail" else 1
    bad_c = 5
    chunks[bad_s, bad_c, 3] ^= 0xFF
    failed = [0, 11]
    d_chunks, d_out, d_md5 = nxec.DeviceBuffer(chunks.nbytes), nxec.DeviceBuffer(length), nxec.DeviceBuffer(digests.nbytes)
    d_tail, d_ok, d_nbad = nxec.DeviceBuffer(k * M), nxec.DeviceBuffer(ns * n), nxec.DeviceBuffer(8)
    try:
        d_chunks.upload(chunks.reshape(-1))
        d_md5.upload(digests.reshape(-1))
        d_ok.memset(0xEE)
        d_nbad.memset(0)
        gpu_ctx.decode_object_verify(n, k, failed, d_chunks.ptr, length, M, d_md5.ptr, d_out.ptr, d_tail.ptr, d_ok.ptr,
                                     d_nbad.ptr)
        gpu_ctx.sync()
        ok = d_ok.download().reshape(ns, n)
        nbad = int(d_nbad.download().view(np.uint64)[0])
        assert nbad == 1
        alive = [c for c in range(n) if c not in failed][:k]
        for s in range(ns):
            for c in alive:
                assert ok[s, c] == (0 if (s, c) == (bad_s, bad_c) else 1), (s, c)
        out = d_out.download()
        good = [s for s in range(ns) if s != bad_s]
        for s in good:  # stripes without a bad chunk decode to the object's bytes
            lo, hi = s * k * M, min(length, (s + 1) * k * M)
            assert np.array_equal(out[lo:hi], obj[lo:hi]), s
    finally:
        for b in (d_chunks, d_out, d_md5, d_tail, d_ok, d_nbad):
            b.free()


@pytest.mark.gpu
def test_void_drop_in_retries_after_an_injected_device_error(golden):
    """Option A: rs.cc's ISA-L calls through include/nxec_isal_compat.h with the
    first attempt of every nxec_ec_encode_data failing (NXEC_TEST_FAULT=encode):
    the retry on a fresh context produces the golden parity, nothing aborts."""
    binary = os.path.join(ROOT, "build", "isal_compat_test")
    c = next(c for c in golden["encode"] if c["n"] == 14 and c["k"] == 10 and c["cs"] == 4096)
    r = subprocess.run([binary, "14", "10", "4096"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, NXEC_TEST_FAULT="encode"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "retrying once on a fresh context" in r.stderr
    assert c["parity_sha256"] in r.stdout, r.stdout[-500:]


AUTO_SWITCH = r"""
import ctypes as C, hashlib, sys, threading
sys.path.insert(0, {root!r})
import numpy as np
from nexoedge_amd import _lib, nxec
import oracle
lib = _lib.lib
n, k, cs = 14, 10, 256 << 10
enc = nxec.gen_rs_matrix(n, k)[k:]
bad = []
def worker(t, iters):
    rng = np.random.default_rng(t)
    for it in range(iters):
        data = [rng.integers(0, 256, size=cs, dtype=np.uint8) for _ in range(k)]
        outs, mi, mo = nxec.encode_host_md5(enc, data)
        want = oracle.rs_encode(n, k, np.concatenate(data), cs)
        for r in range(n - k):
            if not (np.array_equal(outs[r], want[k + r]) and bytes(mo[r]) == hashlib.md5(want[k + r].tobytes()).digest()):
                bad.append((t, it, r))
        for j in range(k):
            if bytes(mi[j]) != hashlib.md5(data[j].tobytes()).digest():
                bad.append((t, it, 'd', j))
def stats():
    h, g, th = C.c_ulonglong(), C.c_ulonglong(), C.c_int()
    lib.nxec_digest_place_stats(C.byref(h), C.byref(g), C.byref(th))
    return h.value, g.value
worker(99, 3)  # one caller: the pool
h1, g1 = stats()
ths = [threading.Thread(target=worker, args=(t, 12)) for t in range(6)]
[x.start() for x in ths]
[x.join() for x in ths]
h2, g2 = stats()
print("ONE", h1, g1, "MANY", h2 - h1, g2 - g1, "BAD", len(bad), flush=True)
"""


@pytest.mark.gpu
def test_auto_placement_moves_many_callers_to_the_gpu():
    """include/nxec.h §2, NXEC_DIGEST_PLACE=auto: a lone caller hashes on the
    host pool; once more threads call than the crossover (here
    NXEC_DIGEST_CPUS=2, so 6 callers > 2) the calls move to the
    coding kernel -- every digest and parity byte right either way."""
    r = _run(AUTO_SWITCH.format(root=ROOT), {"NXEC_DIGEST_CPUS": "2", "NXEC_DIGEST_PLACE": "auto"}, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("ONE")][0].split()
    one_h, one_g, many_h, many_g, nbad = int(line[1]), int(line[2]), int(line[4]), int(line[5]), int(line[7])
    assert nbad == 0
    assert one_h == 3 and one_g == 0, line
    assert many_g > many_h and many_h + many_g == 72, line
