"""Fused encode + per-chunk MD5 (k_encode_md5, nexoedge_amd/csrc/nxec_encode_md5.hip).

The proxy's write path (chunk_manager.cc:66-452) codes each stripe with
RSCode::encode and then hashes every chunk (Chunk::computeMD5, :175).  The
fused kernel does both in one pass; bar: parity bit-exact with the oracle
(the reference's ISA-L arithmetic), digests equal to hashlib's MD5, and both
byte-identical to the two-kernel path on the same inputs -- the public calls
the fused kernel replaces (coding through nxec_encode_object / recover without
digests, then nxec_md5_chunks).
"""
import hashlib

import numpy as np
import pytest

import oracle
from helpers import fill_bytes
from nexoedge_amd import nxec

pytestmark = pytest.mark.gpu


def _md5_interleaved(ctx, parts, ns, n):
    """[ns][n][16] digests from nxec_md5_chunks calls, each part (base,
    chunk_stride, stripe_stride, nchunks, length, nstripes, first chunk id, first stripe)."""
    out = np.zeros((ns, n, 16), dtype=np.uint8)
    for base, cst, sst, nch, length, nst, c0, s0 in parts:
        if nst == 0 or nch == 0:
            continue
        d = nxec.DeviceBuffer(nst * nch * 16)
        ctx.md5_chunks(base, cst, sst, nch, length, nst, d.ptr)
        ctx.sync()
        out[s0:s0 + nst, c0:c0 + nch] = d.download().reshape(nst, nch, 16)
        d.free()
    return out


def _encode_object(ctx, n, k, M, obj_buf, length, fused):
    """nxec_encode_object with digests (fused: the full stripes through
    k_mul_md5), or -- the two-kernel reference -- the same call without digests
    followed by nxec_md5_chunks over the object, the tail arena and the parity."""
    ns, nf, cl = nxec.object_layout(n, k, length, M)
    p = n - k
    par = nxec.DeviceBuffer(max(ns * p * M, 1))
    tail = nxec.DeviceBuffer(k * M)
    md5 = nxec.DeviceBuffer(ns * n * 16 + 3)
    if fused:
        # digests at an odd address: the kernel writes them byte-wise
        ctx.encode_object(n, k, obj_buf.ptr, length, M, par.ptr, tail.ptr, md5.ptr + 3)
        ctx.sync()
        dig = md5.download()[3:].reshape(ns, n, 16)
    else:
        ctx.encode_object(n, k, obj_buf.ptr, length, M, par.ptr, tail.ptr, None)
        ctx.sync()
        t = ns - nf
        dig = _md5_interleaved(ctx, [(obj_buf.ptr, M, k * M, k, M, nf, 0, 0), (par.ptr, M, p * M, p, M, nf, k, 0),
                                     (tail.ptr, cl, k * cl, k, cl, t, 0, nf),
                                     (par.ptr + nf * p * M, M, p * M, p, cl, t, k, nf)], ns, n)
    out = par.download().reshape(ns, p, M), dig
    for b in (par, tail, md5):
        b.free()
    return out


@pytest.mark.parametrize("n,k,M,nstripes", [
    (14, 10, 256, 1),        # one step, one stripe
    (14, 10, 4096, 37),      # groups of 16 stripes + a partial group
    (5, 4, 256, 300),        # p = 1, many groups
    (6, 4, 65536, 17),       # config-1 geometry, 256 steps
    (24, 20, 512, 13),       # k = 20, p = 4: S = 10 stripes per group, one LDS table copy
    (16, 12, 1024, 21),      # k = 12: largest k with two table copies
    (17, 13, 768, 33),       # k = 13, chunk an odd multiple of the step
    (3, 1, 256, 40),         # k = 1
    (9, 7, 2048, 5),         # fewer stripes than CUs x S: S shrinks
])
def test_fused_encode_md5_matches_oracle_and_hashlib(gpu_ctx, n, k, M, nstripes):
    length = nstripes * k * M  # full stripes only: all of them through the fused kernel
    obj = fill_bytes(length, 9100 + n * 31 + M)
    ob = nxec.DeviceBuffer(length)
    ob.upload(obj)
    par, dig = _encode_object(gpu_ctx, n, k, M, ob, length, fused=True)
    par2, dig2 = _encode_object(gpu_ctx, n, k, M, ob, length, fused=False)
    ob.free()
    assert np.array_equal(par, par2)
    assert np.array_equal(dig, dig2)
    p = n - k
    for s in sorted({0, nstripes // 2, nstripes - 1}):
        st = oracle.rs_encode(n, k, obj[s * k * M:(s + 1) * k * M], M)
        for i in range(p):
            assert np.array_equal(par[s, i], st[k + i]), (s, i)
        for c in range(n):
            assert dig[s, c].tobytes().hex() == hashlib.md5(st[c].tobytes()).hexdigest(), (s, c)


def test_fused_encode_md5_object_with_tail(gpu_ctx):
    """Full stripes through the fused kernel, the zero-padded last stripe
    (chunk_manager.cc:390-399) through encode + MD5: every digest vs hashlib."""
    n, k, M = 14, 10, 8192
    length = 5 * k * M + 12345
    obj = fill_bytes(length, 4242)
    ob = nxec.DeviceBuffer(length)
    ob.upload(obj)
    par, dig = _encode_object(gpu_ctx, n, k, M, ob, length, fused=True)
    ob.free()
    ns, nf, cl = nxec.object_layout(n, k, length, M)
    assert (ns, nf) == (6, 5)
    for s in range(ns):
        cs = M if s < nf else cl
        sd = np.zeros(k * cs, dtype=np.uint8)
        piece = obj[s * k * M:s * k * M + k * cs]
        sd[:len(piece)] = piece
        st = oracle.rs_encode(n, k, sd, cs)
        for i in range(n - k):
            assert np.array_equal(par[s, i, :cs], st[k + i])
        for c in range(n):
            assert dig[s, c].tobytes().hex() == hashlib.md5(st[c].tobytes()).hexdigest(), (s, c)


def test_fused_encode_md5_full_batch(gpu_ctx):
    """BASELINE size: 4096 RS(10,4) stripes of 1 MiB (56 GiB).  Fused parity and
    all 57 344 digests equal the two-kernel path's (whose digests
    test_rs10_4_full_batch_roundtrip pins to hashlib stripe by stripe); three
    stripes re-checked against the oracle and hashlib here."""
    n, k, M, ns = 14, 10, 1 << 20, 4096
    p = n - k
    length = ns * k * M
    ob = nxec.DeviceBuffer(length)
    ob.fill_random(321)
    par = nxec.DeviceBuffer(ns * p * M)
    dig = [nxec.DeviceBuffer(ns * n * 16) for _ in range(2)]
    sums = []
    for fused in (True, False):
        par.memset(0)
        if fused:
            gpu_ctx.encode_object(n, k, ob.ptr, length, M, par.ptr, None, dig[0].ptr)
        else:  # the two kernels: coding, then the MD5 of the object's and the parity's chunks
            gpu_ctx.encode_object(n, k, ob.ptr, length, M, par.ptr, None, None)
            gpu_ctx.md5_chunks(ob.ptr, M, k * M, k, M, ns, dig[1].ptr)
        gpu_ctx.sync()
        sums.append(par.checksum())
    assert sums[0] == sums[1]
    d0 = dig[0].download().reshape(ns, n, 16)
    dpar = nxec.DeviceBuffer(ns * p * 16)
    gpu_ctx.md5_chunks(par.ptr, M, p * M, p, M, ns, dpar.ptr)
    gpu_ctx.sync()
    d1 = np.concatenate([dig[1].download(ns * k * 16).reshape(ns, k, 16), dpar.download().reshape(ns, p, 16)], axis=1)
    dpar.free()
    assert np.array_equal(d0, d1)
    for s in (0, 1777, ns - 1):
        data = ob.download(k * M, offset=s * k * M)
        st = oracle.rs_encode(n, k, data, M)
        pp = par.download(p * M, offset=s * p * M).reshape(p, M)
        for i in range(p):
            assert np.array_equal(pp[i], st[k + i])
        for c in range(n):
            assert d0[s, c].tobytes().hex() == hashlib.md5(st[c].tobytes()).hexdigest(), (s, c)
    for b in [ob, par] + dig:
        b.free()


@pytest.mark.parametrize("n,k,cs,cstride,sstride,ns", [
    (14, 10, 65536, 65536, 14 * 65536, 40),              # packed [s][n][cs]
    (14, 10, 65536, 65536 + 2048, 15 * (65536 + 2048), 33),  # padded chunk and stripe strides
    (20, 16, 4096, 4096 + 16, 21 * (4096 + 16), 300),    # RS(16,4), odd stride padding
    (6, 4, 1000, 1008, 6 * 1008, 9),                     # len not a multiple of 256: encode + MD5 launches
])
def test_rs_encode_md5_stripes(gpu_ctx, n, k, cs, cstride, sstride, ns):
    """nxec_rs_encode_md5_stripes == nxec_rs_encode_stripes + nxec_md5_chunks on the
    same batch; sampled stripes vs the oracle and hashlib."""
    host = np.zeros((ns, sstride), dtype=np.uint8)
    data = fill_bytes(ns * k * cs, 77 + cs).reshape(ns, k, cs)
    for s in range(ns):
        for j in range(k):
            host[s, j * cstride:j * cstride + cs] = data[s, j]
    a = nxec.DeviceBuffer(host.nbytes)
    b = nxec.DeviceBuffer(host.nbytes)
    a.upload(host)
    b.upload(host)
    da = nxec.DeviceBuffer(ns * n * 16)
    db = nxec.DeviceBuffer(ns * n * 16)
    gpu_ctx.rs_encode_md5(n, k, a.ptr, cstride, sstride, cs, ns, da.ptr)
    gpu_ctx.rs_encode(n, k, b.ptr, cstride, sstride, cs, ns)
    gpu_ctx.md5_chunks(b.ptr, cstride, sstride, n, cs, ns, db.ptr)
    gpu_ctx.sync()
    ha, hb = a.download().reshape(ns, sstride), b.download().reshape(ns, sstride)
    assert np.array_equal(ha, hb)
    ga, gb = da.download().reshape(ns, n, 16), db.download().reshape(ns, n, 16)
    assert np.array_equal(ga, gb)
    for s in sorted({0, ns // 3, ns - 1}):
        st = oracle.rs_encode(n, k, data[s].reshape(-1), cs)
        for c in range(n):
            assert np.array_equal(ha[s, c * cstride:c * cstride + cs], st[c]), (s, c)
            assert ga[s, c].tobytes().hex() == hashlib.md5(st[c].tobytes()).hexdigest(), (s, c)
    for x in (a, b, da, db):
        x.free()


@pytest.mark.parametrize("n,k,cs,cstride,sstride,ns,failed", [
    (16, 12, 65536, 65536, 17 * 65536, 40, [0]),           # config-4 geometry, single failure (the repair path)
    (16, 12, 65536, 65536, 16 * 65536, 21, [15]),          # a parity chunk
    (14, 10, 4096, 4096 + 16, 14 * (4096 + 16), 300, [1, 4, 11, 13]),  # scattered 4 erasures, padded strides
    (20, 16, 768, 768, 20 * 768, 33, [0, 1, 2]),
    (6, 4, 1000, 1008, 6 * 1008, 9, [2]),                  # len not a multiple of 256: recover + MD5 launches
    (24, 20, 512, 512, 24 * 512, 13, [5, 23]),             # k = 20
])
def test_rs_recover_md5_stripes(gpu_ctx, n, k, cs, cstride, sstride, ns, failed):
    """Repair with checksums (rs.cc:238-322 + Chunk::computeMD5, chunk_manager.cc:1173):
    the rebuilt chunks equal the oracle's encode of the same data, their digests
    equal hashlib's, and fused == recover + nxec_md5_chunks of the rebuilt chunks."""
    data = fill_bytes(ns * k * cs, 313 + cs + len(failed)).reshape(ns, k, cs)
    full = np.zeros((ns, sstride), dtype=np.uint8)
    for s in range(ns):
        st = oracle.rs_encode(n, k, data[s].reshape(-1), cs)
        for c in range(n):
            full[s, c * cstride:c * cstride + cs] = st[c]
    damaged = full.copy()
    for s in range(ns):
        for f in failed:
            damaged[s, f * cstride:f * cstride + cs] = 0xA5
    outs = []
    for fused in (True, False):
        b = nxec.DeviceBuffer(damaged.nbytes)
        b.upload(damaged)
        d = nxec.DeviceBuffer(ns * len(failed) * 16)
        if fused:
            gpu_ctx.rs_recover_md5(n, k, failed, b.ptr, cstride, sstride, cs, ns, d.ptr)
            gpu_ctx.sync()
            dig = d.download().reshape(ns, len(failed), 16)
        else:
            gpu_ctx.rs_recover(n, k, failed, b.ptr, cstride, sstride, cs, ns)
            gpu_ctx.sync()
            dig = _md5_interleaved(gpu_ctx, [(b.ptr + f * cstride, cstride, sstride, 1, cs, ns, r, 0)
                                             for r, f in enumerate(failed)], ns, len(failed))
        outs.append((b.download().reshape(ns, sstride), dig))
        b.free()
        d.free()
    assert np.array_equal(outs[0][0], full)
    assert np.array_equal(outs[1][0], full)
    assert np.array_equal(outs[0][1], outs[1][1])
    for s in sorted({0, ns // 2, ns - 1}):
        for r, f in enumerate(failed):
            assert outs[0][1][s, r].tobytes().hex() == hashlib.md5(full[s, f * cstride:f * cstride + cs].tobytes()).hexdigest()


def test_rs_recover_md5_full_batch(gpu_ctx):
    """Config 4 at full size: 4096 RS(12,4) 1 MiB stripes on the recommended
    layout (17 MiB stripes), chunk 0 rebuilt with its MD5.  The rebuilt batch's
    checksum equals the original's; digests equal the two-kernel path's and,
    for three stripes, hashlib's."""
    n, k, cs, ns = 16, 12, 1 << 20, 4096
    cst, sst = nxec.batch_layout(n, cs, 0)
    buf = nxec.DeviceBuffer(ns * sst)
    buf.fill_random(4040)
    gpu_ctx.rs_encode(n, k, buf.ptr, cst, sst, cs, ns)
    gpu_ctx.sync()
    ref = buf.checksum()
    digs = []
    for fused in (True, False):
        # erase chunk 0 of every stripe: 0 x chunk 1 -> chunk 0
        gpu_ctx.stripes_mul(np.zeros((1, 1), dtype=np.uint8), buf.ptr, buf.ptr, src_idx=[1], dst_idx=[0],
                            src_chunk_stride=cst, src_stripe_stride=sst, dst_chunk_stride=cst, dst_stripe_stride=sst,
                            length=cs, nstripes=ns)
        gpu_ctx.sync()
        assert buf.checksum() != ref
        d = nxec.DeviceBuffer(ns * 16)
        if fused:
            gpu_ctx.rs_recover_md5(n, k, [0], buf.ptr, cst, sst, cs, ns, d.ptr)
        else:
            gpu_ctx.rs_recover(n, k, [0], buf.ptr, cst, sst, cs, ns)
            gpu_ctx.md5_chunks(buf.ptr, cst, sst, 1, cs, ns, d.ptr)
        gpu_ctx.sync()
        assert buf.checksum() == ref
        digs.append(d.download().reshape(ns, 16))
        d.free()
    assert np.array_equal(digs[0], digs[1])
    for s in (0, 2049, ns - 1):
        c0 = buf.download(cs, offset=s * sst)
        assert digs[0][s].tobytes().hex() == hashlib.md5(c0.tobytes()).hexdigest()
    buf.free()


def _object_chunks(n, k, M, obj, par_h, length):
    """[ns][n][M] chunks as the agents store them: data chunks cut from the
    object (last stripe zero padded, chunk_manager.cc:390-399), parity from
    nxec_encode_object's [ns][n-k][M] parity."""
    ns, nf, cl = nxec.object_layout(n, k, length, M)
    ch = np.zeros((ns, n, M), dtype=np.uint8)
    for s in range(ns):
        cs = M if s < nf else cl
        sd = np.zeros(k * cs, dtype=np.uint8)
        piece = obj[s * k * M:s * k * M + k * cs]
        sd[:len(piece)] = piece
        ch[s, :k, :cs] = sd.reshape(k, cs)
        ch[s, k:, :cs] = par_h[s, :, :cs]
    return ch


@pytest.mark.parametrize("failed", [[], [1, 4, 11, 13], [10, 11], [0, 1, 2, 3]])
def test_decode_object_verify(gpu_ctx, failed):
    """Read path with checksums (Chunk::verifyMD5 of every fetched chunk,
    chunk_manager.cc:1548-1556, then decodeFile), fused verify + decode: the
    object comes back intact, every chunk read is flagged ok, a corrupted
    input is flagged and counted.  (The verify launches + decode form runs in
    test_decode_object_verify_many_losses.)"""
    n, k, M = 14, 10, 65536
    length = 5 * k * M + 77777
    obj = fill_bytes(length, 6060 + len(failed))
    ob = nxec.DeviceBuffer(length)
    ob.upload(obj)
    ns, nf, cl = nxec.object_layout(n, k, length, M)
    par = nxec.DeviceBuffer(ns * (n - k) * M)
    tail = nxec.DeviceBuffer(k * M)
    md5 = nxec.DeviceBuffer(ns * n * 16)
    gpu_ctx.encode_object(n, k, ob.ptr, length, M, par.ptr, tail.ptr, md5.ptr)
    gpu_ctx.sync()
    ch = _object_chunks(n, k, M, obj, par.download().reshape(ns, n - k, M), length)
    alive = [c for c in range(n) if c not in failed][:k]
    bad_s, bad_c = 2, alive[0]
    ch[bad_s, bad_c, 100] ^= 0x5A  # one fetched chunk corrupted in transit
    for c in failed:
        ch[:, c] = 0xEE
    cb = nxec.DeviceBuffer(ch.nbytes)
    cb.upload(ch)
    out = nxec.DeviceBuffer(length)
    ok = nxec.DeviceBuffer(ns * n)
    ok.memset(7)
    nb = nxec.DeviceBuffer(8)
    nb.memset(0)
    gpu_ctx.decode_object_verify(n, k, failed, cb.ptr, length, M, md5.ptr, out.ptr, tail.ptr, ok.ptr, nb.ptr)
    gpu_ctx.sync()
    flags = ok.download().reshape(ns, n)
    want = np.full((ns, n), 7, dtype=np.uint8)
    want[:, alive] = 1
    want[bad_s, bad_c] = 0
    assert np.array_equal(flags, want)
    assert int(nb.download().view(np.uint64)[0]) == 1
    got = out.download()
    keep = np.ones(length, dtype=bool)
    keep[bad_s * k * M:(bad_s + 1) * k * M] = False  # the flagged stripe is re-planned by the caller
    assert np.array_equal(got[keep], obj[keep])
    for b in (ob, par, tail, md5, cb, out, ok, nb):
        b.free()


def test_decode_object_verify_many_losses(gpu_ctx):
    """More lost data chunks than one fused pass rebuilds (e = 5 > 4): the
    verify launches + decode path, same contract."""
    n, k, M = 20, 14, 4096
    length = 7 * k * M + 999
    failed = [0, 2, 4, 6, 8]
    obj = fill_bytes(length, 8181)
    ob = nxec.DeviceBuffer(length)
    ob.upload(obj)
    ns, nf, cl = nxec.object_layout(n, k, length, M)
    par = nxec.DeviceBuffer(ns * (n - k) * M)
    tail = nxec.DeviceBuffer(k * M)
    md5 = nxec.DeviceBuffer(ns * n * 16)
    gpu_ctx.encode_object(n, k, ob.ptr, length, M, par.ptr, tail.ptr, md5.ptr)
    gpu_ctx.sync()
    ch = _object_chunks(n, k, M, obj, par.download().reshape(ns, n - k, M), length)
    alive = [c for c in range(n) if c not in failed][:k]
    ch[ns - 1, alive[-1], 3] ^= 1  # corrupt an input of the (ragged) last stripe
    for c in failed:
        ch[:, c] = 0
    cb = nxec.DeviceBuffer(ch.nbytes)
    cb.upload(ch)
    out = nxec.DeviceBuffer(length)
    ok = nxec.DeviceBuffer(ns * n)
    ok.memset(9)
    nb = nxec.DeviceBuffer(8)
    nb.memset(0)
    gpu_ctx.decode_object_verify(n, k, failed, cb.ptr, length, M, md5.ptr, out.ptr, tail.ptr, ok.ptr, nb.ptr)
    gpu_ctx.sync()
    want = np.full((ns, n), 9, dtype=np.uint8)
    want[:, alive] = 1
    want[ns - 1, alive[-1]] = 0
    assert np.array_equal(ok.download().reshape(ns, n), want)
    assert int(nb.download().view(np.uint64)[0]) == 1
    assert np.array_equal(out.download()[:nf * k * M], obj[:nf * k * M])
    for b in (ob, par, tail, md5, cb, out, ok, nb):
        b.free()


@pytest.mark.parametrize("env", [("NXEC_EM_TABLES", "nib"), ("NXEC_EM_HASHSRC", "global")])
@pytest.mark.parametrize("M,nstripes", [(256, 1), (4096, 37), (65536, 300)])
def test_fused_encode_md5_variants_ab(gpu_ctx, monkeypatch, env, M, nstripes):
    """The fused write kernel's A/B variants (k = 10): conflict-free
    split-nibble tables (NXEC_EM_TABLES=nib) and hash lanes reading the source
    chunks from global memory (NXEC_EM_HASHSRC=global).  Parity and digests equal
    the default kernel's and the oracle / hashlib.  The variants are built only
    with `make PROBES=1` (nxec_design_probes()); the product build skips."""
    if not nxec.design_probes():
        pytest.skip("library built without the design-probe kernels (make PROBES=1)")
    n, k = 14, 10
    length = nstripes * k * M
    obj = fill_bytes(length, 7300 + M)
    ob = nxec.DeviceBuffer(length)
    ob.upload(obj)
    par, dig = _encode_object(gpu_ctx, n, k, M, ob, length, fused=True)
    monkeypatch.setenv(*env)
    par2, dig2 = _encode_object(gpu_ctx, n, k, M, ob, length, fused=True)
    ob.free()
    assert np.array_equal(par, par2)
    assert np.array_equal(dig, dig2)
    for s in sorted({0, nstripes - 1}):
        st = oracle.rs_encode(n, k, obj[s * k * M:(s + 1) * k * M], M)
        for i in range(n - k):
            assert np.array_equal(par2[s, i], st[k + i]), (s, i)
        for c in range(n):
            assert dig2[s, c].tobytes().hex() == hashlib.md5(st[c].tobytes()).hexdigest(), (s, c)
