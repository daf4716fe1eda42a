"""Pin the CPU oracle (oracle/nxec_oracle.c) to the reference.

tests/golden/golden.json holds outputs of the reference itself (ISA-L 2.22
ec_base.c compiled from /root/reference's tarball, driven by rs.cc's glue in
oracle/gen_golden.c).  Every oracle function must reproduce them bit for bit
before it is trusted as the checker of the HIP path.  CPU only.
"""
import hashlib

import numpy as np
import pytest

import oracle
from helpers import case_seed, fill_bytes, hexbytes, mixed_pattern, sha


def test_prng_matches_oracle():
    for n, seed in [(1, 7), (31, 12345), (1000, 99), (4097, 2**63 + 5)]:
        assert np.array_equal(fill_bytes(n, seed), oracle.fill_bytes(n, seed))


def test_field_tables(golden):
    mt = np.array([[oracle.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    assert hashlib.sha256(mt.tobytes()).hexdigest() == golden["gf_mul_table_sha256"]
    assert np.array_equal(mt[3], hexbytes(golden["gf_mul_row_3_hex"]))
    inv = np.array([oracle.gf_inv(a) for a in range(256)], dtype=np.uint8)
    assert np.array_equal(inv, hexbytes(golden["gf_inv_hex"]))


def test_encode_matrices(golden):
    for m in golden["matrices"]:
        a = oracle.gen_rs_matrix(m["n"], m["k"])
        assert a.tobytes().hex() == m["hex"], (m["n"], m["k"])


def test_init_tables(golden):
    for t in golden["init_tables"]:
        n, k = t["n"], t["k"]
        a = oracle.gen_rs_matrix(n, k)
        assert oracle.init_tables(a[k:]).tobytes().hex() == t["hex"]


def test_inverses(golden):
    for t in golden["inverses"]:
        n, k = t["n"], t["k"]
        a = oracle.gen_rs_matrix(n, k)
        rc, inv = oracle.invert_matrix(a[t["rows"]])
        assert rc == t["ret"] and inv.tobytes().hex() == t["inv_hex"]


def test_encode(golden):
    for c in golden["encode"]:
        n, k, cs = c["n"], c["k"], c["cs"]
        data = fill_bytes(k * cs, c["seed"])
        st = oracle.rs_encode(n, k, data, cs)
        assert np.array_equal(st[:k].reshape(-1), data)
        assert sha(st[k:]) == c["parity_sha256"], (n, k, cs)
        if "parity_hex" in c:
            assert st[k:].tobytes().hex() == c["parity_hex"]


def test_encode_data_via_tables(golden):
    # ec_encode_data semantics: the coefficient is byte [1] of each 32-B table
    for c in golden["encode"][:40]:
        n, k, cs = c["n"], c["k"], c["cs"]
        data = fill_bytes(k * cs, c["seed"]).reshape(k, cs)
        a = oracle.gen_rs_matrix(n, k)
        outs = oracle.encode_data(oracle.init_tables(a[k:]), k, n - k, list(data))
        assert sha(np.stack(outs)) == c["parity_sha256"]


def test_decode(golden):
    for c in golden["decode"]:
        n, k, cs = c["n"], c["k"], c["cs"]
        data = fill_bytes(k * cs, c["seed"])
        st = oracle.rs_encode(n, k, data, cs)
        ok, ids, mi, _ = oracle.rs_pre_decode(n, k, c["failed"], False)
        assert ok and len(ids) == c["ninputs"] and mi == k
        ok, out = oracle.rs_decode(n, k, ids[:k], [st[i] for i in ids[:k]])
        assert ok == c["ok"] == 1
        assert sha(out) == c["data_sha256"], (n, k, cs, c["failed"])
        assert c["matches_original"] == 1 and np.array_equal(out.reshape(-1), data)


def test_repair(golden):
    for c in golden["repair"]:
        n, k, cs, f = c["n"], c["k"], c["cs"], c["failed"]
        data = fill_bytes(k * cs, c["seed"])
        st = oracle.rs_encode(n, k, data, cs)
        ok, ids, mi, rm = oracle.rs_pre_decode(n, k, f, True)
        assert ok and len(ids) == c["ninputs"]
        assert rm.tobytes().hex() == c["repair_matrix_hex"], (n, k, f)
        ok, out = oracle.rs_decode(n, k, ids[:k], [st[i] for i in ids[:k]], is_repair=True, targets=f)
        assert ok == 1 and sha(out) == c["repaired_sha256"], (n, k, f)
        # applying the plan's repair matrix directly gives the same chunks
        outs = oracle.matmul(rm, [st[i] for i in ids[:k]])
        assert sha(np.stack(outs)) == c["repaired_sha256"]


def test_car_repair(golden):
    for c in golden["car"]:
        n, k, cs, f, g = c["n"], c["k"], c["cs"], c["failed"], c["rack_size"]
        data = fill_bytes(k * cs, c["seed"])
        st = oracle.rs_encode(n, k, data, cs)
        ok, ids, _, rm = oracle.rs_pre_decode(n, k, [f], True)
        assert rm[0].tobytes().hex() == c["repair_row_hex"]
        partials = []
        for (start, size), want in zip(c["groups"], c["partials_sha256"]):
            part = oracle.matmul(rm[:, start:start + size], [st[i] for i in ids[start:start + size]])[0]
            assert sha(part) == want
            partials.append(part)
        ok, out = oracle.rs_decode(n, k, list(range(len(partials))), partials, is_repair=True, targets=[f],
                                   use_car=True)
        assert ok == 1 and sha(out) == c["final_sha256"] and np.array_equal(out[0], st[f])


def test_agent_known_answer(golden):
    ka = golden["known_answer_agent_enc"]
    a = np.full(ka["cs"], ka["fill"], dtype=np.uint8)
    out = oracle.matmul(np.array([ka["coeffs"]], dtype=np.uint8), [a, a])[0]
    assert int((out == 0).sum()) == ka["zeros"] == ka["cs"]


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_matches_reference_library_random():
    """Cross-check against the compiled reference on random coefficient matrices."""
    ref = oracle.RefISAL()
    rng = np.random.default_rng(5)
    for _ in range(30):
        k = int(rng.integers(1, 24))
        rows = int(rng.integers(1, 8))
        cs = int(rng.integers(1, 3000))
        coeffs = rng.integers(0, 256, size=(rows, k), dtype=np.uint8)
        srcs = [rng.integers(0, 256, size=cs, dtype=np.uint8) for _ in range(k)]
        want = [np.zeros(cs, dtype=np.uint8) for _ in range(rows)]
        ref.encode(coeffs, srcs, want)
        got = oracle.matmul(coeffs, srcs)
        assert all(np.array_equal(g, w) for g, w in zip(got, want))


@pytest.mark.parametrize("level", [0, 256, 512])
def test_cpu_simd_baseline_matches_oracle(level):
    """The CPU-baseline SIMD stand-in (oracle/nxec_cpu_simd.c) is bit-exact with the
    oracle for ragged lengths and 1..9 rows (multi-pass)."""
    if level > oracle.simd_level():
        pytest.skip(f"host lacks SIMD level {level}")
    rng = np.random.default_rng(level + 3)
    for k, rows, length in [(10, 4, 4096 + 77), (1, 1, 63), (12, 1, 200), (16, 9, 1000), (4, 3, 64 * 5 + 31), (7, 2, 5)]:
        c = rng.integers(0, 256, size=(rows, k), dtype=np.uint8)
        srcs = [rng.integers(0, 256, size=length, dtype=np.uint8) for _ in range(k)]
        outs = [np.zeros(length, dtype=np.uint8) for _ in range(rows)]
        assert oracle.simd_encode(c, srcs, outs, level) == level
        want = oracle.matmul(c, srcs)
        for r in range(rows):
            assert np.array_equal(outs[r], want[r]), (k, rows, length, r)
