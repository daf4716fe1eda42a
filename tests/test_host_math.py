"""libnxec's host planning math (section 1 and rs_plan of include/nxec.h)
against the reference's golden vectors.  These are host-side matrix routines
(no GPU), exactly like rs.cc:26,196,219,290,316 run on the host."""
import pytest
import numpy as np

from nexoedge_amd import nxec
from helpers import hexbytes


def test_gf_mul_and_inv(golden):
    mt = np.array([[nxec.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    import hashlib
    assert hashlib.sha256(mt.tobytes()).hexdigest() == golden["gf_mul_table_sha256"]
    inv = np.array([nxec.gf_inv(a) for a in range(256)], dtype=np.uint8)
    assert np.array_equal(inv, hexbytes(golden["gf_inv_hex"]))


def test_gen_rs_matrix(golden):
    for m in golden["matrices"]:
        assert nxec.gen_rs_matrix(m["n"], m["k"]).tobytes().hex() == m["hex"]


def test_init_tables(golden):
    for t in golden["init_tables"]:
        n, k = t["n"], t["k"]
        assert nxec.init_tables(nxec.gen_rs_matrix(n, k)[k:]).tobytes().hex() == t["hex"]


def test_invert(golden):
    for t in golden["inverses"]:
        n, k = t["n"], t["k"]
        inv = nxec.invert_matrix(nxec.gen_rs_matrix(n, k)[t["rows"]])
        assert inv is not None and inv.tobytes().hex() == t["inv_hex"]
    assert nxec.invert_matrix(np.zeros((3, 3), dtype=np.uint8)) is None


def test_plan_matches_reference_repair_matrices(golden):
    for c in golden["repair"]:
        n, k, f = c["n"], c["k"], c["failed"]
        ids, mi, rm = nxec.rs_plan(n, k, f, True)
        assert len(ids) == c["ninputs"] and mi == k
        assert rm.tobytes().hex() == c["repair_matrix_hex"], (n, k, f)


def test_plan_read_inputs(golden):
    for c in golden["decode"]:
        ids, mi, _ = nxec.rs_plan(c["n"], c["k"], c["failed"], False)
        assert len(ids) == c["ninputs"] and mi == c["k"]
        assert not set(ids) & set(c["failed"]) and ids == sorted(ids)


def test_plan_rejects_too_many_failures():
    import pytest
    with pytest.raises(nxec.NxecError):
        nxec.rs_plan(6, 4, [0, 1, 2], False)


def test_decode_matrix_rows_are_consistent():
    # data targets -> inverse rows; parity targets -> enc row x inverse
    n, k = 14, 10
    enc = nxec.gen_rs_matrix(n, k)
    ids = [1, 2, 3, 5, 6, 7, 8, 9, 10, 12]
    m = nxec.decode_matrix(n, k, ids, [0, 4, 11, 13])
    inv = nxec.invert_matrix(enc[ids])
    assert np.array_equal(m[0], inv[0]) and np.array_equal(m[1], inv[4])
    for row, t in ((2, 11), (3, 13)):
        want = np.zeros(k, dtype=np.uint8)
        for j in range(k):
            s = 0
            for l in range(k):
                s ^= nxec.gf_mul(int(inv[l, j]), int(enc[t, l]))
            want[j] = s
        assert np.array_equal(m[row], want)


def test_car_plan_matches_reference_grouping(golden):
    """CAR planning (chunk_manager.cc:929-986) against the golden CAR cases:
    racks of g chunks (chunk i on rack i // g)."""
    for c in golden["car"]:
        n, k, f, g = c["n"], c["k"], c["failed"], c["rack_size"]
        racks = [list(range(r, min(r + g, n))) for r in range(0, n, g)]
        subs = nxec.car_plan(n, k, f, racks)
        row = bytes.fromhex(c["repair_row_hex"])
        ids, _, _ = nxec.rs_plan(n, k, [f], True)
        assert [len(ch) for ch, _ in subs] == [size for _, size in c["groups"]]
        for (chunks, coeffs), (start, size) in zip(subs, c["groups"]):
            assert chunks == ids[start:start + size]
            assert bytes(coeffs) == row[start:start + size]


def test_car_plan_unordered_racks_and_errors():
    import pytest
    n, k = 16, 12
    racks = [[12, 13, 14, 15], [3, 1, 0, 2], [7, 6, 5, 4], [8, 9, 10, 11]]
    subs = nxec.car_plan(n, k, 5, racks)
    ids, _, rm = nxec.rs_plan(n, k, [5], True)
    pos = {cid: i for i, cid in enumerate(ids[:k])}
    flat = [(cid, int(cf)) for ch, cfs in subs for cid, cf in zip(ch, cfs)]
    assert sorted(c for c, _ in flat) == sorted(ids[:k])
    assert all(cf == rm[0][pos[cid]] for cid, cf in flat)
    assert [ch for ch, _ in subs][:2] == [[12], [3, 1, 0, 2]]  # rack order and in-rack order kept
    with pytest.raises(nxec.NxecError):
        nxec.car_plan(n, k, 5, [[0, 1, 2]])  # racks do not cover the inputs


@pytest.mark.parametrize("n,k,length,M,want", [
    (14, 10, 0, 1 << 20, (0, 0, 0)),
    (14, 10, 10 << 20, 1 << 20, (1, 1, 1 << 20)),
    (14, 10, (30 << 20) + 1, 1 << 20, (4, 3, 1)),
    (6, 4, 4 << 20, 1 << 20, (1, 1, 1 << 20)),
    (6, 4, 4097, 4096, (1, 0, 1025)),
    (16, 12, 12 * 4096 * 5 + 13, 4096, (6, 5, 2)),
])
def test_object_layout(n, k, length, M, want):
    """Stripe split of proxy_file_ops.cc:557-666 and chunk size of rs.cc:52-55."""
    assert nxec.object_layout(n, k, length, M) == want


def test_survey_named_boundary(golden):
    """The §8b-named forms: nxec_gen_rs_matrix / nxec_init_tables equal the
    ISA-L-named ones; nxec_invert_matrix equals the golden inverse and leaves
    its input untouched (unlike ISA-L's gf_invert_matrix)."""
    import ctypes as C

    from nexoedge_amd._lib import lib
    for m in golden["matrices"][:10]:
        n, k = m["n"], m["k"]
        a = np.zeros(n * k, dtype=np.uint8)
        lib.nxec_gen_rs_matrix(a.ctypes.data, n, k)
        assert a.tobytes().hex() == m["hex"]
    for t in golden["init_tables"][:10]:
        n, k = t["n"], t["k"]
        c = np.ascontiguousarray(nxec.gen_rs_matrix(n, k)[k:])
        tb = np.zeros(c.size * 32, dtype=np.uint8)
        lib.nxec_init_tables(k, n - k, c.ctypes.data, tb.ctypes.data)
        assert tb.tobytes().hex() == t["hex"]
    for t in golden["inverses"][:50]:
        n, k = t["n"], t["k"]
        src = np.ascontiguousarray(nxec.gen_rs_matrix(n, k)[t["rows"]])
        before = src.copy()
        out = np.zeros_like(src)
        assert lib.nxec_invert_matrix(src.ctypes.data, out.ctypes.data, k) == 0
        assert out.tobytes().hex() == t["inv_hex"] and np.array_equal(src, before)
    z = np.zeros(9, dtype=np.uint8)
    assert lib.nxec_invert_matrix(z.ctypes.data, np.zeros(9, dtype=np.uint8).ctypes.data, 3) == -1


def test_every_tool_is_cited():
    """tools/ holds only what DESIGN.md, README.md, INTEGRATION.md, the
    Makefile or a test cites (one-off scripts live in tools/archive, outside
    the GPU push); at most 25 entries."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    entries = sorted(e for e in os.listdir(os.path.join(root, "tools")) if e not in ("archive", "__pycache__"))
    assert len(entries) <= 25, entries
    text = "".join(open(os.path.join(root, f)).read() for f in ("DESIGN.md", "README.md", "INTEGRATION.md", "Makefile"))
    tdir = os.path.join(root, "tests")
    text += "".join(open(os.path.join(tdir, f)).read() for f in os.listdir(tdir) if f.endswith(".py"))
    missing = [e for e in entries if f"tools/{e}" not in text]
    assert not missing, missing


def test_every_cited_profile_exists():
    """Every profiles/rNN_* file DESIGN.md, README.md or INTEGRATION.md cites
    is committed (the evidence the text quotes is there to be checked)."""
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = "".join(open(os.path.join(root, f)).read() for f in ("DESIGN.md", "README.md", "INTEGRATION.md"))
    names = set(re.findall(r"\b(r0[1-9]_[A-Za-z0-9_\-.]+?\.(?:jsonl|json|log|csv|txt))(?![A-Za-z0-9])", text))
    assert len(names) > 100
    missing = sorted(n for n in names if not os.path.exists(os.path.join(root, "profiles", n)))
    assert not missing, missing

