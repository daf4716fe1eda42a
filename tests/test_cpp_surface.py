"""The C++ coding surface (RSCode / CodingUtils / CodingGenerator / DecodingPlan,
nexoedge_amd/csrc/coding) driven like the reference's coding_test.cc, on the GPU.

build/rs_surface_test self-checks every round trip (memcmp, like the
reference) and prints digests; here they are compared with the golden
vectors of the reference and, where the golden set has no entry, with the
CPU oracle.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle
from helpers import case_seed, fill_bytes, sha

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "rs_surface_test")


def test_surface_binary_built():
    assert os.path.exists(BIN), "run `make` (build/rs_surface_test)"


@pytest.mark.gpu
def test_rscode_surface_matches_reference(golden):
    cs = 1000
    r = subprocess.run([BIN, str(cs)], capture_output=True, text=True, timeout=600)
    out = r.stdout.splitlines()
    fails = [l for l in out if l.startswith("FAIL")]
    assert r.returncode == 0 and not fails and out[-1].startswith("PASSED"), (fails[:10], r.stderr[-2000:])

    enc_golden = {(c["n"], c["k"]): c["parity_sha256"] for c in golden["encode"] if c["cs"] == cs}
    rep_golden = {(c["n"], c["k"], tuple(c["failed"])): c for c in golden["repair"] if c["cs"] == cs}
    stripes = {}

    def stripe(n, k):
        if (n, k) not in stripes:
            stripes[(n, k)] = oracle.rs_encode(n, k, fill_bytes(k * cs, case_seed(n, k, cs)), cs)
        return stripes[(n, k)]

    checked = {"ENC": 0, "DEC": 0, "REP": 0, "RP2": 0}
    for line in out:
        f = line.split()
        if not f or f[0] not in checked:
            continue
        n, k = int(f[1]), int(f[2])
        st = stripe(n, k)
        if f[0] == "ENC":
            want = enc_golden.get((n, k)) or sha(st[k:])
            assert f[4] == want, line
        elif f[0] == "DEC":
            assert f[4] == sha(st[:k]), line
        else:
            failed = tuple(int(x) for x in f[4].split(","))
            g = rep_golden.get((n, k, failed))
            if g is not None:
                assert f[5] == g["repair_matrix_hex"] and f[6] == g["repaired_sha256"], line
            else:
                ok, ids, _, rm = oracle.rs_pre_decode(n, k, list(failed), True)
                assert f[5] == rm.tobytes().hex(), line
                assert f[6] == sha(st[list(failed)]), line
        checked[f[0]] += 1
    # 2 CAR modes x (54 coding_test pairs + 3 config geometries)
    assert checked["ENC"] == 2 * 57 and checked["DEC"] == 2 * 57
    assert checked["REP"] > 500 and checked["RP2"] > 2000


COMPAT = os.path.join(ROOT, "build", "isal_compat_test")


def test_compat_binary_built():
    assert os.path.exists(COMPAT), "run `make` (build/isal_compat_test)"


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,cs", [(14, 10, 1000), (6, 4, 31), (20, 16, 4096), (16, 12, 65537), (4, 2, 1)])
def test_isal_compat_header_drop_in(golden, n, k, cs):
    """rs.cc's ISA-L call sequence, recompiled against nxec_isal_compat.h, gives
    the reference's parity and restores the data."""
    r = subprocess.run([COMPAT, str(n), str(k), str(cs)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dict(l.split(" ", 1) for l in r.stdout.splitlines() if " " in l)
    want = [c["parity_sha256"] for c in golden["encode"] if (c["n"], c["k"], c["cs"]) == (n, k, cs)]
    assert want and lines["PARITY"].strip() == want[0]
    assert lines["DECODED"].strip() == sha(fill_bytes(k * cs, case_seed(n, k, cs)))
