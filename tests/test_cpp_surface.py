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
@pytest.mark.parametrize("cs", [1000, 65537])
def test_rscode_surface_matches_reference(golden, cs):
    """cs = 65537: the chunks RSCode::encode allocates come from the pinned
    arena (Chunk::allocateData >= 64 KiB), so encode runs the no-staging path."""
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


FLOW = os.path.join(ROOT, "build", "chunk_manager_flow_test")


def _flow(cases, timeout=300):
    args = [str(v) for c in cases for v in c]
    r = subprocess.run([FLOW] + args, capture_output=True, text=True, timeout=timeout)
    blocks, cur = [], None
    for line in r.stdout.splitlines():
        f = line.split()
        if not f:
            continue
        if f[0] == "CASE":
            cur = {"case": tuple(int(x) for x in f[1:]), "part": []}
            blocks.append(cur)
        elif cur is not None and f[0] == "PART":
            cur["part"].append(f[2])
        elif cur is not None and f[0] in ("ENC", "FINAL", "MATCH", "REFUSED_WITHOUT_CAR"):
            cur[f[0]] = f[1]
        elif cur is not None and f[0] == "OPTIONS":
            cur["OPTIONS"] = f[1:]
    return r, blocks


def test_default_options_read_config_via_bridge():
    """CodingOptions() + setN/setK, as ChunkManager builds them
    (chunk_manager.cc:25-27, 1789-1791), carries Config's CAR flag through the
    bridge (CPU: the options line is printed before any GPU call)."""
    assert os.path.exists(FLOW), "run `make` (build/chunk_manager_flow_test)"
    for car in (1, 0):
        _, blocks = _flow([(16, 12, 1000, 0, 4, car, 1)], timeout=60)
        assert blocks and blocks[0]["OPTIONS"] == [f"16-12{car}", f"16-12{car}"], blocks


@pytest.mark.gpu
@pytest.mark.parametrize("at_proxy", [1, 0])
def test_chunk_manager_flow_replica_car_repair(golden, at_proxy):
    """CAR single-failure repair with CAR taken from Config only (no setRepairUsingCAR
    call, as in the reference), at the proxy (accessGroupedChunks + RSCode::decode
    with G < k partials, chunk_manager.cc:1029,1141) and at an agent
    (RPR_CHUNK_REQ, agent.cc:249-339): partials and result equal the golden CAR cases."""
    cases = [(c["n"], c["k"], c["cs"], c["failed"], c["rack_size"], 1, at_proxy) for c in golden["car"]]
    r, blocks = _flow(cases)
    assert r.returncode == 0 and len(blocks) == len(cases), (r.stdout[-3000:], r.stderr[-2000:])
    for c, b in zip(golden["car"], blocks):
        assert b["MATCH"] == "1", b
        assert b["part"] == list(c["partials_sha256"]), (c, b)
        assert b["FINAL"] == c["final_sha256"], (c, b)
        enc = [e["parity_sha256"] for e in golden["encode"] if (e["n"], e["k"], e["cs"]) == (c["n"], c["k"], c["cs"])]
        if enc:
            assert b["ENC"] == enc[0]


@pytest.mark.gpu
@pytest.mark.parametrize("at_proxy", [1, 0])
def test_chunk_manager_flow_replica_conventional_repair(golden, at_proxy):
    """Same flows with repair_using_car = 0: k inputs and the plan's repair row,
    at the proxy (RSCode::decode) and at an agent (CodingUtils::encode with the
    proxy's matrix, agent.cc:339); fewer than k inputs are refused (rs.cc:133-136)."""
    cases = [(c["n"], c["k"], c["cs"], c["failed"], c["rack_size"], 0, at_proxy) for c in golden["car"]]
    r, blocks = _flow(cases)
    assert r.returncode == 0 and len(blocks) == len(cases), (r.stdout[-3000:], r.stderr[-2000:])
    for c, b in zip(golden["car"], blocks):
        assert b["MATCH"] == "1" and b["FINAL"] == c["final_sha256"], (c, b)
        if at_proxy:
            assert b["REFUSED_WITHOUT_CAR"] == "1", b


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


BATCH = os.path.join(ROOT, "build", "stripe_batch_test")


def test_stripe_batch_binary_built():
    assert os.path.exists(BATCH), "run `make` (build/stripe_batch_test)"


@pytest.mark.gpu
def test_stripe_batch_matches_per_stripe_rscode():
    """StripeBatch (whole-file encode + MD5 / decode, the batched ChunkManager
    entry) vs the per-stripe RSCode::encode path the reference takes, every
    chunk of every stripe, plus OpenSSL MD5 and the decoded file."""
    r = subprocess.run([BATCH], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("PASSED 0 failures"), (r.stdout[-3000:], r.stderr[-2000:])


REPLAY = os.path.join(ROOT, "build", "chunk_replay_test")


def test_chunk_replay_cpu():
    """The reference's Chunk ownership sequences (shallow `=` + freeData =
    false, move, return by value) against csrc/coding/chunk.hh without a GPU:
    every alias is the original buffer, every MD5 matches its bytes."""
    assert os.path.exists(REPLAY), "run `make` (build/chunk_replay_test)"
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    r = subprocess.run([REPLAY], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "PASSED 0 failures" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("cs", ["262144", "1048576", "1000"])
def test_chunk_replay_gpu(cs):
    """The same sequences with RSCode::encode / CodingUtils::encode on the GPU:
    writeFileStripe's computeMD5 (chunk_manager.cc:175) returns the digests the
    encode kernel computed, and each equals OpenSSL's MD5 of the chunk's bytes
    (checked in the binary for every chunk and every borrowed view)."""
    r = subprocess.run([REPLAY, cs], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASSED 0 failures (gpu)" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
