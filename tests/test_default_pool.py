"""The default pool of the drop-in entry points (include/nxec.h §2,
nexoedge_amd/csrc/nxec_context.cpp): an unmodified proxy shares one RSCode
across its worker threads and never selects a GPU (chunk_manager.cc:
1779-1801, zmq.cc:83), so every call leases a pool member -- by default one
context per visible device -- chosen by nxec_default_pick.

CPU: the selection rule (pure) and the argument checks.  GPU: 16 threads
through RSCode::encode / decode / repair with the pool forced to 8 contexts
on the one device, bit-exact against the oracle with every member used
(build/dropin_pool_test), and the Python-level properties (the caller's
current device is left alone, the `current` rule serves one member).
"""
import json
import os
import subprocess

import pytest

from nexoedge_amd import _lib, nxec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "dropin_pool_test")


# ---- the selection rule (no device) ----

def test_pick_fewest_in_flight():
    assert nxec.default_pick([0, 0, 0, 0]) == 0
    assert nxec.default_pick([3, 1, 2, 1]) == 1
    assert nxec.default_pick([2, 2, 2, 0]) == 3


def test_pick_prefers_local_node_on_ties():
    nodes = [0, 0, 1, 1]
    # equal load: a device on the caller's node
    assert nxec.default_pick([0, 0, 0, 0], nodes, caller_node=1) == 2
    assert nxec.default_pick([0, 0, 0, 0], nodes, caller_node=0) == 0
    # the local devices one call busier than a remote one: the remote one
    assert nxec.default_pick([1, 1, 0, 1], nodes, caller_node=0) == 2
    # local busier by one, remote equal to it: local (a remote call costs half a call)
    assert nxec.default_pick([1, 1, 1, 1], nodes, caller_node=1) == 2
    # unknown caller node or unknown device node: no preference
    assert nxec.default_pick([0, 0, 0, 0], nodes, caller_node=-1) == 0
    assert nxec.default_pick([0, 0], [-1, 1], caller_node=1) == 0


def test_pick_sticks_to_previous_member_on_exact_ties():
    assert nxec.default_pick([0, 0, 0, 0], prev=2) == 2
    assert nxec.default_pick([1, 0, 0, 0], prev=0) == 1  # not a tie: the idle one
    nodes = [0, 0, 1, 1]
    assert nxec.default_pick([0, 0, 0, 0], nodes, caller_node=1, prev=0) == 2  # remote prev loses to local
    assert nxec.default_pick([0, 0, 0, 0], nodes, caller_node=1, prev=3) == 3


def test_pick_spreads_concurrent_callers():
    """16 callers arriving one after another, none finished: each takes the
    least-loaded member, so 8 members end with 2 calls each, and with two
    nodes every caller stays on its own node while that node has the fewest."""
    inflight = [0] * 8
    nodes = [0] * 4 + [1] * 4
    for c in range(16):
        i = nxec.default_pick(inflight, nodes, caller_node=c % 2)
        assert nodes[i] == c % 2
        inflight[i] += 1
    assert inflight == [2] * 8
    # all callers on node 0: its 4 devices fill to 1, then the remote 4 are used
    inflight = [0] * 8
    for _ in range(8):
        inflight[nxec.default_pick(inflight, nodes, caller_node=0)] += 1
    assert inflight == [1] * 8


def test_pick_rejects_bad_arguments():
    L = _lib.lib
    assert L.nxec_default_pick(0, None, None, -1, -1) == _lib.NXEC_ERR_INVALID
    assert L.nxec_default_pick(2, None, None, -1, -1) == _lib.NXEC_ERR_INVALID


def test_default_devices_arguments():
    import ctypes
    L = _lib.lib
    assert L.nxec_default_devices(None, 3) == _lib.NXEC_ERR_INVALID
    bad = (ctypes.c_int * 2)(0, -1)
    assert L.nxec_default_devices(bad, 2) == _lib.NXEC_ERR_INVALID
    cnt = ctypes.c_int(-1)
    assert L.nxec_default_pool_stats(None, None, None, None, 4, ctypes.byref(cnt)) == _lib.NXEC_ERR_INVALID
    assert L.nxec_default_pool_stats(None, None, None, None, 0, ctypes.byref(cnt)) == 0


def test_pool_binary_built():
    assert os.path.exists(BIN), "run `make` (build/dropin_pool_test)"


# ---- on the GPU ----

@pytest.mark.gpu
def test_rscode_16_threads_over_8_member_pool():
    """VERDICT r05 #1's acceptance test: 16 threads share one RSCode, the
    pool is 8 contexts on the one device; every encode bit-exact against the
    oracle, every 4-erasure decode and repair equal to the original, every
    member served calls, no caller's current device changed."""
    r = subprocess.run([BIN, "8", "16", "12", str(256 << 10)], capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, (r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(line[-1])
    assert res["ok"] and res["members"] == 8 and min(res["served"]) > 0, res
    assert sum(res["served"]) == res["calls"], res


_IN_PROCESS = r"""
import sys, threading
sys.path.insert(0, {root!r})
import numpy as np
import oracle
from nexoedge_amd import nxec
nxec.default_devices([0, 0, 0])
n, k, cs = 14, 10, 4096 + 48
enc = nxec.gen_rs_matrix(n, k)[k:]
errs = []
def worker(t):
    rng = np.random.default_rng(t)
    for it in range(20):
        data = [rng.integers(0, 256, cs, dtype=np.uint8) for _ in range(k)]
        got = nxec.encode_host(enc, data)
        want = oracle.matmul(enc, data)
        if not all(np.array_equal(g, w) for g, w in zip(got, want)):
            errs.append((t, it))
th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
[x.start() for x in th]
[x.join() for x in th]
st = nxec.default_pool_stats()
print("POOL", len(st), sum(s["calls"] for s in st), sum(s["inflight"] for s in st), len(errs))
nxec.default_devices("current")
nxec.encode_host(enc, [np.zeros(64, np.uint8)] * k)
print("CURRENT", len(nxec.default_pool_stats()))
"""


@pytest.mark.gpu
def test_pool_reconfiguration_and_python_callers():
    """A 3-member pool served from 6 Python threads (nxec_encode_host, the
    CodingUtils::encode entry): bit-exact, 120 calls, none left in flight;
    then the `current` rule (rounds 1-5) serves from the calling thread's
    device, whose member is listed (members are never destroyed)."""
    env = dict(os.environ)
    r = subprocess.run(["python", "-c", _IN_PROCESS.format(root=ROOT)], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    pool = [l for l in r.stdout.splitlines() if l.startswith("POOL")][0].split()
    assert pool[1:] == ["3", "120", "0", "0"], pool
    cur = [l for l in r.stdout.splitlines() if l.startswith("CURRENT")][0].split()
    assert int(cur[1]) >= 1, cur


_ENV_POOL = r"""
import sys
sys.path.insert(0, {root!r})
import numpy as np
from nexoedge_amd import nxec
n, k = 14, 10
enc = nxec.gen_rs_matrix(n, k)[k:]
try:
    nxec.encode_host(enc, [np.zeros(4096, np.uint8)] * k)
    st = nxec.default_pool_stats()
    print("POOL", len(st), [s["device"] for s in st], sum(s["calls"] for s in st))
except nxec.NxecError as e:
    print("ERROR", e.code)
"""


@pytest.mark.gpu
@pytest.mark.parametrize("value,want", [("0,0", "POOL 2 [0, 0] 1"), ("current", "POOL 1 [0] 1"),
                                        ("all", "POOL 1 [0] 1"), ("0,x", "ERROR -2")])
def test_default_devices_setting(value, want):
    """NXEC_DEFAULT_DEVICES (INTEGRATION.md deployment settings): a device
    list makes one member per entry, `current` and `all` one member on the
    one-GPU box, a malformed value fails the call with NXEC_ERR_INVALID
    instead of guessing."""
    env = dict(os.environ, NXEC_DEFAULT_DEVICES=value)
    r = subprocess.run(["python", "-c", _ENV_POOL.format(root=ROOT)], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith(("POOL", "ERROR"))][0]
    assert line == want, line


_ADMIT = r"""
import sys, threading
sys.path.insert(0, {root!r})
import numpy as np
import oracle
from nexoedge_amd import nxec
nxec.default_devices([0, 0, 0, 0])
n, k, cs = 14, 10, (256 << 10) + 16
enc = nxec.gen_rs_matrix(n, k)[k:]
nxec.default_admission(0, reset=True)
inputs = [[np.random.default_rng(100 * t + i).integers(0, 256, cs, dtype=np.uint8) for i in range(k)]
          for t in range(24)]
errs, go = [], threading.Barrier(24)
def worker(t):
    go.wait()
    for it in range(3):
        got = nxec.encode_host(enc, inputs[t])
        if not all(np.array_equal(g, w) for g, w in zip(got, oracle.matmul(enc, inputs[t]))):
            errs.append((t, it))
th = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
[x.start() for x in th]
[x.join() for x in th]
a = nxec.default_admission(0)
print("ADMIT", a["limit"], a["running"], a["peak"], int(a["waited"] > 0), len(errs))
"""


@pytest.mark.gpu
def test_admission_bounds_calls_per_device():
    """Per-device admission: 24 threads through a 4-member pool
    on the one device, each admitted call held 30 ms (NXEC_TEST_FAULT=
    admit_stall) -- never more than 8 run at once, the gate fills (callers
    waited) and drains (none running after), every encode bit-exact."""
    env = dict(os.environ, NXEC_TEST_FAULT="admit_stall")
    r = subprocess.run(["python", "-c", _ADMIT.format(root=ROOT)], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("ADMIT")][0].split()
    assert line[1:] == ["8", "0", "8", "1", "0"], line


def test_admission_rejects_bad_device():
    with pytest.raises(nxec.NxecError):
        nxec.default_admission(-1)
