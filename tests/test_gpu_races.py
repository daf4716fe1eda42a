"""Races between callers that share one context (include/nxec.h: a context may
be shared by threads, as the reference shares one RSCode, chunk_manager.cc:
1779-1801).  Each case runs in its own process, with the NXEC_TEST_FAULT
stall that opens the window (read once per process)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_ZERO_LINE = r"""
import sys, threading, time, hashlib, ctypes as C
sys.path.insert(0, {root!r})
import numpy as np
from nexoedge_amd import nxec
ctx = nxec.Context(0)
n, k = 14, 10
p = n - k
res = {{}}

def write(name, M, lengths, delay):
    time.sleep(delay)
    st = C.c_void_p()
    assert nxec._lib.lib.nxec_stream_create(C.byref(st)) == 0
    rng = np.random.default_rng(M)
    offs = np.concatenate([[0], np.cumsum([(L + 15) // 16 * 16 for L in lengths])]).astype(int)
    host = rng.integers(0, 256, size=int(offs[-1]) + 16, dtype=np.uint8)
    arena = nxec.DeviceBuffer(host.size)
    arena.upload(host)
    total, tail_bytes = nxec.objects_layout(n, k, lengths, M)
    par, tail, md5 = (nxec.DeviceBuffer(total * p * M), nxec.DeviceBuffer(max(tail_bytes, 16)),
                      nxec.DeviceBuffer(total * n * 16))
    tail.memset(0)
    ctx.encode_objects(n, k, [arena.ptr + int(o) for o in offs[:-1]], lengths, M, par.ptr, tail.ptr, md5.ptr,
                       stream=st.value, flags=nxec.OBJECTS_TAIL_INPLACE)
    assert nxec._lib.lib.nxec_stream_sync(st) == 0
    dig = md5.download().reshape(total, n, 16)
    bad, g = 0, 0
    for o, L in zip(offs[:-1], lengths):
        ns, nf, cl = nxec.object_layout(n, k, L, M)
        for s in range(ns):
            cs = M if s < nf else cl
            base = o + s * k * M
            for j in range(k):  # data chunks: the object's bytes, zero padded past its end
                chunk = np.zeros(cs, np.uint8)
                lo, hi = base + j * cs, min(base + (j + 1) * cs, o + L)
                if hi > lo:
                    chunk[:hi - lo] = host[lo:hi]
                bad += dig[g + s, j].tobytes() != hashlib.md5(chunk.tobytes()).digest()
        g += ns
    res[name] = bad

# A: last stripes whose chunks past the data read the 1 MiB zero line, held
# 400 ms between taking the line and launching; B: a 4 MiB chunk size grows
# the line meanwhile (before the fix its old line was freed under A)
a = threading.Thread(target=write, args=("A", 4096, [10 * 4096 + 1, 2 * 10 * 4096 + 33, 5, 7 * 4096 + 3], 0.0))
b = threading.Thread(target=write, args=("B", 4 << 20, [3, 4 << 20], 0.1))
a.start(); b.start(); a.join(); b.join()
print("RESULT", res.get("A"), res.get("B"))
"""


@pytest.mark.gpu
def test_zero_line_growth_while_another_call_holds_it():
    """nxec_encode_objects_ex takes the context's zero line,
    then plans and launches; a concurrent call with a larger chunk size grows
    the line.  The old line is retired, not freed, so the first call's kernel
    still reads zeros: every digest of both calls equals hashlib's."""
    env = dict(os.environ, NXEC_TEST_FAULT="zero_stall")
    r = subprocess.run(["python", "-c", _ZERO_LINE.format(root=ROOT)], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0]
    assert line.split()[1:] == ["0", "0"], line
