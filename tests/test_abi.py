"""The C-ABI library loads, exports every symbol include/nxec.h declares, and
fails loudly (no CPU fallback) when no GPU is visible.  CPU only."""
import ctypes
import os
import re
import subprocess

import pytest

import nexoedge_amd
from nexoedge_amd import _lib, nxec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "nxec.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nxec_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_isal_replacements():
    syms = declared_symbols()
    for s in ("nxec_ec_encode_data", "nxec_ec_init_tables", "nxec_gf_gen_rs_matrix", "nxec_gf_invert_matrix",
              "nxec_gf_mul", "nxec_stripes_mul", "nxec_rs_encode_stripes", "nxec_rs_recover_stripes",
              "nxec_rs_decode_stripes"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    missing = [s for s in declared_symbols() if not hasattr(_lib.lib, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (nxec_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_python_binding_covers_header():
    assert set(declared_symbols()) <= set(_lib.EXPORTED)


def test_library_is_gfx950_code():
    # the offload bundle inside the .so names its target triple
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_version():
    assert "gfx950" in nexoedge_amd.__version__


@pytest.mark.skipif(nxec.device_count() > 0, reason="a GPU is visible")
def test_no_device_fails_loudly():
    with pytest.raises(nxec.NxecError) as e:
        nxec.Context(0)
    assert e.value.code == _lib.NXEC_ERR_NODEV
    import numpy as np
    with pytest.raises(nxec.NxecError):
        nxec.encode_host(np.ones((1, 2), dtype=np.uint8), [np.zeros(16, np.uint8)] * 2)


def test_invalid_arguments_rejected_before_device_use():
    # argument validation happens before any device work
    rc = _lib.lib.nxec_stripes_mul(None, 1, 2, None, None, None, 0, 0, None, None, 0, 0, None, 16, 1, None)
    assert rc == _lib.NXEC_ERR_INVALID
    rc = _lib.lib.nxec_rs_encode_stripes(None, 3, 4, None, 0, 0, 16, 1, None)
    assert rc == _lib.NXEC_ERR_INVALID
    assert b"invalid" in _lib.lib.nxec_last_error()
    # the fused checksum entries: no context, bad (n,k), missing buffers, negative sizes
    f = (ctypes.c_int32 * 1)(0)
    assert _lib.lib.nxec_rs_encode_md5_stripes(None, 14, 10, None, 0, 0, 256, 1, None, None) == _lib.NXEC_ERR_INVALID
    assert _lib.lib.nxec_rs_recover_md5_stripes(None, 14, 10, f, 1, None, 0, 0, 256, 1, None, None) == \
        _lib.NXEC_ERR_INVALID


def test_status_forms_return_errors_instead_of_aborting():
    """The ISA-L-signature drop-in has a _status twin that reports bad arguments
    (and device errors) as return codes; the process keeps running."""
    import numpy as np

    t = np.zeros(32 * 4, dtype=np.uint8)
    src = (ctypes.c_void_p * 2)()
    dst = (ctypes.c_void_p * 2)()
    tp = ctypes.c_void_p(t.ctypes.data)
    assert _lib.lib.nxec_ec_encode_data_status(16, 0, 1, tp, src, dst) == _lib.NXEC_ERR_INVALID  # k < 1
    assert _lib.lib.nxec_ec_encode_data_status(16, 2, 0, tp, src, dst) == _lib.NXEC_ERR_INVALID  # rows < 1
    assert _lib.lib.nxec_ec_encode_data_status(16, 2, 1, None, src, dst) == _lib.NXEC_ERR_INVALID  # no tables
    assert _lib.lib.nxec_ec_encode_data_status(-1, 2, 1, tp, src, dst) == _lib.NXEC_ERR_INVALID  # len < 0
    assert _lib.lib.nxec_encode_host(16, 200, 1, tp, src, dst) == _lib.NXEC_ERR_INVALID  # k > NXEC_MAX_K
    assert b"invalid" in _lib.lib.nxec_last_error()


def test_arena_without_device_falls_back():
    """nxec_host_alloc reports failure (it never hands out unpinned memory) when
    no device is usable; Chunk::allocateData then uses ordinary memory."""
    if nxec.device_count() > 0:
        pytest.skip("a GPU is visible")
    p = ctypes.c_void_p()
    rc = _lib.lib.nxec_host_alloc(1 << 20, ctypes.byref(p))
    assert rc in (_lib.NXEC_ERR_NODEV, _lib.NXEC_ERR_NOMEM) and not p.value
    assert _lib.lib.nxec_host_arena_owns(None) == 0


def test_batch_layout_policy():
    """nxec_batch_layout (host-only arithmetic): chunk strides of >= 2 MiB
    chunks padded (3 KiB for multiples of 4 MiB, 5 KiB at 2 MiB, 2 KiB
    otherwise); stripes of a power-of-two number of MiB padded by one chunk;
    any even number of MiB only when recover-heavy; three measured small
    shapes padded, other small chunks packed (profiles/r02_layout_sweep.log,
    r05_layout_big_pads.log, r05_layout_small_chunk_pads.log)."""
    M = 1 << 20
    assert nxec.batch_layout(14, M) == (M, 14 * M)
    assert nxec.batch_layout(14, M, 1) == (M, 15 * M)
    assert nxec.batch_layout(16, M) == (M, 17 * M)
    assert nxec.batch_layout(20, M) == (M, 20 * M)
    assert nxec.batch_layout(20, M, 1) == (M, 21 * M)
    assert nxec.batch_layout(20, 256 << 10) == ((256 << 10) + 4096, 20 * ((256 << 10) + 4096))  # measured shapes
    assert nxec.batch_layout(14, 128 << 10)[0] == (128 << 10) + 10240
    assert nxec.batch_layout(14, 256 << 10)[0] == (256 << 10) + 12288
    assert nxec.batch_layout(16, 256 << 10) == (256 << 10, 16 * (256 << 10))  # not measured: packed
    assert nxec.batch_layout(15, M, 1) == (M, 15 * M)  # already odd
    cs, ss = nxec.batch_layout(20, 4 * M)
    assert cs == 4 * M + 3072 and ss == 20 * cs
    assert nxec.batch_layout(20, 8 * M)[0] == 8 * M + 3072
    assert nxec.batch_layout(14, 2 * M)[0] == 2 * M + 5120
    assert nxec.batch_layout(20, 3 * M)[0] == 3 * M + 2048
    for n, ln in [(14, M), (16, M), (20, 4 * M), (6, 3 * M + 5), (4, 2 * M)]:
        for fl in (0, 1):
            cs, ss = nxec.batch_layout(n, ln, fl)
            assert cs >= ln and ss >= n * cs and cs % 16 == 0 and ss % 16 == 0


VOID_FORM = r"""
import ctypes, sys
sys.path.insert(0, {root!r})
from nexoedge_amd import _lib
lib = _lib.lib
k, rows, n = 2, 1, 64
t = (ctypes.c_ubyte * (32 * k * rows))()
lib.nxec_ec_init_tables(k, rows, (ctypes.c_ubyte * 2)(1, 1), t)
bufs = [(ctypes.c_ubyte * n)() for _ in range(k + rows)]
data = (ctypes.c_void_p * k)(*[ctypes.addressof(b) for b in bufs[:k]])
code = (ctypes.c_void_p * rows)(*[ctypes.addressof(b) for b in bufs[k:]])
lib.nxec_ec_encode_data(n, k, rows, t, data, code)
print("RETURNED", flush=True)
"""


def test_void_form_retries_then_aborts_without_a_device():
    """Option A: nxec_ec_encode_data keeps ISA-L's void
    signature (erasure_code.h:98).  A device error is retried once on a fresh
    context through the staged path; only when that fails too (here: no
    device at all) does it abort -- never return undefined parity.  The
    _status form reports the same failure as a return code."""
    import signal
    import sys

    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-c", VOID_FORM.format(root=ROOT)], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == -signal.SIGABRT, (r.returncode, r.stderr[-2000:])
    assert "retrying once on a fresh context" in r.stderr and "RETURNED" not in r.stdout
    # bad arguments are not retried (they cannot succeed)
    bad = VOID_FORM.replace("lib.nxec_ec_encode_data(n, k, rows", "lib.nxec_ec_encode_data(-1, k, rows")
    r = subprocess.run([sys.executable, "-c", bad.format(root=ROOT)], capture_output=True, text=True, timeout=120,
                       env=env)
    assert r.returncode == -signal.SIGABRT and "retrying" not in r.stderr


def test_digest_table_is_per_thread_and_taken_once():
    """include/nxec.h §6b: a digest noted by a coding call is found only by
    the same thread, only for the same (pointer, length), and only once."""
    import threading

    import numpy as np

    buf = np.zeros(4096, dtype=np.uint8)
    d = np.arange(16, dtype=np.uint8)
    got = np.zeros(16, dtype=np.uint8)
    lib = _lib.lib
    lib.nxec_digest_clear()
    assert lib.nxec_digest_note(buf.ctypes.data, 4096, d.ctypes.data) == 0
    seen = []
    th = threading.Thread(target=lambda: seen.append(lib.nxec_digest_take(buf.ctypes.data, 4096, got.ctypes.data)))
    th.start()
    th.join()
    assert seen == [0]  # another thread's table is empty
    assert lib.nxec_digest_take(buf.ctypes.data, 4096, got.ctypes.data) == 1 and (got == d).all()
    assert lib.nxec_digest_take(buf.ctypes.data, 4096, got.ctypes.data) == 0
    lib.nxec_digest_note(buf.ctypes.data, 4096, d.ctypes.data)
    lib.nxec_digest_forget(buf.ctypes.data)
    assert lib.nxec_digest_take(buf.ctypes.data, 4096, got.ctypes.data) == 0
    assert lib.nxec_chunk_md5_mode() in (0, 1, 2)


def test_arena_bound_defaults_to_a_fraction_of_ram():
    """the pinned arena's default bound is an eighth of physical
    memory, at most 16 GiB (NXEC_HOST_ARENA_MAX overrides)."""
    if "NXEC_HOST_ARENA_MAX" in os.environ:
        pytest.skip("bound set explicitly")
    ram = os.sysconf("SC_PHYS_PAGES") * os.sysconf("SC_PAGESIZE")
    assert _lib.lib.nxec_host_arena_cap() == min(16 << 30, ram // 8)
    assert _lib.lib.nxec_host_arena_trim(0) == 0


PLACE_ENV = r"""
import ctypes, sys
sys.path.insert(0, {root!r})
from nexoedge_amd import _lib
print("MODE", _lib.lib.nxec_digest_placement(), flush=True)
"""


def test_digest_placement_modes():
    """include/nxec.h §2: nxec_encode_host_md5's digest placement -- auto by
    default, NXEC_DIGEST_PLACE=gpu|host pins it, the setter returns the
    previous mode and rejects unknown ones."""
    lib = _lib.lib
    prev = lib.nxec_digest_placement()
    try:
        assert lib.nxec_set_digest_placement(1) == prev
        assert lib.nxec_digest_placement() == 1
        assert lib.nxec_set_digest_placement(2) == 1
        assert lib.nxec_set_digest_placement(7) == _lib.NXEC_ERR_INVALID
        assert lib.nxec_digest_placement() == 2
    finally:
        lib.nxec_set_digest_placement(prev)
    h, g, t = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_int()
    assert lib.nxec_digest_place_stats(ctypes.byref(h), ctypes.byref(g), ctypes.byref(t)) == 0
    assert 0 <= t.value <= 16
    for env, want in ((None, 0), ("auto", 0), ("gpu", 1), ("host", 2)):
        e = dict(os.environ)
        e.pop("NXEC_DIGEST_PLACE", None)
        if env:
            e["NXEC_DIGEST_PLACE"] = env
        out = subprocess.run(["python", "-c", PLACE_ENV.format(root=ROOT)], capture_output=True, text=True,
                             env=e, timeout=120).stdout
        assert f"MODE {want}" in out, (env, out)


@pytest.mark.skipif(nxec.device_count() > 0, reason="a GPU is visible")
def test_host_placed_digests_fail_loudly_without_a_device():
    """A call placed on the host digest pool still codes on the GPU: with no
    device it returns the error (no CPU coding) after its queued input digests
    have drained -- no hang, the pool stays usable."""
    import numpy as np

    lib = _lib.lib
    prev = lib.nxec_set_digest_placement(2)
    try:
        for _ in range(3):
            with pytest.raises(nxec.NxecError) as e:
                nxec.encode_host_md5(np.ones((1, 3), dtype=np.uint8), [np.arange(70000, dtype=np.uint8)] * 3)
            assert e.value.code == _lib.NXEC_ERR_NODEV
    finally:
        lib.nxec_set_digest_placement(prev)


def test_product_build_and_round4_entry_points_without_a_device():
    """The product build carries no design-probe kernels (make PROBES=1 does),
    and the round-4 entry points validate before any device use: the kernel
    timers and every flag combination of the multi-file write refuse a
    missing context."""
    assert nxec.design_probes() is False
    ms, n = ctypes.c_double(-1.0), ctypes.c_int64(-1)
    assert _lib.lib.nxec_kernel_timing(None, 1) == _lib.NXEC_ERR_INVALID
    assert _lib.lib.nxec_kernel_time(None, ctypes.byref(ms), ctypes.byref(n)) == _lib.NXEC_ERR_INVALID
    ln = (ctypes.c_int64 * 1)(100)
    ptrs = (ctypes.c_void_p * 1)(None)
    for flags in (0, nxec.OBJECTS_TAIL_INPLACE, nxec.OBJECTS_ASYNC, nxec.OBJECTS_TAIL_INPLACE | nxec.OBJECTS_ASYNC, 4):
        assert _lib.lib.nxec_encode_objects_ex(None, 14, 10, 1, ptrs, ln, 1 << 20, None, None, None, flags,
                                               None) == _lib.NXEC_ERR_INVALID


def test_round5_entry_points_without_a_device():
    """The round-5 entry points validate before any device use: the layout
    calibration and the pipelined frames read refuse a missing context or
    bad geometry, and an empty read (no stripes, or zero-length chunks) is a
    no-op (with no stripes, no frame tables are needed)."""
    cs, ss = ctypes.c_int64(-1), ctypes.c_int64(-1)
    L = _lib.lib
    assert L.nxec_batch_layout_tuned(None, 14, 10, 1 << 20, 0, 0, ctypes.byref(cs), ctypes.byref(ss)) == \
        _lib.NXEC_ERR_INVALID
    assert (cs.value, ss.value) == (-1, -1)
    f = (ctypes.c_int32 * 4)(6, 7, 8, 9)
    fr = (ctypes.c_void_p * 14)()
    out = (ctypes.c_void_p * 10)()
    assert L.nxec_decode_frames(None, 14, 10, f, 4, fr, out, 1 << 20, 1, 0) == _lib.NXEC_ERR_INVALID
    assert b"nxec_decode_frames" in L.nxec_last_error() or b"invalid" in L.nxec_last_error()
    # bad geometry / negative sizes / missing frame tables are refused before the context is touched
    fake = ctypes.c_void_p(1)  # never dereferenced: validation fails first
    assert L.nxec_decode_frames(fake, 3, 4, f, 0, fr, out, 16, 1, 0) == _lib.NXEC_ERR_INVALID
    assert L.nxec_decode_frames(fake, 14, 10, f, 4, fr, out, -1, 1, 0) == _lib.NXEC_ERR_INVALID
    assert L.nxec_decode_frames(fake, 14, 10, f, 4, None, out, 16, 1, 0) == _lib.NXEC_ERR_INVALID
    assert L.nxec_decode_frames(fake, 14, 10, None, 4, fr, out, 16, 1, 0) == _lib.NXEC_ERR_INVALID
    # nothing to read: no frames needed, no device touched
    assert L.nxec_decode_frames(fake, 14, 10, f, 4, None, None, 16, 0, 0) == _lib.NXEC_OK
    assert L.nxec_decode_frames(fake, 14, 10, f, 4, fr, out, 0, 1, 0) == _lib.NXEC_OK


DEPLOYMENT_SETTINGS = {"NXEC_HOST_THREADS", "NXEC_HOST_DIRECT", "NXEC_SLOT_POOL_MAX", "NXEC_HOST_ARENA_MAX",
                       "NXEC_CHUNK_ARENA_MIN", "NXEC_CHUNK_MD5", "NXEC_DIGEST_PLACE", "NXEC_DIGEST_THREADS",
                       "NXEC_DIGEST_CPUS", "NXEC_DEFAULT_DEVICES"}
TEST_HOOKS = {"NXEC_TEST_FAULT", "NXEC_SYSFS_ROOT"}


def test_product_library_reads_only_the_documented_settings():
    """The default libnxec.so names no environment variable but the deployment
    settings INTEGRATION.md lists (each with its default) and the two test
    hooks, and carries no design-probe kernel: the A/B knobs and their
    kernels exist only in a `make PROBES=1` build (nxec_tuning.h)."""
    import re
    import subprocess
    if nxec.design_probes():
        pytest.skip("design-probe build")
    blob = open(_lib.LIB_PATH, "rb").read()
    names = set(re.findall(rb"NXEC_[A-Z][A-Z0-9_]+", blob))
    env_like = {n.decode() for n in names if not n.startswith((b"NXEC_ERR", b"NXEC_OK"))}
    assert env_like == DEPLOYMENT_SETTINGS | TEST_HOOKS, env_like ^ (DEPLOYMENT_SETTINGS | TEST_HOOKS)
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    table = doc[doc.index("## Deployment settings"):]
    for name in DEPLOYMENT_SETTINGS:
        assert re.search(r"^\| `" + name + r"` \| [^|]+ \|", table, re.M), name
    # probe kernels: k_mul_md5<K, HSRC, PROBE, NIBBLE, HASHSRC_GLOBAL> with a probe
    # or variant argument set, k_files_md5<K, PROBE != 0, ...>
    syms = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    em = re.findall(rb"k_mul_md5ILi(\d+)ELb([01])ELi(\d+)ELb([01])ELb([01])E", blob)
    fm = re.findall(rb"k_files_md5ILi(\d+)ELi(\d+)E", blob)
    assert em and fm, "kernel names not found in the library"
    assert all(int(p) == 0 and nib == b"0" and hg == b"0" for _, _, p, nib, hg in em)
    assert all(int(p) == 0 for _, p in fm)
    assert "nxec_design_probes" in syms
