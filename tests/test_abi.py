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
    chunks padded by 2 KiB; stripes of a power-of-two number of MiB padded by
    one chunk; any even number of MiB only when recover-heavy; 256 KiB and
    64 KiB chunks left packed (profiles/r02_layout_sweep.log)."""
    M = 1 << 20
    assert nxec.batch_layout(14, M) == (M, 14 * M)
    assert nxec.batch_layout(14, M, 1) == (M, 15 * M)
    assert nxec.batch_layout(16, M) == (M, 17 * M)
    assert nxec.batch_layout(20, M) == (M, 20 * M)
    assert nxec.batch_layout(20, M, 1) == (M, 21 * M)
    assert nxec.batch_layout(20, 256 << 10) == (256 << 10, 20 * (256 << 10))
    assert nxec.batch_layout(15, M, 1) == (M, 15 * M)  # already odd
    cs, ss = nxec.batch_layout(20, 4 * M)
    assert cs == 4 * M + 2048 and ss == 20 * cs
    for n, ln in [(14, M), (16, M), (20, 4 * M), (6, 3 * M + 5), (4, 2 * M)]:
        for fl in (0, 1):
            cs, ss = nxec.batch_layout(n, ln, fl)
            assert cs >= ln and ss >= n * cs and cs % 16 == 0 and ss % 16 == 0
