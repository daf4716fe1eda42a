"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU oracle (nxec_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; it is the checker, never the thing measured or shipped.

Parity pinning: tests/test_oracle_golden.py checks every function here
against tests/golden/golden.json, produced by the reference ISA-L 2.22 code
(oracle/build_ref.sh + oracle/gen_golden.c).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libisal_base.so")

if not os.path.exists(LIB):
    raise ImportError(f"{LIB} missing; run `make oracle/liboracle.so`")

_o = C.CDLL(LIB)
vp = C.c_void_p
_o.orc_gf_mul.restype = C.c_ubyte
_o.orc_gf_mul.argtypes = [C.c_ubyte, C.c_ubyte]
_o.orc_gf_inv.restype = C.c_ubyte
_o.orc_gf_inv.argtypes = [C.c_ubyte]
_o.orc_gen_rs_matrix.argtypes = [vp, C.c_int, C.c_int]
_o.orc_invert_matrix.restype = C.c_int
_o.orc_invert_matrix.argtypes = [vp, vp, C.c_int]
_o.orc_init_tables.argtypes = [C.c_int, C.c_int, vp, vp]
_o.orc_encode_data.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp]
_o.orc_matmul.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp]
_o.orc_rs_encode.restype = C.c_int
_o.orc_rs_encode.argtypes = [C.c_int, C.c_int, vp, C.c_int64, vp]
_o.orc_rs_pre_decode.restype = C.c_int
_o.orc_rs_pre_decode.argtypes = [C.c_int, C.c_int, vp, C.c_int, C.c_int, vp, C.POINTER(C.c_int),
                                 C.POINTER(C.c_int), vp]
_o.orc_rs_decode.restype = C.c_int
_o.orc_rs_decode.argtypes = [C.c_int, C.c_int, vp, C.c_int, vp, C.c_int64, C.c_int, vp, C.c_int, C.c_int, vp,
                             C.POINTER(C.c_int)]
_o.orc_coding_utils_encode.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, vp]
_o.orc_fill_bytes.argtypes = [vp, C.c_int64, C.c_uint64]
_o.orc_time_encode.restype = C.c_double
_o.orc_time_encode.argtypes = [C.c_int, C.c_int, vp, vp, vp, C.c_int64, C.c_int64, C.c_int]


def _p(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def gf_mul(a: int, b: int) -> int:
    return int(_o.orc_gf_mul(a, b))


def gf_inv(a: int) -> int:
    return int(_o.orc_gf_inv(a))


def gen_rs_matrix(n: int, k: int) -> np.ndarray:
    a = np.zeros((n, k), dtype=np.uint8)
    _o.orc_gen_rs_matrix(_p(a), n, k)
    return a


def invert_matrix(m: np.ndarray):
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros_like(m)
    rc = _o.orc_invert_matrix(_p(m), _p(out), m.shape[0])
    return rc, out


def init_tables(coeffs: np.ndarray) -> np.ndarray:
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape
    out = np.zeros(rows * k * 32, dtype=np.uint8)
    _o.orc_init_tables(k, rows, _p(c), _p(out))
    return out


def fill_bytes(nbytes: int, seed: int) -> np.ndarray:
    out = np.zeros(nbytes, dtype=np.uint8)
    _o.orc_fill_bytes(_p(out), nbytes, C.c_uint64(seed))
    return out


_o.orc_fill_bytes_at.argtypes = [vp, C.c_int64, C.c_uint64, C.c_int64]


def fill_bytes_at(out: np.ndarray, seed: int, byte_off: int) -> np.ndarray:
    """Bytes [byte_off, byte_off + out.nbytes) of fill_bytes(., seed) into `out`
    (byte_off a multiple of 8)."""
    assert byte_off % 8 == 0 and out.dtype == np.uint8 and out.flags["C_CONTIGUOUS"]
    _o.orc_fill_bytes_at(_p(out), out.nbytes, C.c_uint64(seed), byte_off // 8)
    return out


def matmul(coeffs: np.ndarray, srcs: Sequence[np.ndarray]) -> List[np.ndarray]:
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape
    n = len(srcs[0])
    ins = [np.ascontiguousarray(s, dtype=np.uint8) for s in srcs]
    outs = [np.zeros(n, dtype=np.uint8) for _ in range(rows)]
    _o.orc_matmul(n, k, rows, _p(c), (vp * k)(*[s.ctypes.data for s in ins]),
                  (vp * rows)(*[o.ctypes.data for o in outs]))
    return outs


_o.orc_simd_level.restype = C.c_int
_o.orc_simd_encode.restype = C.c_int
_o.orc_simd_encode.argtypes = [C.c_int, C.c_size_t, C.c_int, C.c_int, vp, vp, vp]


_o.orc_simd_rscode_encode_range.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp]
_o.orc_simd_rscode_decode_range.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, vp, vp,
                                            C.c_int, vp, vp]


def simd_rscode_encode_range(level: int, n: int, k: int, cs: int, lo: int, hi: int, data: np.ndarray,
                             chunks: np.ndarray, parity_rows: np.ndarray) -> None:
    """RSCode::encode (rs.cc:57-92) for stripes [lo, hi): copy data [s][k][cs] into
    the stripe's chunks [s][n][cs] (rs.cc:80), then SIMD-encode the parity."""
    pr = np.ascontiguousarray(parity_rows, dtype=np.uint8)
    _o.orc_simd_rscode_encode_range(level, n, k, cs, lo, hi, _p(data), _p(chunks), _p(pr))


def simd_rscode_decode_range(level: int, n: int, k: int, cs: int, lo: int, hi: int, chunks: np.ndarray,
                             ids: Sequence[int], matrix: np.ndarray, out: np.ndarray) -> None:
    """rows x k matrix over chunks `ids` of stripes [lo, hi) -> out [s][rows][cs]."""
    m = np.ascontiguousarray(matrix, dtype=np.uint8)
    i = np.asarray(list(ids), dtype=np.int32)
    _o.orc_simd_rscode_decode_range(level, n, k, cs, lo, hi, _p(chunks), _p(i), m.shape[0], _p(m), _p(out))


def simd_level() -> int:
    """512 (AVX-512BW), 256 (AVX2) or 0: the CPU-baseline SIMD path this host runs."""
    return _o.orc_simd_level()


def simd_encode(coeffs: np.ndarray, srcs: Sequence[np.ndarray], outs: Sequence[np.ndarray], level: int = -1) -> int:
    """CPU baseline stand-in for ISA-L's SIMD ec_encode_data (nxec_cpu_simd.c):
    outs[r] = sum_j coeffs[r, j] * srcs[j].  Writes into `outs`; returns the level used."""
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape
    return _o.orc_simd_encode(level, len(srcs[0]), k, rows, _p(c), (vp * k)(*[s.ctypes.data for s in srcs]),
                              (vp * rows)(*[o.ctypes.data for o in outs]))


def encode_data(gftbls: np.ndarray, k: int, rows: int, srcs: Sequence[np.ndarray]) -> List[np.ndarray]:
    n = len(srcs[0])
    t = np.ascontiguousarray(gftbls, dtype=np.uint8)
    ins = [np.ascontiguousarray(s, dtype=np.uint8) for s in srcs]
    outs = [np.zeros(n, dtype=np.uint8) for _ in range(rows)]
    _o.orc_encode_data(n, k, rows, _p(t), (vp * k)(*[s.ctypes.data for s in ins]),
                       (vp * rows)(*[o.ctypes.data for o in outs]))
    return outs


def rs_encode(n: int, k: int, data: np.ndarray, cs: int) -> np.ndarray:
    """RSCode::encode -> n x cs stripe."""
    d = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.zeros(n * cs, dtype=np.uint8)
    assert _o.orc_rs_encode(n, k, _p(d), cs, _p(out)) == 1
    return out.reshape(n, cs)


def rs_pre_decode(n: int, k: int, failed: Sequence[int], is_repair: bool):
    f = np.asarray(list(failed) + [0], dtype=np.int32)
    ids = np.zeros(n, dtype=np.int32)
    ni, mi = C.c_int(0), C.c_int(0)
    rm = np.zeros(max(1, len(failed)) * k, dtype=np.uint8)
    ok = _o.orc_rs_pre_decode(n, k, _p(f), len(failed), int(is_repair), _p(ids), C.byref(ni), C.byref(mi), _p(rm))
    return ok, ids[: ni.value].tolist(), mi.value, rm[: len(failed) * k].reshape(len(failed), k)


def rs_decode(n: int, k: int, input_ids: Sequence[int], inputs: Sequence[np.ndarray], is_repair: bool = False,
              targets: Optional[Sequence[int]] = None, use_car: bool = False):
    cs = len(inputs[0]) if inputs else 0
    ids = np.asarray(list(input_ids) + [0], dtype=np.int32)
    tg = np.asarray(list(targets or []) + [0], dtype=np.int32)
    ins = [np.ascontiguousarray(s, dtype=np.uint8) for s in inputs]
    out = np.zeros(max(n, 1) * max(cs, 1), dtype=np.uint8)
    nt = C.c_int(0)
    ok = _o.orc_rs_decode(n, k, _p(ids), len(inputs), (vp * max(1, len(ins)))(*[s.ctypes.data for s in ins]), cs,
                          int(is_repair), _p(tg), len(targets or []), int(use_car), _p(out), C.byref(nt))
    return ok, out[: nt.value * cs].reshape(nt.value, cs)


def time_encode(k: int, rows: int, coeffs: np.ndarray, src: np.ndarray, dst: np.ndarray, cs: int, nstripes: int,
                threads: int) -> float:
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    return float(_o.orc_time_encode(k, rows, _p(c), _p(src), _p(dst), cs, nstripes, threads))


def ref_available() -> bool:
    return os.path.exists(REF_LIB)


class RefISAL:
    """The reference ISA-L 2.22 base-C library built by build_ref.sh (oracle/_ref).

    Used as the `kind: reference` CPU baseline and to cross-check the oracle."""

    def __init__(self):
        self.lib = C.CDLL(REF_LIB)
        self.lib.ec_init_tables.argtypes = [C.c_int, C.c_int, vp, vp]
        self.lib.ec_encode_data.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp]
        self.lib.gf_gen_rs_matrix.argtypes = [vp, C.c_int, C.c_int]

    def encode(self, coeffs: np.ndarray, srcs: Sequence[np.ndarray], outs: Sequence[np.ndarray]) -> None:
        c = np.ascontiguousarray(coeffs, dtype=np.uint8)
        rows, k = c.shape
        t = np.zeros(rows * k * 32, dtype=np.uint8)
        self.lib.ec_init_tables(k, rows, _p(c), _p(t))
        self.lib.ec_encode_data(len(srcs[0]), k, rows, _p(t), (vp * k)(*[s.ctypes.data for s in srcs]),
                                (vp * rows)(*[o.ctypes.data for o in outs]))
