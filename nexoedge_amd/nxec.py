"""Python view of the C ABI (include/nxec.h) for tests, benchmarks and tools.

Everything here is plumbing around libnxec: device buffers, contexts and the
RS entry points.  The coding arithmetic itself only exists in the gfx950
kernels; host-side helpers below are the planning math (matrices), which the
reference also runs on the host (rs.cc:26,196,219,290,316).
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import NXEC_OK, AgentReq, NxecError, check, lib


def _u8(a: np.ndarray) -> C.c_void_p:
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


def _i32(v: Optional[Iterable[int]]):
    if v is None:
        return None, None
    arr = np.ascontiguousarray(np.asarray(list(v), dtype=np.int32))
    return arr, C.c_void_p(arr.ctypes.data)


# ---------------------------------------------------------------- host math
def gf_mul(a: int, b: int) -> int:
    return int(lib.nxec_gf_mul(a, b))


def gf_inv(a: int) -> int:
    return int(lib.nxec_gf_inv(a))


def gen_rs_matrix(n: int, k: int) -> np.ndarray:
    """ISA-L gf_gen_rs_matrix (rs.cc:26): n x k, identity on top."""
    a = np.zeros((n, k), dtype=np.uint8)
    lib.nxec_gf_gen_rs_matrix(_u8(a), n, k)
    return a


def invert_matrix(m: np.ndarray) -> Optional[np.ndarray]:
    src = np.ascontiguousarray(m, dtype=np.uint8).copy()
    n = src.shape[0]
    out = np.zeros((n, n), dtype=np.uint8)
    rc = lib.nxec_gf_invert_matrix(_u8(src), _u8(out), n)
    return None if rc != 0 else out


def init_tables(coeffs: np.ndarray) -> np.ndarray:
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape
    out = np.zeros(rows * k * 32, dtype=np.uint8)
    lib.nxec_ec_init_tables(k, rows, _u8(c), _u8(out))
    return out


def rs_plan(n: int, k: int, failed: Sequence[int], is_repair: bool):
    """RSCode::preDecode (rs.cc:238-322) -> (input_ids, min_inputs, repair_matrix|None)."""
    f, fp = _i32(failed)
    ids = np.zeros(n, dtype=np.int32)
    ni, mi = C.c_int(0), C.c_int(0)
    rm = np.zeros((max(len(failed), 1), k), dtype=np.uint8)
    rc = lib.nxec_rs_plan(n, k, fp, len(failed), 1 if is_repair else 0, C.c_void_p(ids.ctypes.data), C.byref(ni),
                          C.byref(mi), _u8(rm))
    check(rc, "nxec_rs_plan")
    return ids[: ni.value].tolist(), mi.value, (rm[: len(failed)] if is_repair else None)


def decode_matrix(n: int, k: int, input_ids: Sequence[int], targets: Sequence[int]) -> np.ndarray:
    a, ap = _i32(input_ids)
    t, tp = _i32(targets)
    out = np.zeros((max(len(targets), 1), k), dtype=np.uint8)
    check(lib.nxec_rs_decode_matrix(n, k, ap, tp, len(targets), _u8(out)), "nxec_rs_decode_matrix")
    return out[: len(targets)]


LAYOUT_RECOVER_HEAVY = 1
OBJECTS_TAIL_INPLACE = 1  # nxec_encode_objects_ex: only the partial last-stripe chunk to the tail arena
OBJECTS_ASYNC = 2  # nxec_encode_objects_ex: return once queued on the stream


def batch_layout(n: int, length: int, flags: int = 0):
    """(chunk_stride, stripe_stride) of the library's recommended batch layout (nxec_batch_layout)."""
    c, st = C.c_int64(), C.c_int64()
    check(lib.nxec_batch_layout(n, length, flags, C.byref(c), C.byref(st)), "nxec_batch_layout")
    return c.value, st.value


def _groups(groups: Sequence[Sequence[int]]):
    offs = [0]
    flat = []
    for g in groups:
        flat.extend(int(c) for c in g)
        offs.append(len(flat))
    o, op = _i32(offs)
    c, cp = _i32(flat if flat else [0])
    return (o, c), op, cp


def object_layout(n: int, k: int, length: int, max_chunk_size: int):
    """(nstripes, full_stripes, last_chunk_size) of an object (nxec_object_layout)."""
    ns, nf, cl = C.c_int64(), C.c_int64(), C.c_int64()
    check(lib.nxec_object_layout(n, k, length, max_chunk_size, C.byref(ns), C.byref(nf), C.byref(cl)),
          "nxec_object_layout")
    return ns.value, nf.value, cl.value


def objects_layout(n: int, k: int, lengths: Sequence[int], max_chunk_size: int):
    """(total_stripes, tail_bytes) of a multi-object batch (nxec_objects_layout)."""
    ln = np.ascontiguousarray(np.asarray(list(lengths), dtype=np.int64))
    ts, tb = C.c_int64(), C.c_int64()
    check(lib.nxec_objects_layout(n, k, len(ln), C.c_void_p(ln.ctypes.data), max_chunk_size, C.byref(ts),
                                  C.byref(tb)), "nxec_objects_layout")
    return ts.value, tb.value


def car_plan(n: int, k: int, failed: int, groups: Sequence[Sequence[int]]):
    """CAR repair plan (chunk_manager.cc:929-986) -> list of (chunk_ids, coeffs) per agent sub-group."""
    keep, op, cp = _groups(groups)
    so = np.zeros(len(groups) + 2, dtype=np.int32)
    sc = np.zeros(k, dtype=np.int32)
    cf = np.zeros(k, dtype=np.uint8)
    ns = C.c_int(0)
    check(lib.nxec_car_plan(n, k, failed, op, cp, len(groups), C.c_void_p(so.ctypes.data), C.c_void_p(sc.ctypes.data),
                            _u8(cf), C.byref(ns)), "nxec_car_plan")
    return [(sc[so[g]:so[g + 1]].tolist(), cf[so[g]:so[g + 1]].copy()) for g in range(ns.value)]


# ------------------------------------------------------- host-buffer encode
def encode_host(coeffs: np.ndarray, data: Sequence[np.ndarray]) -> list:
    """CodingUtils::encode / ec_encode_data on host buffers (GPU-executed)."""
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape
    n = len(data[0]) if data else 0
    ins = [np.ascontiguousarray(d, dtype=np.uint8) for d in data]
    outs = [np.zeros(n, dtype=np.uint8) for _ in range(rows)]
    inp = (C.c_void_p * k)(*[d.ctypes.data for d in ins])
    outp = (C.c_void_p * rows)(*[o.ctypes.data for o in outs])
    check(lib.nxec_encode_host(n, k, rows, _u8(c), inp, outp), "nxec_encode_host")
    return outs


def encode_host_md5(coeffs: np.ndarray, data: Sequence, outs: Optional[Sequence] = None, hash_inputs: bool = True):
    """nxec_encode_host_md5: encode_host plus the MD5 of the inputs (when
    hash_inputs) and outputs from the same GPU pass.  data / outs may be numpy
    arrays or (address, length) pairs of host memory (e.g. arena blocks).
    Returns (outputs, input digests (k x 16) or None, output digests (rows x 16))."""
    c = np.ascontiguousarray(coeffs, dtype=np.uint8)
    rows, k = c.shape

    def addr(a):
        return (int(a[0]), int(a[1])) if isinstance(a, tuple) else (a.ctypes.data, len(a))

    ins = [a if isinstance(a, tuple) else np.ascontiguousarray(a, dtype=np.uint8) for a in data]
    n = addr(ins[0])[1] if ins else 0
    if outs is None:
        outs = [np.zeros(n, dtype=np.uint8) for _ in range(rows)]
    md5_in = np.zeros((k, 16), dtype=np.uint8) if hash_inputs else None
    md5_out = np.zeros((rows, 16), dtype=np.uint8)
    inp = (C.c_void_p * k)(*[addr(d)[0] for d in ins])
    outp = (C.c_void_p * rows)(*[addr(o)[0] for o in outs])
    check(lib.nxec_encode_host_md5(n, k, rows, _u8(c), inp, outp,
                                   _u8(md5_in) if md5_in is not None else None, _u8(md5_out)),
          "nxec_encode_host_md5")
    return outs, md5_in, md5_out


def ec_encode_data(gftbls: np.ndarray, k: int, rows: int, data: Sequence[np.ndarray]) -> list:
    """Drop-in ISA-L signature: coefficients come from 32-byte tables."""
    t = np.ascontiguousarray(gftbls, dtype=np.uint8)
    n = len(data[0])
    ins = [np.ascontiguousarray(d, dtype=np.uint8) for d in data]
    outs = [np.zeros(n, dtype=np.uint8) for _ in range(rows)]
    inp = (C.c_void_p * k)(*[d.ctypes.data for d in ins])
    outp = (C.c_void_p * rows)(*[o.ctypes.data for o in outs])
    check(lib.nxec_ec_encode_data_status(n, k, rows, _u8(t), inp, outp), "nxec_ec_encode_data")
    return outs


# ------------------------------------------------------------- device side
def storage_classes(path: str) -> list:
    """nxec_storage_classes_load: the classes of a storage_class.ini in file order, as dicts
    (Config's reading, src/common/config.cc:267-282, :664-705)."""
    count = C.c_int()
    check(lib.nxec_storage_classes_load(path.encode(), None, 0, C.byref(count)), "nxec_storage_classes_load")
    arr = (_lib.StorageClass * max(count.value, 1))()
    check(lib.nxec_storage_classes_load(path.encode(), arr, len(arr), C.byref(count)), "nxec_storage_classes_load")
    return [{"name": c.name.decode(), "coding": "rs" if c.coding == 0 else "unknown", "n": c.n, "k": c.k, "f": c.f,
             "max_chunk_size": c.max_chunk_size, "default": bool(c.is_default)} for c in arr[:count.value]]


def proxy_repair_using_car(path: str) -> bool:
    """nxec_proxy_repair_using_car: misc.repair_using_car of a proxy.ini (config.cc:320)."""
    car = C.c_int()
    check(lib.nxec_proxy_repair_using_car(path.encode(), C.byref(car)), "nxec_proxy_repair_using_car")
    return bool(car.value)


def design_probes() -> bool:
    """True when libnxec carries the design-probe kernels (make PROBES=1)."""
    return bool(lib.nxec_design_probes())


def device_count() -> int:
    c = C.c_int(0)
    rc = lib.nxec_device_count(C.byref(c))
    return c.value if rc == NXEC_OK else 0


def device_info(dev: int = 0) -> dict:
    name = C.create_string_buffer(64)
    cus = C.c_int(0)
    mem = C.c_int64(0)
    check(lib.nxec_device_info(dev, name, 64, C.byref(cus), C.byref(mem)), "nxec_device_info")
    return {"arch": name.value.decode(), "cus": cus.value, "mem": mem.value}


def default_devices(devices=None) -> None:
    """nxec_default_devices: the default pool of the drop-in entry points.
    None: one context per visible device (the default); "current": the
    calling thread's current device; a list: those devices, one context per
    entry (duplicates allowed)."""
    if devices is None:
        check(lib.nxec_default_devices(None, 0), "nxec_default_devices")
    elif devices == "current":
        check(lib.nxec_default_devices(None, -1), "nxec_default_devices")
    else:
        arr = (C.c_int * len(devices))(*[int(d) for d in devices])
        check(lib.nxec_default_devices(arr, len(devices)), "nxec_default_devices")


def default_pool_stats() -> list:
    """[{device, node, calls, inflight}] per member of the default pool."""
    cnt = C.c_int()
    check(lib.nxec_default_pool_stats(None, None, None, None, 0, C.byref(cnt)), "nxec_default_pool_stats")
    n = cnt.value
    dv, nd, inf = (C.c_int * max(n, 1))(), (C.c_int * max(n, 1))(), (C.c_int * max(n, 1))()
    calls = (C.c_ulonglong * max(n, 1))()
    check(lib.nxec_default_pool_stats(dv, nd, calls, inf, n, C.byref(cnt)), "nxec_default_pool_stats")
    return [{"device": dv[i], "node": nd[i], "calls": calls[i], "inflight": inf[i]} for i in range(min(n, cnt.value))]


def default_admission(device: int = 0, reset: bool = False) -> dict:
    """nxec_default_admission: the device's admission gate of the default
    pool -- {limit, running, peak, waited}; reset restarts peak and waited."""
    lim, run, peak = C.c_int(), C.c_int(), C.c_int()
    waited = C.c_ulonglong()
    check(lib.nxec_default_admission(int(device), C.byref(lim), C.byref(run), C.byref(peak), C.byref(waited),
                                     int(bool(reset))), "nxec_default_admission")
    return {"limit": lim.value, "running": run.value, "peak": peak.value, "waited": waited.value}


def default_pick(inflight: Sequence[int], nodes: Optional[Sequence[int]] = None, caller_node: int = -1,
                 prev: int = -1) -> int:
    """nxec_default_pick: the member the default pool leases for one call."""
    n = len(inflight)
    inf = (C.c_int * n)(*inflight)
    nd = (C.c_int * n)(*nodes) if nodes is not None else None
    r = lib.nxec_default_pick(n, inf, nd, int(caller_node), int(prev))
    if r < 0:
        check(r, "nxec_default_pick")
    return r


def set_device(dev: int) -> None:
    """nxec_set_device: make `dev` the calling thread's current device (its
    allocations, e.g. DeviceBuffer, land there)."""
    check(lib.nxec_set_device(int(dev)), "nxec_set_device")


def device_sync() -> None:
    check(lib.nxec_device_sync(), "nxec_device_sync")


def bind_thread_numa(device: int) -> int:
    """Binds the calling thread (and threads it starts later) to the CPUs of
    the NUMA node of GPU `device` (nxec_bind_thread_to_device); returns the
    node, -1 when unknown (affinity unchanged)."""
    node = C.c_int(-1)
    check(lib.nxec_bind_thread_to_device(device, C.byref(node)), "nxec_bind_thread_to_device")
    return node.value


def pci_numa_node(bus_id: str) -> int:
    node = C.c_int(-1)
    check(lib.nxec_pci_numa_node(bus_id.encode(), C.byref(node)), "nxec_pci_numa_node")
    return node.value


def numa_node_cpus(node: int) -> list:
    cnt = C.c_int(0)
    check(lib.nxec_numa_node_cpus(node, None, 0, C.byref(cnt)), "nxec_numa_node_cpus")
    arr = (C.c_int * max(cnt.value, 1))()
    check(lib.nxec_numa_node_cpus(node, arr, cnt.value, C.byref(cnt)), "nxec_numa_node_cpus")
    return list(arr[:cnt.value])


def bind_thread_pci(bus_id: str) -> int:
    node = C.c_int(-1)
    check(lib.nxec_bind_thread_to_pci(bus_id.encode(), C.byref(node)), "nxec_bind_thread_to_pci")
    return node.value


class DeviceBuffer:
    """Raw device allocation (hipMalloc) with host copy helpers."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(lib.nxec_dev_malloc(C.byref(p), max(self.nbytes, 1)), "nxec_dev_malloc")
        self.ptr = p.value

    def __int__(self):
        return self.ptr

    def addr(self, offset: int = 0) -> C.c_void_p:
        return C.c_void_p(self.ptr + offset)

    def upload(self, arr: np.ndarray, offset: int = 0, stream=None) -> None:
        a = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        assert offset + a.nbytes <= self.nbytes
        check(lib.nxec_memcpy_h2d(self.addr(offset), C.c_void_p(a.ctypes.data), a.nbytes, stream), "h2d")
        check(lib.nxec_stream_sync(stream), "sync")

    def download(self, nbytes: Optional[int] = None, offset: int = 0, stream=None) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, dtype=np.uint8)
        check(lib.nxec_memcpy_d2h(C.c_void_p(out.ctypes.data), self.addr(offset), n, stream), "d2h")
        check(lib.nxec_stream_sync(stream), "sync")
        return out

    def fill_random(self, seed: int, nbytes: Optional[int] = None, offset: int = 0, stream=None) -> None:
        n = self.nbytes - offset if nbytes is None else nbytes
        check(lib.nxec_fill_random(self.addr(offset), n, C.c_uint64(seed), stream), "fill")
        check(lib.nxec_stream_sync(stream), "sync")

    def memset(self, value: int, nbytes: Optional[int] = None, offset: int = 0, stream=None) -> None:
        n = self.nbytes - offset if nbytes is None else nbytes
        check(lib.nxec_memset(self.addr(offset), value, n, stream), "memset")
        check(lib.nxec_stream_sync(stream), "sync")

    def memset2d(self, value: int, offset: int, pitch: int, width: int, height: int, stream=None) -> None:
        """Asynchronous: `height` rows of `width` bytes, `pitch` apart, from `offset` (hipMemset2DAsync)."""
        assert offset + (height - 1) * pitch + width <= self.nbytes if height else True
        check(lib.nxec_memset2d(self.addr(offset), pitch, value, width, height, stream), "memset2d")

    def copy_within(self, dst_offset: int, src_offset: int, nbytes: int, stream=None) -> None:
        """Asynchronous device-to-device copy inside this buffer (hipMemcpyAsync)."""
        assert max(dst_offset, src_offset) + nbytes <= self.nbytes
        check(lib.nxec_memcpy_d2d(self.addr(dst_offset), self.addr(src_offset), nbytes, stream), "d2d")

    def checksum(self, nbytes: Optional[int] = None, offset: int = 0, stream=None) -> int:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = C.c_uint64(0)
        check(lib.nxec_checksum(self.addr(offset), n, C.byref(out), stream), "checksum")
        return out.value

    def free(self) -> None:
        if self.ptr:
            lib.nxec_dev_free(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """hipHostMalloc'd host memory exposed as a numpy uint8 array."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib.nxec_host_malloc_pinned(C.byref(p), max(int(nbytes), 1)), "nxec_host_malloc_pinned")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_ubyte * max(self.nbytes, 1)).from_address(self.ptr))[: self.nbytes]

    def free(self) -> None:
        if self.ptr:
            self.array = None
            lib.nxec_host_free_pinned(C.c_void_p(self.ptr))
            self.ptr = 0


class Event:
    def __init__(self):
        p = C.c_void_p()
        check(lib.nxec_event_create(C.byref(p)), "nxec_event_create")
        self.ptr = p.value

    def record(self, stream=None) -> None:
        check(lib.nxec_event_record(C.c_void_p(self.ptr), stream), "nxec_event_record")

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float(0)
        check(lib.nxec_event_elapsed_ms(C.c_void_p(self.ptr), C.c_void_p(end.ptr), C.byref(ms)), "elapsed")
        return float(ms.value)


class Request:
    """Handle of an asynchronous frame copy (nxec_request_t)."""

    def __init__(self, handle: C.c_void_p):
        self._h = handle

    def wait(self) -> None:
        h, self._h = self._h, None
        if h is not None:
            check(lib.nxec_request_wait(h), "nxec_request_wait")

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            lib.nxec_request_wait(self._h)


class Context:
    """An nxec_ctx_t bound to one device: stream + staging pools."""

    def __init__(self, device: int = 0):
        p = C.c_void_p()
        check(lib.nxec_ctx_create(device, C.byref(p)), "nxec_ctx_create")
        self.ptr = p.value
        self.device = device

    @property
    def stream(self) -> C.c_void_p:
        return C.c_void_p(lib.nxec_ctx_stream(C.c_void_p(self.ptr)))

    def sync(self) -> None:
        check(lib.nxec_stream_sync(self.stream), "nxec_stream_sync")

    def stripes_mul(self, coeffs: np.ndarray, src: int, dst: int, *, src_idx=None, dst_idx=None, copy_idx=None,
                    src_chunk_stride: int, src_stripe_stride: int, dst_chunk_stride: int, dst_stripe_stride: int,
                    length: int, nstripes: int, stream=None) -> None:
        c = np.ascontiguousarray(coeffs, dtype=np.uint8)
        rows, k = c.shape
        si, sip = _i32(src_idx)
        di, dip = _i32(dst_idx)
        ci, cip = _i32(copy_idx)
        rc = lib.nxec_stripes_mul(C.c_void_p(self.ptr), rows, k, _u8(c), C.c_void_p(int(src)), sip,
                                  src_chunk_stride, src_stripe_stride, C.c_void_p(int(dst)), dip, dst_chunk_stride,
                                  dst_stripe_stride, cip, length, nstripes, stream)
        check(rc, "nxec_stripes_mul")

    def stripes_mul_ptrs(self, coeffs: np.ndarray, src_ptrs: int, dst_ptrs: int, length: int, nstripes: int,
                         stream=None) -> None:
        c = np.ascontiguousarray(coeffs, dtype=np.uint8)
        rows, k = c.shape
        rc = lib.nxec_stripes_mul_ptrs(C.c_void_p(self.ptr), rows, k, _u8(c), C.c_void_p(int(src_ptrs)),
                                       C.c_void_p(int(dst_ptrs)), length, nstripes, stream)
        check(rc, "nxec_stripes_mul_ptrs")

    def rs_encode(self, n: int, k: int, stripes: int, chunk_stride: int, stripe_stride: int, length: int,
                  nstripes: int, stream=None) -> None:
        check(lib.nxec_rs_encode_stripes(C.c_void_p(self.ptr), n, k, C.c_void_p(int(stripes)), chunk_stride,
                                         stripe_stride, length, nstripes, stream), "nxec_rs_encode_stripes")

    def rs_recover(self, n: int, k: int, failed: Sequence[int], stripes: int, chunk_stride: int,
                   stripe_stride: int, length: int, nstripes: int, stream=None) -> None:
        f, fp = _i32(failed)
        check(lib.nxec_rs_recover_stripes(C.c_void_p(self.ptr), n, k, fp, len(failed), C.c_void_p(int(stripes)),
                                          chunk_stride, stripe_stride, length, nstripes, stream),
              "nxec_rs_recover_stripes")

    def rs_decode(self, n: int, k: int, failed: Sequence[int], stripes: int, chunk_stride: int, stripe_stride: int,
                  out: int, out_chunk_stride: int, out_stripe_stride: int, length: int, nstripes: int,
                  stream=None) -> None:
        f, fp = _i32(failed)
        check(lib.nxec_rs_decode_stripes(C.c_void_p(self.ptr), n, k, fp, len(failed), C.c_void_p(int(stripes)),
                                         chunk_stride, stripe_stride, C.c_void_p(int(out)), out_chunk_stride,
                                         out_stripe_stride, length, nstripes, stream), "nxec_rs_decode_stripes")

    def rs_car_repair(self, n: int, k: int, failed: int, groups, stripes: int, chunk_stride: int, stripe_stride: int,
                      partials: int, partial_chunk_stride: int, partial_stripe_stride: int, length: int, nstripes: int,
                      stream=None) -> None:
        keep, op, cp = _groups(groups)
        check(lib.nxec_rs_car_repair_stripes(C.c_void_p(self.ptr), n, k, failed, op, cp, len(groups),
                                             C.c_void_p(int(stripes)), chunk_stride, stripe_stride,
                                             C.c_void_p(int(partials)), partial_chunk_stride, partial_stripe_stride, length,
                                             nstripes, stream),
              "nxec_rs_car_repair_stripes")

    def md5_chunks(self, base: int, chunk_stride: int, stripe_stride: int, nchunks: int, length: int, nstripes: int,
                   digests: int, stream=None) -> None:
        check(lib.nxec_md5_chunks(C.c_void_p(self.ptr), C.c_void_p(int(base)), chunk_stride, stripe_stride, nchunks,
                                  length, nstripes, C.c_void_p(int(digests)), stream), "nxec_md5_chunks")

    def rs_encode_md5(self, n: int, k: int, stripes: int, chunk_stride: int, stripe_stride: int, length: int,
                      nstripes: int, digests: int, stream=None) -> None:
        """nxec_rs_encode_md5_stripes: parity + MD5 of all n chunks per stripe (digests [s][n][16])."""
        check(lib.nxec_rs_encode_md5_stripes(C.c_void_p(self.ptr), n, k, C.c_void_p(int(stripes)), chunk_stride,
                                             stripe_stride, length, nstripes, C.c_void_p(int(digests)), stream),
              "nxec_rs_encode_md5_stripes")

    def rs_recover_md5(self, n: int, k: int, failed: Sequence[int], stripes: int, chunk_stride: int,
                       stripe_stride: int, length: int, nstripes: int, digests: int, stream=None) -> None:
        """nxec_rs_recover_md5_stripes: rebuild `failed` in place + MD5 of each rebuilt chunk ([s][nfailed][16])."""
        f, fp = _i32(failed)
        check(lib.nxec_rs_recover_md5_stripes(C.c_void_p(self.ptr), n, k, fp, len(failed), C.c_void_p(int(stripes)),
                                              chunk_stride, stripe_stride, length, nstripes, C.c_void_p(int(digests)),
                                              stream), "nxec_rs_recover_md5_stripes")

    def md5_verify_chunks(self, base: int, chunk_stride: int, stripe_stride: int, nchunks: int, length: int,
                          nstripes: int, expected: int, ok: int, nbad=None, stream=None) -> None:
        check(lib.nxec_md5_verify_chunks(C.c_void_p(self.ptr), C.c_void_p(int(base)), chunk_stride, stripe_stride,
                                         nchunks, length, nstripes, C.c_void_p(int(expected)), C.c_void_p(int(ok)),
                                         C.c_void_p(int(nbad)) if nbad else None, stream), "nxec_md5_verify_chunks")

    def encode_object(self, n: int, k: int, obj: int, length: int, max_chunk_size: int, parity: int, tail=None,
                      md5=None, stream=None) -> None:
        check(lib.nxec_encode_object(C.c_void_p(self.ptr), n, k, C.c_void_p(int(obj)), length, max_chunk_size,
                                     C.c_void_p(int(parity)), C.c_void_p(int(tail) if tail else None),
                                     C.c_void_p(int(md5) if md5 else None), stream), "nxec_encode_object")

    def encode_objects(self, n: int, k: int, objects: Sequence[int], lengths: Sequence[int], max_chunk_size: int,
                       parity: int, tail=None, md5=None, stream=None, flags: int = 0) -> None:
        """nxec_encode_objects_ex; flags = OBJECTS_TAIL_INPLACE writes only each
        last stripe's partial data chunk to the tail arena, OBJECTS_ASYNC returns
        once the work is queued on the stream (include/nxec.h)."""
        ptrs = (C.c_void_p * max(len(objects), 1))(*[int(o) if o else None for o in objects])
        ln = np.ascontiguousarray(np.asarray(list(lengths), dtype=np.int64))
        check(lib.nxec_encode_objects_ex(C.c_void_p(self.ptr), n, k, len(ln), ptrs, C.c_void_p(ln.ctypes.data),
                                         max_chunk_size, C.c_void_p(int(parity)),
                                         C.c_void_p(int(tail) if tail else None),
                                         C.c_void_p(int(md5) if md5 else None), flags, stream), "nxec_encode_objects")

    def kernel_timing(self, enable: bool = True) -> None:
        """nxec_kernel_timing: event-time the coding launches of encode_objects (totals reset)."""
        check(lib.nxec_kernel_timing(C.c_void_p(self.ptr), int(enable)), "nxec_kernel_timing")

    def kernel_time(self):
        """nxec_kernel_time: (milliseconds, launches) since kernel_timing()."""
        ms, n = C.c_double(), C.c_int64()
        check(lib.nxec_kernel_time(C.c_void_p(self.ptr), C.byref(ms), C.byref(n)), "nxec_kernel_time")
        return ms.value, n.value

    def encode_object_host(self, n: int, k: int, obj: int, length: int, max_chunk_size: int, parity: int,
                           md5=None, batch_stripes: int = 0) -> None:
        check(lib.nxec_encode_object_host(C.c_void_p(self.ptr), n, k, C.c_void_p(int(obj)), length, max_chunk_size,
                                          C.c_void_p(int(parity)), C.c_void_p(int(md5) if md5 else None),
                                          batch_stripes), "nxec_encode_object_host")

    def decode_object(self, n: int, k: int, failed: Sequence[int], chunks: int, length: int, max_chunk_size: int,
                      obj: int, tail=None, stream=None) -> None:
        f, fp = _i32(failed)
        check(lib.nxec_decode_object(C.c_void_p(self.ptr), n, k, fp, len(failed), C.c_void_p(int(chunks)), length,
                                     max_chunk_size, C.c_void_p(int(obj)), C.c_void_p(int(tail) if tail else None),
                                     stream), "nxec_decode_object")

    def decode_object_ex(self, n: int, k: int, failed: Sequence[int], chunks: int, chunk_stride: int,
                         stripe_stride: int, length: int, max_chunk_size: int, obj: int, tail=None, stream=None) -> None:
        f, fp = _i32(failed)
        check(lib.nxec_decode_object_ex(C.c_void_p(self.ptr), n, k, fp, len(failed), C.c_void_p(int(chunks)),
                                        chunk_stride, stripe_stride, length, max_chunk_size, C.c_void_p(int(obj)),
                                        C.c_void_p(int(tail) if tail else None), stream), "nxec_decode_object_ex")

    def decode_object_verify(self, n: int, k: int, failed: Sequence[int], chunks: int, length: int,
                             max_chunk_size: int, md5: int, obj: int, tail, ok: int, nbad=None, stream=None) -> None:
        """nxec_decode_object_verify: decode_object + MD5 check of every chunk read (ok [ns][n] bytes)."""
        f, fp = _i32(failed)
        check(lib.nxec_decode_object_verify(C.c_void_p(self.ptr), n, k, fp, len(failed), C.c_void_p(int(chunks)),
                                            length, max_chunk_size, C.c_void_p(int(md5)), C.c_void_p(int(obj)),
                                            C.c_void_p(int(tail) if tail else None), C.c_void_p(int(ok)),
                                            C.c_void_p(int(nbad) if nbad else None), stream),
              "nxec_decode_object_verify")

    def agent_encode_batch(self, reqs, chunk_size: int, batch_bytes: int = 0) -> None:
        """nxec_agent_encode_batch: reqs = [(matrix (no x ni), inputs [ni arrays], outputs [no arrays],
        md5 (no x 16 uint8 array) or None[, md5_inputs (ni x 16) or None])], host numpy buffers of
        chunk_size bytes."""
        keep = []
        arr = (AgentReq * max(len(reqs), 1))()
        for i, req in enumerate(reqs):
            m, ins, outs, md5 = req[:4]
            md5_in = req[4] if len(req) > 4 else None
            m = np.ascontiguousarray(m, dtype=np.uint8)
            ip = (C.c_void_p * len(ins))(*[a.ctypes.data for a in ins])
            op = (C.c_void_p * len(outs))(*[a.ctypes.data for a in outs])
            keep += [m, ip, op]
            arr[i] = AgentReq(len(ins), len(outs), m.ctypes.data, C.cast(ip, C.c_void_p), C.cast(op, C.c_void_p),
                              md5.ctypes.data if md5 is not None else None,
                              md5_in.ctypes.data if md5_in is not None else None)
        check(lib.nxec_agent_encode_batch(C.c_void_p(self.ptr), arr, len(reqs), chunk_size, batch_bytes),
              "nxec_agent_encode_batch")

    def rs_encode_host_batch(self, n: int, k: int, h_data: int, h_parity: int, length: int, nstripes: int,
                             batch_stripes: int = 0) -> None:
        check(lib.nxec_rs_encode_host_batch(C.c_void_p(self.ptr), n, k, C.c_void_p(int(h_data)),
                                            C.c_void_p(int(h_parity)), length, nstripes, batch_stripes),
              "nxec_rs_encode_host_batch")

    def gather_chunks(self, frames: Sequence[int], length: int, dst: int, dst_stride: int, stream=None) -> None:
        """nxec_gather_chunks: host frame addresses -> dst + i*dst_stride (device)."""
        fp = (C.c_void_p * max(len(frames), 1))(*[int(f) for f in frames])
        check(lib.nxec_gather_chunks(C.c_void_p(self.ptr), fp, len(frames), length, C.c_void_p(int(dst)), dst_stride,
                                     stream), "nxec_gather_chunks")

    def scatter_chunks(self, src: int, src_stride: int, frames: Sequence[int], length: int, stream=None) -> None:
        """nxec_scatter_chunks: src + i*src_stride (device) -> host frame addresses."""
        fp = (C.c_void_p * max(len(frames), 1))(*[int(f) for f in frames])
        check(lib.nxec_scatter_chunks(C.c_void_p(self.ptr), C.c_void_p(int(src)), src_stride, len(frames), length, fp,
                                      stream), "nxec_scatter_chunks")

    def gather_chunks_async(self, frames: Sequence[int], length: int, dst: int, dst_stride: int,
                            stream=None) -> "Request":
        """nxec_gather_chunks_async; wait() on the returned request."""
        fp = (C.c_void_p * max(len(frames), 1))(*[int(f) for f in frames])
        req = C.c_void_p()
        check(lib.nxec_gather_chunks_async(C.c_void_p(self.ptr), fp, len(frames), length, C.c_void_p(int(dst)),
                                           dst_stride, stream, C.byref(req)), "nxec_gather_chunks_async")
        return Request(req)

    def scatter_chunks_async(self, src: int, src_stride: int, frames: Sequence[int], length: int,
                             stream=None) -> "Request":
        """nxec_scatter_chunks_async; wait() on the returned request."""
        fp = (C.c_void_p * max(len(frames), 1))(*[int(f) for f in frames])
        req = C.c_void_p()
        check(lib.nxec_scatter_chunks_async(C.c_void_p(self.ptr), C.c_void_p(int(src)), src_stride, len(frames),
                                            length, fp, stream, C.byref(req)), "nxec_scatter_chunks_async")
        return Request(req)

    def rs_recover_frames(self, n: int, k: int, failed: Sequence[int], frames: Sequence[int], length: int,
                          nstripes: int) -> None:
        """nxec_rs_recover_frames: frames = nstripes*n host addresses ([s][c]; 0 = absent)."""
        f, fp = _i32(failed)
        tab = (C.c_void_p * max(len(frames), 1))(*[int(x) if x else None for x in frames])
        check(lib.nxec_rs_recover_frames(C.c_void_p(self.ptr), n, k, fp, len(failed), tab, length, nstripes),
              "nxec_rs_recover_frames")

    def batch_layout_tuned(self, n: int, k: int, length: int, flags: int = 0, budget_bytes: int = 0):
        """nxec_batch_layout_tuned: (chunk_stride, stripe_stride) measured on this device."""
        cs, ss = C.c_int64(), C.c_int64()
        check(lib.nxec_batch_layout_tuned(C.c_void_p(self.ptr), n, k, length, flags, budget_bytes, C.byref(cs),
                                          C.byref(ss)), "nxec_batch_layout_tuned")
        return int(cs.value), int(ss.value)

    def decode_frames(self, n: int, k: int, failed: Sequence[int], in_frames: Sequence[int],
                      out_frames: Sequence[int], length: int, nstripes: int, batch_stripes: int = 0) -> None:
        """nxec_decode_frames: in_frames = nstripes*n host addresses ([s][c]; 0 =
        absent), out_frames = nstripes*k ([s][j]): the pipelined read path."""
        f, fp = _i32(failed)
        tin = (C.c_void_p * max(len(in_frames), 1))(*[int(x) if x else None for x in in_frames])
        tout = (C.c_void_p * max(len(out_frames), 1))(*[int(x) if x else None for x in out_frames])
        check(lib.nxec_decode_frames(C.c_void_p(self.ptr), n, k, fp, len(failed), tin, tout, length, nstripes,
                                     batch_stripes), "nxec_decode_frames")

    def describe_launch(self, rows: int, k: int, length: int, nstripes: int) -> str:
        buf = C.create_string_buffer(512)
        check(lib.nxec_describe_launch(C.c_void_p(self.ptr), rows, k, length, nstripes, buf, 512), "describe")
        return buf.value.decode()

    def close(self) -> None:
        if self.ptr:
            lib.nxec_ctx_destroy(C.c_void_p(self.ptr))
            self.ptr = 0


class Group:
    """nxec_group_t: one context per device, stripes sharded in contiguous
    ranges, one host thread per device (no collectives)."""

    def __init__(self, devices: Sequence[int]):
        d = np.ascontiguousarray(list(devices), dtype=np.int32)
        p = C.c_void_p()
        check(lib.nxec_group_create(C.c_void_p(d.ctypes.data), len(d), C.byref(p)), "nxec_group_create")
        self.ptr = p.value
        self.devices = [int(x) for x in d]

    def __len__(self) -> int:
        return int(lib.nxec_group_size(C.c_void_p(self.ptr)))

    @staticmethod
    def shard(nstripes: int, nparts: int, part: int):
        """(first, count) of part `part` (nxec_group_shard)."""
        f, c = C.c_int64(), C.c_int64()
        check(lib.nxec_group_shard(nstripes, nparts, part, C.byref(f), C.byref(c)), "nxec_group_shard")
        return int(f.value), int(c.value)

    def rs_encode_host_batch(self, n: int, k: int, h_data: int, h_parity: int, length: int, nstripes: int,
                             batch_stripes: int = 0) -> None:
        check(lib.nxec_group_rs_encode_host_batch(C.c_void_p(self.ptr), n, k, C.c_void_p(int(h_data)),
                                                  C.c_void_p(int(h_parity)), length, nstripes, batch_stripes),
              "nxec_group_rs_encode_host_batch")

    def rs_encode(self, n: int, k: int, stripes: Sequence[int], chunk_stride: int, stripe_stride: int, length: int,
                  nstripes: Sequence[int]) -> None:
        ptrs = (C.c_void_p * len(stripes))(*[int(x) for x in stripes])
        ns = np.ascontiguousarray(list(nstripes), dtype=np.int64)
        check(lib.nxec_group_rs_encode_stripes(C.c_void_p(self.ptr), n, k, ptrs, chunk_stride, stripe_stride, length,
                                               C.c_void_p(ns.ctypes.data)), "nxec_group_rs_encode_stripes")

    def rs_recover(self, n: int, k: int, failed: Sequence[int], stripes: Sequence[int], chunk_stride: int,
                   stripe_stride: int, length: int, nstripes: Sequence[int]) -> None:
        f = np.ascontiguousarray(list(failed), dtype=np.int32)
        ptrs = (C.c_void_p * len(stripes))(*[int(x) for x in stripes])
        ns = np.ascontiguousarray(list(nstripes), dtype=np.int64)
        check(lib.nxec_group_rs_recover_stripes(C.c_void_p(self.ptr), n, k, C.c_void_p(f.ctypes.data), len(f), ptrs,
                                                chunk_stride, stripe_stride, length, C.c_void_p(ns.ctypes.data)),
              "nxec_group_rs_recover_stripes")

    def rs_encode_async(self, n: int, k: int, stripes: Sequence[int], chunk_stride: int, stripe_stride: int,
                        length: int, nstripes: Sequence[int]) -> None:
        """nxec_group_rs_encode_stripes_async: queued on every member, returns at once (errors at wait())."""
        ptrs = (C.c_void_p * len(stripes))(*[int(x) for x in stripes])
        ns = np.ascontiguousarray(list(nstripes), dtype=np.int64)
        check(lib.nxec_group_rs_encode_stripes_async(C.c_void_p(self.ptr), n, k, ptrs, chunk_stride, stripe_stride,
                                                     length, C.c_void_p(ns.ctypes.data)),
              "nxec_group_rs_encode_stripes_async")

    def rs_recover_async(self, n: int, k: int, failed: Sequence[int], stripes: Sequence[int], chunk_stride: int,
                         stripe_stride: int, length: int, nstripes: Sequence[int]) -> None:
        f = np.ascontiguousarray(list(failed), dtype=np.int32)
        ptrs = (C.c_void_p * len(stripes))(*[int(x) for x in stripes])
        ns = np.ascontiguousarray(list(nstripes), dtype=np.int64)
        check(lib.nxec_group_rs_recover_stripes_async(C.c_void_p(self.ptr), n, k, C.c_void_p(f.ctypes.data), len(f),
                                                      ptrs, chunk_stride, stripe_stride, length,
                                                      C.c_void_p(ns.ctypes.data)),
              "nxec_group_rs_recover_stripes_async")

    def wait(self) -> None:
        """nxec_group_wait: every queued call done on every member (raises the first member failure)."""
        check(lib.nxec_group_wait(C.c_void_p(self.ptr)), "nxec_group_wait")

    def close(self) -> None:
        if self.ptr:
            lib.nxec_group_destroy(C.c_void_p(self.ptr))
            self.ptr = 0


__all__ = [
    "Group", "NxecError", "gf_mul", "gf_inv", "gen_rs_matrix", "invert_matrix", "init_tables", "rs_plan", "decode_matrix",
    "encode_host", "ec_encode_data", "car_plan", "device_count", "device_info", "device_sync", "set_device", "DeviceBuffer", "PinnedBuffer",
    "Event", "Context",
]
