"""ctypes loader for libnxec.so (the C ABI in include/nxec.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) into
``nexoedge_amd/lib/libnxec.so``.  Importing this module fails loudly when it
is missing: there is no Python or CPU fallback for the coding kernels.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# NXEC_LIB: another build of the library (design A/Bs of compile-time variants;
# tools only -- the product and the tests load the in-tree build)
LIB_PATH = os.environ.get("NXEC_LIB") or os.path.join(_HERE, "lib", "libnxec.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libnxec.so not found at {LIB_PATH}; build it with `make` (or __graft_entry__.build()). "
        "nexoedge_amd has no CPU fallback."
    )

lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)

u8p = C.POINTER(C.c_ubyte)
i32p = C.POINTER(C.c_int32)
vp = C.c_void_p
i64 = C.c_int64

_PROTOS = {
    "nxec_last_error": (C.c_char_p, []),
    "nxec_version": (C.c_char_p, []),
    "nxec_design_probes": (C.c_int, []),
    "nxec_gf_mul": (C.c_ubyte, [C.c_ubyte, C.c_ubyte]),
    "nxec_gf_inv": (C.c_ubyte, [C.c_ubyte]),
    "nxec_gf_gen_rs_matrix": (None, [vp, C.c_int, C.c_int]),
    "nxec_gf_invert_matrix": (C.c_int, [vp, vp, C.c_int]),
    "nxec_ec_init_tables": (None, [C.c_int, C.c_int, vp, vp]),
    "nxec_gen_rs_matrix": (None, [vp, C.c_int, C.c_int]),
    "nxec_invert_matrix": (C.c_int, [vp, vp, C.c_int]),
    "nxec_init_tables": (None, [C.c_int, C.c_int, vp, vp]),
    "nxec_encode_data": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, vp]),
    "nxec_matmul_batch": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, i64, i64, vp, i64, i64, i64, i64, vp]),
    "nxec_ec_encode_data": (None, [C.c_int, C.c_int, C.c_int, vp, vp, vp]),
    "nxec_ec_encode_data_status": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, vp]),
    "nxec_encode_host": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, vp]),
    "nxec_encode_host_ex": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp]),
    "nxec_encode_host_md5": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp]),
    "nxec_default_devices": (C.c_int, [vp, C.c_int]),
    "nxec_default_pool_stats": (C.c_int, [vp, vp, vp, vp, C.c_int, vp]),
    "nxec_default_pick": (C.c_int, [C.c_int, vp, vp, C.c_int, C.c_int]),
    "nxec_default_admission": (C.c_int, [C.c_int, vp, vp, vp, vp, C.c_int]),
    "nxec_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "nxec_ctx_destroy": (None, [vp]),
    "nxec_ctx_stream": (vp, [vp]),
    "nxec_stripes_mul": (
        C.c_int,
        [vp, C.c_int, C.c_int, vp, vp, vp, i64, i64, vp, vp, i64, i64, vp, i64, i64, vp],
    ),
    "nxec_stripes_mul_ptrs": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, vp, i64, i64, vp]),
    "nxec_rs_encode_stripes": (C.c_int, [vp, C.c_int, C.c_int, vp, i64, i64, i64, i64, vp]),
    "nxec_rs_recover_stripes": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, i64, i64, vp]),
    "nxec_rs_decode_stripes": (
        C.c_int,
        [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, vp, i64, i64, i64, i64, vp],
    ),
    "nxec_car_plan": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp, vp, vp, C.POINTER(C.c_int)]),
    "nxec_rs_car_repair_stripes": (
        C.c_int,
        [vp, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp, i64, i64, vp, i64, i64, i64, i64, vp],
    ),
    "nxec_md5_chunks": (C.c_int, [vp, vp, i64, i64, C.c_int, i64, i64, vp, vp]),
    "nxec_rs_encode_md5_stripes": (C.c_int, [vp, C.c_int, C.c_int, vp, i64, i64, i64, i64, vp, vp]),
    "nxec_rs_recover_md5_stripes": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, i64, i64, vp, vp]),
    "nxec_decode_object_verify": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, vp, vp, vp, vp, vp, vp]),
    "nxec_md5_verify_chunks": (C.c_int, [vp, vp, i64, i64, C.c_int, i64, i64, vp, vp, vp, vp]),
    "nxec_object_layout": (C.c_int, [C.c_int, C.c_int, i64, i64, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]),
    "nxec_encode_object": (C.c_int, [vp, C.c_int, C.c_int, vp, i64, i64, vp, vp, vp, vp]),
    "nxec_encode_object_host": (C.c_int, [vp, C.c_int, C.c_int, vp, i64, i64, vp, vp, i64]),
    "nxec_objects_layout": (C.c_int, [C.c_int, C.c_int, C.c_int, vp, i64, C.POINTER(i64), C.POINTER(i64)]),
    "nxec_encode_objects": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, i64, vp, vp, vp, vp]),
    "nxec_kernel_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "nxec_kernel_time": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "nxec_encode_objects_ex": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, i64, vp, vp, vp, C.c_int, vp]),
    "nxec_decode_object": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, vp, vp, vp]),
    "nxec_decode_object_ex": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, i64, i64, vp, vp, vp]),
    "nxec_agent_encode_batch": (C.c_int, [vp, vp, C.c_int, i64, i64]),
    "nxec_rs_encode_host_batch": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, i64, i64, i64]),
    "nxec_gather_chunks": (C.c_int, [vp, vp, i64, i64, vp, i64, vp]),
    "nxec_scatter_chunks": (C.c_int, [vp, vp, i64, i64, i64, vp, vp]),
    "nxec_rs_recover_frames": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64]),
    "nxec_batch_layout_tuned": (C.c_int, [vp, C.c_int, C.c_int, i64, C.c_int, i64, C.POINTER(i64), C.POINTER(i64)]),
    "nxec_decode_frames": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, vp, i64, i64, i64]),
    "nxec_gather_chunks_async": (C.c_int, [vp, vp, i64, i64, vp, i64, vp, C.POINTER(vp)]),
    "nxec_scatter_chunks_async": (C.c_int, [vp, vp, i64, i64, i64, vp, vp, C.POINTER(vp)]),
    "nxec_request_wait": (C.c_int, [vp]),
    "nxec_rs_plan":(C.c_int, [C.c_int, C.c_int, vp, C.c_int, C.c_int, vp, C.POINTER(C.c_int), C.POINTER(C.c_int), vp]),
    "nxec_rs_decode_matrix": (C.c_int, [C.c_int, C.c_int, vp, vp, C.c_int, vp]),
    "nxec_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "nxec_set_device": (C.c_int, [C.c_int]),
    "nxec_device_info": (C.c_int, [C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(i64)]),
    "nxec_dev_malloc": (C.c_int, [C.POINTER(vp), C.c_size_t]),
    "nxec_dev_free": (C.c_int, [vp]),
    "nxec_host_malloc_pinned": (C.c_int, [C.POINTER(vp), C.c_size_t]),
    "nxec_host_free_pinned": (C.c_int, [vp]),
    "nxec_host_register": (C.c_int, [vp, C.c_size_t]),
    "nxec_host_unregister": (C.c_int, [vp]),
    "nxec_memcpy_h2d": (C.c_int, [vp, vp, C.c_size_t, vp]),
    "nxec_memcpy_d2h": (C.c_int, [vp, vp, C.c_size_t, vp]),
    "nxec_memcpy_d2d": (C.c_int, [vp, vp, C.c_size_t, vp]),
    "nxec_memset": (C.c_int, [vp, C.c_int, C.c_size_t, vp]),
    "nxec_memset2d": (C.c_int, [vp, C.c_size_t, C.c_int, C.c_size_t, C.c_size_t, vp]),
    "nxec_stream_create": (C.c_int, [C.POINTER(vp)]),
    "nxec_stream_destroy": (C.c_int, [vp]),
    "nxec_stream_sync": (C.c_int, [vp]),
    "nxec_device_sync": (C.c_int, []),
    "nxec_event_create": (C.c_int, [C.POINTER(vp)]),
    "nxec_event_destroy": (C.c_int, [vp]),
    "nxec_event_record": (C.c_int, [vp, vp]),
    "nxec_event_elapsed_ms": (C.c_int, [vp, vp, C.POINTER(C.c_float)]),
    "nxec_fill_random": (C.c_int, [vp, C.c_size_t, C.c_uint64, vp]),
    "nxec_checksum": (C.c_int, [vp, C.c_size_t, C.POINTER(C.c_uint64), vp]),
    "nxec_describe_launch": (C.c_int, [vp, C.c_int, C.c_int, i64, i64, C.c_char_p, C.c_int]),
    "nxec_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(vp)]),
    "nxec_batch_layout": (C.c_int, [C.c_int, i64, C.c_int, C.POINTER(i64), C.POINTER(i64)]),
    "nxec_host_free": (C.c_int, [vp]),
    "nxec_host_arena_owns": (C.c_int, [vp]),
    "nxec_host_arena_stats": (C.c_int, [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "nxec_host_arena_cap": (C.c_size_t, []),
    "nxec_host_arena_trim": (C.c_int, [C.c_size_t]),
    "nxec_host_range_mapped": (C.c_int, [vp, C.c_size_t]),
    "nxec_chunk_md5_mode": (C.c_int, []),
    "nxec_digest_clear": (None, []),
    "nxec_digest_note": (C.c_int, [vp, i64, vp]),
    "nxec_digest_take": (C.c_int, [vp, i64, vp]),
    "nxec_digest_forget": (None, [vp]),
    "nxec_digest_epoch": (C.c_uint64, []),
    "nxec_digest_epoch_bump": (None, []),
    "nxec_set_digest_placement": (C.c_int, [C.c_int]),
    "nxec_digest_placement": (C.c_int, []),
    "nxec_digest_place_params": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "nxec_digest_place_stats": (C.c_int, [C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), C.POINTER(C.c_int)]),
    "nxec_storage_classes_load": (C.c_int, [C.c_char_p, vp, C.c_int, C.POINTER(C.c_int)]),
    "nxec_proxy_repair_using_car": (C.c_int, [C.c_char_p, C.POINTER(C.c_int)]),
    "nxec_cxx_abi_check": (C.c_int, [vp]),
    "nxec_cxx_abi_self": (None, [vp]),
    "nxec_reset_work_queues": (C.c_int, []),
    "nxec_debug_poison_next_queue_slot": (C.c_int, [C.c_uint32]),
    "nxec_pci_numa_node": (C.c_int, [C.c_char_p, C.POINTER(C.c_int)]),
    "nxec_numa_node_cpus": (C.c_int, [C.c_int, vp, C.c_int, C.POINTER(C.c_int)]),
    "nxec_bind_thread_to_pci": (C.c_int, [C.c_char_p, C.POINTER(C.c_int)]),
    "nxec_device_numa_node": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "nxec_bind_thread_to_device": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "nxec_group_create": (C.c_int, [vp, C.c_int, C.POINTER(vp)]),
    "nxec_group_destroy": (None, [vp]),
    "nxec_group_size": (C.c_int, [vp]),
    "nxec_group_ctx": (vp, [vp, C.c_int]),
    "nxec_group_shard": (C.c_int, [i64, C.c_int, C.c_int, C.POINTER(i64), C.POINTER(i64)]),
    "nxec_group_rs_encode_host_batch": (C.c_int, [vp, C.c_int, C.c_int, vp, vp, i64, i64, i64]),
    "nxec_group_rs_encode_stripes": (C.c_int, [vp, C.c_int, C.c_int, vp, i64, i64, i64, vp]),
    "nxec_group_rs_recover_stripes": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, i64, vp]),
    "nxec_group_rs_encode_stripes_async": (C.c_int, [vp, C.c_int, C.c_int, vp, i64, i64, i64, vp]),
    "nxec_group_rs_recover_stripes_async": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int, vp, i64, i64, i64, vp]),
    "nxec_group_wait": (C.c_int, [vp]),
    "nxec_layout_choose": (C.c_int, [C.c_int, C.c_int, vp, C.c_double]),
}


class StorageClass(C.Structure):
    """struct nxec_storage_class of include/nxec.h"""
    _fields_ = [("name", C.c_char * 64), ("coding", C.c_int), ("n", C.c_int), ("k", C.c_int), ("f", C.c_int),
                ("max_chunk_size", C.c_int64), ("is_default", C.c_int)]


class AgentReq(C.Structure):
    """struct nxec_agent_req of include/nxec.h"""
    _fields_ = [("ninputs", C.c_int), ("noutputs", C.c_int), ("matrix", vp), ("inputs", vp), ("outputs", vp),
                ("md5", vp), ("md5_inputs", vp)]


for _name, (_res, _args) in _PROTOS.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = tuple(_PROTOS)

NXEC_OK = 0
NXEC_ERR_SINGULAR = -1
NXEC_ERR_INVALID = -2
NXEC_ERR_HIP = -3
NXEC_ERR_NOMEM = -4
NXEC_ERR_NODEV = -5


class NxecError(RuntimeError):
    def __init__(self, code: int, what: str):
        msg = lib.nxec_last_error().decode(errors="replace")
        super().__init__(f"{what} failed ({code}): {msg}")
        self.code = code


def check(rc: int, what: str) -> None:
    if rc != NXEC_OK:
        raise NxecError(rc, what)
