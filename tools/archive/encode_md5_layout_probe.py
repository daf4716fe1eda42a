#!/usr/bin/env python3
"""Probe: nxec_rs_encode_md5_stripes (fused encode + MD5 of all n chunks) on a
device-resident [stripe][chunk] batch under several HBM layouts, against the
two-kernel path (NXEC_FUSED_MD5=0).  RS(10,4) 4096 x 1 MiB by default.

  python3 tools/encode_md5_layout_probe.py [n k chunk_bytes nstripes]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

args = [int(a) for a in sys.argv[1:]]
n, k, cs, ns = args if len(args) == 4 else (14, 10, 1 << 20, 4096)
ctx = nxec.Context(0)
layouts = [("packed", cs, n * cs), ("stripe+1 chunk", cs, (n + 1) * cs), ("chunk+2KiB", cs + 2048, n * (cs + 2048)),
           ("chunk+4KiB", cs + 4096, n * (cs + 4096)), ("chunk+256B", cs + 256, n * (cs + 256))]
big = max(ss for _, _, ss in layouts) * ns
buf = nxec.DeviceBuffer(big)
buf.fill_random(5)
dig = nxec.DeviceBuffer(ns * n * 16)
alg = ns * n * cs
for name, cst, sst in layouts:
    for mode in ("1", "0"):
        os.environ["NXEC_FUSED_MD5"] = mode
        ctx.rs_encode_md5(n, k, buf.ptr, cst, sst, cs, ns, dig.ptr)
        ctx.sync()
        reps = 6
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.rs_encode_md5(n, k, buf.ptr, cst, sst, cs, ns, dig.ptr)
        ctx.sync()
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"RS({n},{k}) {cs >> 10} KiB x {ns} {name:15s} {'fused' if mode == '1' else 'two  '} "
              f"probe={os.environ.get('NXEC_EM_PROBE', '-')} {ms:8.3f} ms ({alg / ms / 1e6 / 8000:.3f} of 8 TB/s)",
              flush=True)
buf.free()
dig.free()
ctx.close()

# repair with checksums (config 4): RS(12,4) 1 MiB x 4096 on 17 MiB stripes, chunk 0 rebuilt + its MD5
if len(args) != 4:
    ctx = nxec.Context(0)
    n, k, cs, ns = 16, 12, 1 << 20, 4096
    cst, sst = nxec.batch_layout(n, cs, 0)
    buf = nxec.DeviceBuffer(ns * sst)
    buf.fill_random(9)
    ctx.rs_encode(n, k, buf.ptr, cst, sst, cs, ns)
    dig = nxec.DeviceBuffer(ns * 16)
    alg = ns * (k + 1) * cs
    for mode in ("1", "0", "1", "0"):
        os.environ["NXEC_FUSED_MD5"] = mode
        ctx.rs_recover_md5(n, k, [0], buf.ptr, cst, sst, cs, ns, dig.ptr)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(6):
            ctx.rs_recover_md5(n, k, [0], buf.ptr, cst, sst, cs, ns, dig.ptr)
        ctx.sync()
        ms = (time.perf_counter() - t0) / 6 * 1e3
        print(f"RS(16,12) repair chunk 0 + MD5, 1 MiB x {ns}, 17 MiB stripes: {'fused' if mode == '1' else 'two  '} "
              f"{ms:8.3f} ms ({alg / ms / 1e6 / 8000:.3f} of 8 TB/s of (k+1)*cs)", flush=True)
    buf.free()
    dig.free()
    ctx.close()

# read with checksums: decode_object_verify of a 4096 x RS(10,4) 1 MiB object, 4 data chunks lost
if len(args) != 4:
    ctx = nxec.Context(0)
    n, k, M, ns = 14, 10, 1 << 20, 4096
    length = ns * k * M
    chunks = nxec.DeviceBuffer(ns * n * M)
    chunks.fill_random(21)
    ctx.rs_encode(n, k, chunks.ptr, M, n * M, M, ns)
    md5 = nxec.DeviceBuffer(ns * n * 16)
    ctx.md5_chunks(chunks.ptr, M, n * M, n, M, ns, md5.ptr)
    out = nxec.DeviceBuffer(length)
    ok = nxec.DeviceBuffer(ns * n)
    failed = [0, 1, 2, 3]
    alg = ns * 2 * k * M  # read k survivors, write k data chunks (full-output decode), as bench --workload object
    for mode in ("1", "0", "1", "0"):
        os.environ["NXEC_FUSED_MD5"] = mode
        ctx.decode_object_verify(n, k, failed, chunks.ptr, length, M, md5.ptr, out.ptr, None, ok.ptr)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(6):
            ctx.decode_object_verify(n, k, failed, chunks.ptr, length, M, md5.ptr, out.ptr, None, ok.ptr)
        ctx.sync()
        ms = (time.perf_counter() - t0) / 6 * 1e3
        print(f"RS(14,10) read + verify, 4 data chunks lost, 1 MiB x {ns}: {'fused' if mode == '1' else 'two  '} "
              f"{ms:8.3f} ms ({alg / ms / 1e6 / 8000:.3f} of 8 TB/s of 2k*cs)", flush=True)
    assert (ok.download().reshape(ns, n)[:, 4:] == 1).all()
    for b in (chunks, md5, out, ok):
        b.free()
    ctx.close()
