#!/usr/bin/env python3
"""Headline benchmark: GiB/s RS(10,4) encode+decode, 1 MiB chunks, device-resident.

One step = one pass of the hot path over one batch: RS(10,4) encode of a
4096-stripe batch (nexoedge (n,k) = (14,10), 1 MiB chunks, [stripe][chunk][byte]
layout in HBM) followed by a 4-erasure recover of the same batch (rotating over
the erasure patterns {0,1,2,3}, {10..13}, {1,4,11,13}).  Bytes are counted the
ISA-L way (erasure_code_perf.c): encode (k+p)*cs, decode (k+e)*cs per stripe.

Multi-GPU: one process per GPU (torch.distributed.run), stripes sharded with
no collective on the data path (weak scaling: every rank owns its own
4096-stripe batch); gloo is used only for the barrier and the max-over-ranks
timing reduction.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import nexoedge_amd  # noqa: E402  (load libnxec before torch: one HIP runtime)
from nexoedge_amd import nxec  # noqa: E402
from nexoedge_amd.dist import RankGroup  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PATTERNS = ([0, 1, 2, 3], [10, 11, 12, 13], [1, 4, 11, 13])
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU (batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-stripes", type=int, default=192)
    ap.add_argument("--host-inclusive", action="store_true", help="also time the pinned H2D->encode->D2H pipeline")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "r01_pmc_traffic.json"))
    return ap.parse_args()


def cpu_baseline(args, n, k, cs):
    """Reference ISA-L 2.22 (base C, oracle/_ref) on the host cores: the same
    encode + (k,e)-recover work on a bounded sample of stripes."""
    import concurrent.futures as cf

    import numpy as np

    import oracle

    kind = "reference" if oracle.ref_available() else "port"
    p, e = n - k, len(PATTERNS[0])
    ns = args.cpu_stripes
    threads = args.cpu_threads
    enc = nxec.gen_rs_matrix(n, k)[k:]
    data = oracle.fill_bytes(ns * k * cs, 99).reshape(ns, k, cs)
    parity = np.zeros((ns, p, cs), dtype=np.uint8)
    rec = np.zeros((ns, e, cs), dtype=np.uint8)
    ref = oracle.RefISAL() if kind == "reference" else None

    def enc_range(lo, hi):
        for s in range(lo, hi):
            if ref:
                ref.encode(enc, list(data[s]), list(parity[s]))
            else:
                parity[s] = np.stack(oracle.matmul(enc, list(data[s])))

    def rec_range(lo, hi, failed):
        ids, _, rm = nxec.rs_plan(n, k, failed, True)
        for s in range(lo, hi):
            st = np.concatenate([data[s], parity[s]])
            srcs = [st[i] for i in ids[:k]]
            if ref:
                ref.encode(rm, srcs, list(rec[s]))
            else:
                rec[s] = np.stack(oracle.matmul(rm, srcs))

    bounds = [(ns * t // threads, ns * (t + 1) // threads) for t in range(threads)]
    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda b: enc_range(*b), bounds))
        t1 = time.perf_counter()
        list(ex.map(lambda b: rec_range(*b, PATTERNS[0]), bounds))
        t2 = time.perf_counter()
    bytes_done = ns * (k + p) * cs + ns * (k + e) * cs
    return {
        "value": round(bytes_done / (t2 - t0) / GIB, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": kind,
        "sample": (f"RS(10,4) (n,k)=({n},{k}) {cs >> 10} KiB chunks, {ns} stripes: encode then recover "
                   f"{PATTERNS[0]} (rs.cc repair path), {threads} threads over stripes; "
                   + ("ISA-L 2.22 ec_base.c built from the reference tarball (pure C: no nasm here for "
                      "ISA-L's SIMD asm)" if kind == "reference" else "oracle restatement")),
        "encode_s": round(t1 - t0, 3),
        "decode_s": round(t2 - t1, 3),
    }


def load_traffic(path, launch_bytes):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    grp = RankGroup()
    world, rank, local = grp.world, grp.rank, grp.local_rank
    n, k, cs, ns = args.n, args.k, args.chunk, args.stripes
    p = n - k
    e = len(PATTERNS[0])
    ctx = nxec.Context(local)
    stream = ctx.stream
    stripe = n * cs
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(0xC0FFEE + rank * 7919)  # synthetic data; parity region overwritten by encode

    enc_bytes = ns * (k + p) * cs
    dec_bytes = ns * (k + e) * cs
    step_bytes = enc_bytes + dec_bytes

    def step(i, evs=None):
        if evs is not None:
            evs[0].record(stream)
        ctx.rs_encode(n, k, buf.ptr, cs, stripe, cs, ns, stream)
        if evs is not None:
            evs[1].record(stream)
        ctx.rs_recover(n, k, PATTERNS[i % len(PATTERNS)], buf.ptr, cs, stripe, cs, ns, stream)
        if evs is not None:
            evs[2].record(stream)

    for i in range(args.warmup):
        step(i)
    ctx.sync()
    nxec.device_sync()

    evs = [[nxec.Event() for _ in range(3)] for _ in range(args.steps)]
    grp.barrier()
    nxec.device_sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, evs[i])
    ctx.sync()
    nxec.device_sync()
    t1 = time.perf_counter()
    grp.barrier()
    local_s = t1 - t0
    elapsed = grp.max(local_s)

    enc_ms = [evs[i][0].elapsed_ms(evs[i][1]) for i in range(args.steps)]
    dec_ms = [evs[i][1].elapsed_ms(evs[i][2]) for i in range(args.steps)]
    enc_avg = sum(enc_ms) / len(enc_ms)
    dec_avg = sum(dec_ms) / len(dec_ms)
    total_bytes = grp.sum(float(step_bytes * args.steps))

    result = None
    if rank == 0:
        # roofline of the dominant kernel (k_mul_vec<10, R16>, encode launch):
        # algorithmic bytes per launch / event-timed launch duration
        enc_gbs = enc_bytes / (enc_avg * 1e-3) / 1e9
        dec_gbs = dec_bytes / (dec_avg * 1e-3) / 1e9
        traffic = load_traffic(args.pmc_summary, enc_bytes)
        result = {
            "metric": "GiB/s RS(10,4) encode+decode, 1 MiB chunks, device-resident",
            "value": round(total_bytes / elapsed / GIB, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes, device-generated)",
            "config": {
                "workload": f"RS(10,4) (n,k)=({n},{k}) encode + {e}-erasure recover, {cs >> 10} KiB chunks, "
                            f"{ns}-stripe batch per GPU, [stripe][chunk][byte] in HBM",
                "stripes_per_gpu": ns,
                "chunk_bytes": cs,
                "erasure_patterns": PATTERNS,
                "byte_accounting": "encode (k+p)*cs + decode (k+e)*cs per stripe (ISA-L erasure_code_perf.c)",
                "parallelism": f"stripe-sharded x{world}, no collectives",
                "launch": json.loads(ctx.describe_launch(p, k, cs, ns)),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(enc_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "k_mul_vec<K=10,R=16> (encode launch)",
                "bytes_per_launch": enc_bytes,
                "avg_launch_ms": round(enc_avg, 4),
                "decode_achieved": round(dec_gbs, 1),
                "decode_frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                "decode_avg_launch_ms": round(dec_avg, 4),
            },
            "user_data_gib_s": round(2 * ns * k * cs * args.steps * world / elapsed / GIB, 2),
        }
    if args.host_inclusive and rank == 0:
        result["host_inclusive"] = host_inclusive(ctx, n, k, cs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, n, k, cs)
    if rank == 0:
        print(json.dumps(result), flush=True)
    buf.free()
    ctx.close()
    grp.close()


def host_inclusive(ctx, n, k, cs, ns=512):
    """Pinned host buffers in and out: H2D data -> encode -> D2H parity, triple-buffered."""
    p = n - k
    hd = nxec.PinnedBuffer(ns * k * cs)
    hp = nxec.PinnedBuffer(ns * p * cs)
    import numpy as np

    hd.array[:] = np.random.default_rng(1).integers(0, 256, size=hd.nbytes, dtype=np.uint8)
    ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
    dt = (time.perf_counter() - t0) / reps
    out = {"encode_GiB_s_(k+p)cs": round(ns * (k + p) * cs / dt / GIB, 2),
           "pcie_bytes_GiB_s": round(ns * (k + p) * cs / dt / GIB, 2), "stripes": ns, "batch": 64}
    hd.free()
    hp.free()
    return out


if __name__ == "__main__":
    main()
