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
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

nxec = None  # nexoedge_amd.nxec, imported in main() (after the rank launcher)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PATTERNS = ([0, 1, 2, 3], [10, 11, 12, 13], [1, 4, 11, 13])
GIB = float(1 << 30)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (= ranks).  Without WORLD_SIZE in the environment (not under torch.distributed.run) "
                         "bench.py starts the N rank processes itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks only rendezvous (gloo), reduce and report")
    ap.add_argument("--steps", type=int, default=50, help="timed steps (default ~1 s of device time at the headline)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU (batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: every CPU of this process's affinity mask)")
    ap.add_argument("--cpu-stripes", type=int, default=192, help="CPU baseline sample (raised to >= one per thread)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="min wall time of the SIMD CPU baseline leg")
    ap.add_argument("--cpu-ref-stripes", type=int, default=96, help="stripes for the (slow) reference base-C leg")
    ap.add_argument("--host-inclusive", dest="host_inclusive", action="store_true", default=True,
                    help="also time the pinned H2D->encode->D2H pipeline (default on; N=1 headline workload only)")
    ap.add_argument("--no-host-inclusive", dest="host_inclusive", action="store_false")
    ap.add_argument("--workload", choices=sorted(["rs10_4", "decode_full", "repair12", "mixed16", "write14", "object",
                                                 "files", "config1"]), default="rs10_4",
                    help="rs10_4 = headline (configs 2+3); decode_full = config 3 on RSCode::decode's all-k output; "
                         "repair12 = config 4; mixed16 = config 5 (one chunk size)")
    ap.add_argument("--failed", type=int, default=None, help="repair12: failed chunk id (default 0)")
    ap.add_argument("--gib", type=float, default=32.0, help="mixed16: GiB of stripes per GPU")
    ap.add_argument("--group", action="store_true",
                    help="rs10_4 only: also drive all N GPUs from ONE process through nxec_group (one host thread "
                         "+ context per device); reported as `group` beside the per-rank value, not as value")
    ap.add_argument("--layout", choices=["auto", "natural", "recover", "tuned"], default="auto",
                    help="HBM batch layout: natural = packed [stripe][n][cs]; auto = nxec_batch_layout (padded "
                         "chunk stride for chunks >= 2 MiB); recover = nxec_batch_layout(RECOVER_HEAVY) (odd "
                         "stripe stride in 1 MiB units); tuned = nxec_batch_layout_tuned (measured on this device)")
    return ap.parse_args(argv)


def _cpu_legs(threads, ns, legs, min_s):
    """Run each leg fn(lo, hi) over `ns` stripes split into `threads` contiguous
    ranges (one C call per thread and leg: ctypes releases the GIL), legs back
    to back, repeating the round until at least `min_s` seconds have elapsed.
    Returns (rounds, [seconds per leg])."""
    import concurrent.futures as cf

    bounds = [(ns * t // threads, ns * (t + 1) // threads) for t in range(threads)]
    bounds = [b for b in bounds if b[1] > b[0]]
    reps, secs = 0, [0.0] * len(legs)
    with cf.ThreadPoolExecutor(len(bounds)) as ex:
        while reps == 0 or sum(secs) < min_s:
            for i, fn in enumerate(legs):
                t0 = time.perf_counter()
                list(ex.map(lambda b: fn(*b), bounds))
                secs[i] += time.perf_counter() - t0
            reps += 1
    return reps, secs


def _host_info():
    """CPU model, nproc, this process's affinity mask and the cgroup CPU quota
    (the GPU box runs the bench in a cgroup: `cpu.max` caps the CPU time all
    threads together get, whatever the affinity mask lists)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    info = {"cpu": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


def _cgroup_cpu_stat():
    """The cgroup's CPU accounting (cpu.stat: usage, throttling), {} when absent."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {ln.split()[0]: int(ln.split()[1]) for ln in f if len(ln.split()) == 2}
    except (OSError, ValueError):
        return {}


def cpu_baseline(args, n, k, cs):
    """The same encode + (k,e)-recover work on a bounded sample of stripes on the
    host cores, one contiguous stripe range per thread:

    * value: RSCode::encode as the reference runs it per stripe -- the rs.cc:80
      copy of the k data chunks into the stripe's chunk buffers, then
      ec_encode_data -- followed by the 4-erasure recover (rs.cc repair rows),
      with the production-class stand-in for ISA-L's SIMD kernels
      (oracle/nxec_cpu_simd.c, split-nibble vpshufb, the faster of AVX-512BW /
      AVX2 here) -- `kind: "port"`.  Threads = this process's CPU affinity
      mask (`cores`); the cgroup quota that shares them is stated in `host`.
    * reference_base_c: the reference's own ISA-L 2.22 base C built from its
      tarball (oracle/_ref), the only ISA-L path buildable here (no nasm).
    * reference_read_decode: the reference's read-path decode, all k rows of
      the k x k inverse (rs.cc:196,228-230), which the recover leg replaces."""
    import numpy as np

    import oracle

    p, e = n - k, len(PATTERNS[0])
    info = _host_info()
    threads = args.cpu_threads or info["affinity"]
    ns = max(args.cpu_stripes, threads)
    enc = nxec.gen_rs_matrix(n, k)[k:]
    ids, _, rm = nxec.rs_plan(n, k, PATTERNS[0], True)
    ids = ids[:k]
    # uniform random bytes (the SIMD path has no data-dependent timing): one
    # random stripe, replicated
    one = oracle.fill_bytes(k * cs, 99).reshape(1, k, cs)
    data = np.empty((ns, k, cs), dtype=np.uint8)
    data[:] = one
    chunks = np.zeros((ns, n, cs), dtype=np.uint8)
    rec = np.zeros((ns, max(e, k), cs), dtype=np.uint8)
    stripe_bytes = (k + p) * cs + (k + e) * cs

    def legs(level):
        fe = lambda lo, hi: oracle.simd_rscode_encode_range(level, n, k, cs, lo, hi, data, chunks, enc)  # noqa: E731
        fr = lambda lo, hi: oracle.simd_rscode_decode_range(level, n, k, cs, lo, hi, chunks, ids, rm, rec)  # noqa: E731
        return [fe, fr]

    best = None
    top = oracle.simd_level()
    for level in sorted({lv for lv in (top, 256) if 0 < lv <= top}, reverse=True):
        reps, (es, rs_) = _cpu_legs(threads, ns, legs(level), args.cpu_seconds)
        gibs = reps * ns * stripe_bytes / (es + rs_) / GIB
        if best is None or gibs > best[0]:
            best = (gibs, level, reps, es, rs_)
    gibs, level, reps, es, rs_ = best
    sample = (f"RS(10,4) (n,k)=({n},{k}) {cs >> 10} KiB chunks, {ns} stripes x {reps} passes: RSCode::encode (rs.cc:80 "
              f"copy of the data chunks + parity) then recover {PATTERNS[0]} (rs.cc repair rows), {threads} threads, "
              f"one contiguous stripe range each")
    out = {
        "value": round(gibs, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": sample + f"; split-nibble vpshufb {'AVX-512BW' if level == 512 else 'AVX2'} stand-in for "
                           "ISA-L's SIMD ec_encode_data (oracle/nxec_cpu_simd.c)",
        "encode_s": round(es, 3),
        "decode_s": round(rs_, 3),
        "host": info,
    }
    # the same legs at the cgroup's CPU count and on one thread
    quota = info.get("cgroup_cpu_quota")
    out["at_affinity"] = {"threads": threads, "value": out["value"]}
    out["value_leg"] = "at_affinity"
    if quota and int(quota) != threads:
        tq = max(1, int(quota))
        r2, (e2, d2) = _cpu_legs(tq, ns, legs(level), args.cpu_seconds / 2)
        out["at_cgroup_quota"] = {"threads": tq, "value": round(r2 * ns * stripe_bytes / (e2 + d2) / GIB, 3)}
        if out["at_cgroup_quota"]["value"] > out["value"]:  # report the host's better figure
            out["value"], out["cores"], out["value_leg"] = out["at_cgroup_quota"]["value"], tq, "at_cgroup_quota"
    nss = min(ns, 16)
    r1, (e1, d1) = _cpu_legs(1, nss, legs(level), 1.0)
    out["single_thread"] = round(r1 * nss * stripe_bytes / (e1 + d1) / GIB, 3)
    # the reference's read decode: all k rows of the inverse (rs.cc:228-230)
    inv = nxec.decode_matrix(n, k, ids, list(range(k)))
    fd = lambda lo, hi: oracle.simd_rscode_decode_range(level, n, k, cs, lo, hi, chunks, ids, inv, rec)  # noqa: E731
    r3, (d3,) = _cpu_legs(threads, ns, [fd], 1.0)
    out["reference_read_decode"] = {"value": round(r3 * ns * (k + e) * cs / d3 / GIB, 3), "unit": "GiB/s (k+e)*cs",
                                    "note": "rs.cc decode: k x k inverse applied to all k rows, SIMD port"}
    if oracle.ref_available():
        ref = oracle.RefISAL()
        nsr = max(min(ns, args.cpu_ref_stripes), min(threads, ns))

        def rfe(lo, hi):
            for s in range(lo, hi):
                ref.encode(enc, list(data[s]), list(chunks[s, k:]))

        def rfr(lo, hi):
            for s in range(lo, hi):
                ref.encode(rm, [chunks[s, i] for i in ids], list(rec[s, :e]))
        r4, (e4, d4) = _cpu_legs(threads, nsr, [rfe, rfr], 0.0)
        out["reference_base_c"] = {
            "value": round(r4 * nsr * stripe_bytes / (e4 + d4) / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "reference", "sample": f"{nsr} stripes, same work (without the rs.cc:80 copy); ISA-L 2.22 "
                                           "ec_base.c built from the reference tarball (pure C)"}
    return out


PMC_SUMMARIES = {  # (workload, chunk, layout) -> labelled per-dispatch PMC file (tools/pmc_label.py) and its op
    # round-6 passes on the shipped library (tools/gpu_r06_final.sh; every dispatch
    # of the roofline kernel labelled with the bench line's bytes per launch);
    # tests/test_bench_line.py checks each file's labels and reports its lib_sha16
    # against libnxec.so; only the default layout the passes ran with (other
    # layouts report traffic null)
    ("rs10_4", 1 << 20, "auto"): ("r06_pmc_rs10_4.json", "encode_recover"),
    ("decode_full", 1 << 20, "auto"): ("r06_pmc_decode_full.json", "decode_full"),
    ("mixed16", 4 << 20, "auto"): ("r06_pmc_mixed16.json", "encode_recover"),
    ("write14", 1 << 20, "auto"): ("r06_pmc_write14.json", "encode_md5_fused"),
    ("repair12", 1 << 20, "auto"): ("r06_pmc_repair12.json", "repair_fused_perm12"),
    ("files", 1 << 20, "auto"): ("r06_pmc_files.json", "encode_objects_md5"),
}


def lib_sha16():
    """First 16 hex digits of the SHA-256 of the loaded libnxec.so (ties a
    committed PMC pass to the library it measured)."""
    import hashlib

    from nexoedge_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_traffic(args, wl_name, launch_bytes):
    """HBM bytes per launch of the roofline kernel from the committed PMC passes
    (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, gfx950 x2 read correction): the
    measured traffic/algorithmic ratio of that op's dispatches times this
    launch's algorithmic bytes, with the PMC file and the library hash it was
    measured on and whether that is the running library (`same_library`:
    false means the pass predates it).  (None, None) when no pass covers this
    workload."""
    key = PMC_SUMMARIES.get((wl_name, args.chunk, args.layout))
    if key is None:
        return None, None
    try:
        with open(os.path.join(ROOT, "profiles", key[0])) as f:
            doc = json.load(f)
        ops = key[1] if isinstance(key[1], tuple) else (key[1],)
        disp = [d for d in doc["dispatches"] if d["op"] == ops[0] or d["op"].startswith(ops[1:])]
    except (OSError, ValueError, KeyError):
        return None, None
    if not disp:
        return None, None
    ratio = sum(d["hbm_bytes"] / d["algorithmic_bytes"] for d in disp) / len(disp)
    src = {"file": "profiles/" + key[0], "lib_sha16": doc.get("lib_sha16"), "dispatches": len(disp),
           "traffic_over_algorithmic": round(ratio, 5)}
    # a pass on another build still bounds the traffic (the kernels' access
    # pattern), but the line says so instead of passing it off as this library's
    src["same_library"] = src["lib_sha16"] == lib_sha16()
    return int(round(ratio * launch_bytes)), src


class Workload:
    """One bench step = the ops in `ops`, each (label, fn(step_index), algorithmic bytes)."""

    def __init__(self, name, metric, config, ops, buffers, roof_kernel, stripes, roof_ops=1, erase=None,
                 roof_bytes=None, kernel_timer=None):
        self.name, self.metric, self.config, self.ops = name, metric, config, ops
        self.buffers, self.roof_kernel, self.stripes = buffers, roof_kernel, stripes
        self.roof_ops = roof_ops  # the first roof_ops ops are launches of the roofline kernel
        # when an op launches more than the roofline kernel: that kernel's own
        # algorithmic bytes per launch, and (start(), read() -> (ms, launches))
        # timing it with HIP events inside the library
        self.roof_bytes, self.kernel_timer = roof_bytes, kernel_timer
        # erase-and-rebuild checks run after the timed region: [(label, erase(), rebuild())] on buffers[0]
        self.erase = erase or []
        # checksum buffers[0] must have after the warmup (None: only consistency is checked)
        self.expect_sum = None


def erase_checks(wl, ctx, want):
    """After the timed region: for each (label, erase, rebuild) the chunks are
    really destroyed (the batch checksum must change), then rebuilt by the
    same op the timed loop ran (it must come back to `want`, the checksum of
    the consistent batch).  A rebuild that writes nothing fails here, which
    re-running it on an intact batch cannot show."""
    out = {}
    for label, erase, rebuild in wl.erase:
        erase()
        ctx.sync()
        destroyed = wl.buffers[0].checksum() != want
        rebuild()
        ctx.sync()
        out[label] = bool(destroyed and wl.buffers[0].checksum() == want)
    return out


def _zero_chunks(buf, chunks, cst, stripe, cs, ns, stream):
    for c in chunks:
        buf.memset2d(0, c * cst, stripe, cs, ns, stream)


def layout(args, n, cs, ctx=None, k=None):
    """(chunk_stride, stripe_stride, description) of the batch layout --layout selects."""
    if args.layout == "natural":
        return cs, n * cs, "packed [stripe][n][cs]"
    if args.layout == "tuned":
        c, st = ctx.batch_layout_tuned(n, k, cs)
        return c, st, f"nxec_batch_layout_tuned: chunk stride {c} B, stripe stride {st} B (measured on this device)"
    flags = nxec.LAYOUT_RECOVER_HEAVY if args.layout == "recover" else 0
    c, st = nxec.batch_layout(n, cs, flags)
    return c, st, f"nxec_batch_layout({args.layout}): chunk stride {c} B, stripe stride {st} B"


def wl_rs10_4(args, ctx, stream, rank):
    """Configs 2+3: RS(10,4) encode + 4-erasure recover, 1 MiB chunks, 4096 stripes."""
    n, k, cs, ns = args.n, args.k, args.chunk, args.stripes
    p, e = n - k, len(PATTERNS[0])
    cst, stripe, lay = layout(args, n, cs, ctx, k)
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(0xC0FFEE + rank * 7919)  # synthetic data; parity region overwritten by encode
    ops = [
        ("encode", lambda i: ctx.rs_encode(n, k, buf.ptr, cst, stripe, cs, ns, stream), ns * (k + p) * cs),
        ("decode", lambda i: ctx.rs_recover(n, k, PATTERNS[i % len(PATTERNS)], buf.ptr, cst, stripe, cs, ns, stream),
         ns * (k + e) * cs),
    ]
    config = {
        "workload": f"RS(10,4) (n,k)=({n},{k}) encode + {e}-erasure recover, {cs >> 10} KiB chunks, "
                    f"{ns}-stripe batch per GPU, [stripe][chunk][byte] in HBM",
        "stripes_per_gpu": ns, "chunk_bytes": cs, "erasure_patterns": PATTERNS, "layout": lay,
        "byte_accounting": "encode (k+p)*cs + decode (k+e)*cs per stripe (ISA-L erasure_code_perf.c)",
        "launch": json.loads(ctx.describe_launch(p, k, cs, ns)),
    }
    kern = config["launch"]["kernel"]
    zero = lambda cl: _zero_chunks(buf, cl, cst, stripe, cs, ns, stream)  # noqa: E731
    erase = [("encode", lambda: zero(range(k, n)), lambda: ops[0][1](0))]
    for i, pat in enumerate(PATTERNS):
        erase.append((f"recover{pat}", lambda pat=pat: zero(pat), lambda i=i: ops[1][1](i)))
    # encode and the 4-row recovers are launches of the same kernel
    # (k_mul_vec<10, 8, ...>): the roofline averages all of them, as rocprofv3's
    # per-kernel mean does
    return Workload("rs10_4", "GiB/s RS(10,4) encode+decode, 1 MiB chunks, device-resident", config, ops, [buf],
                    f"{kern} K={k} rows={p} work-queue (encode + recover launches)", ns, roof_ops=2, erase=erase)


def wl_decode_full(args, ctx, stream, rank):
    """Config 3 on the reference's own read contract: RSCode::decode returns
    all k data chunks of the stripe (the k x k inverse's rows, rs.cc:114,
    175-181, 228-230), not only the lost ones.  nxec_rs_decode_stripes reads
    the k surviving chunks chosen as rs.cc:252-265 does and writes all k data
    chunks to a separate [stripe][k][cs] output: the erased ones rebuilt,
    the surviving ones passed through (unit rows of the inverse).  4 erasures,
    rotating over the headline's three patterns; 2k*cs per stripe."""
    n, k, cs, ns = args.n, args.k, args.chunk, args.stripes
    cst, stripe, lay = layout(args, n, cs, ctx, k)
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(0xDEC0DE + rank * 7919)
    ctx.rs_encode(n, k, buf.ptr, cst, stripe, cs, ns, stream)
    out = nxec.DeviceBuffer(ns * k * cs)

    def dec(pat):
        ctx.rs_decode(n, k, pat, buf.ptr, cst, stripe, out.ptr, cs, k * cs, cs, ns, stream)

    # parity-only loss: every output row is a pass-through of its data chunk,
    # so the output is the data itself -- the checksum every pattern must give
    dec(PATTERNS[1])
    ctx.sync()
    copy_sum = out.checksum()
    ops = [("decode_full", lambda i: dec(PATTERNS[i % len(PATTERNS)]), ns * 2 * k * cs)]
    config = {
        "workload": f"RS(10,4) (n,k)=({n},{k}) full-output decode (all k data chunks, rs.cc:114,228-230), "
                    f"4 erasures, {cs >> 10} KiB chunks, {ns}-stripe batch per GPU",
        "stripes_per_gpu": ns, "chunk_bytes": cs, "erasure_patterns": PATTERNS, "layout": lay,
        "byte_accounting": "k surviving chunks read + k data chunks written = 2k*cs per stripe",
        "launch": json.loads(ctx.describe_launch(len(PATTERNS[0]), k, cs, ns)),
    }
    kern = config["launch"]["kernel"]
    erase = [(f"decode{pat}", lambda: out.memset(0), lambda pat=pat: dec(pat)) for pat in PATTERNS]
    wl = Workload("decode_full", "GiB/s RS(10,4) full-output decode (reference contract), 1 MiB chunks, "
                  "device-resident", config, ops, [out, buf], f"{kern} K={k} copy-through (full-output decode)", ns,
                  erase=erase)
    wl.expect_sum = copy_sum
    return wl


def wl_repair12(args, ctx, stream, rank):
    """Config 4: RS(12,4) single-failure repair; fused (k+1) recover and the
    unfused agent partial-encode path (racks of 4 chunks: partial 1 x g encodes,
    container_manager.cc:251, then the CAR XOR finalize, rs.cc:94-109)."""
    n, k, cs, ns, g = 16, 12, args.chunk, args.stripes, 4
    cst, stripe, lay = layout(args, n, cs, ctx, k)
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(0xBEEF + rank)
    ctx.rs_encode(n, k, buf.ptr, cst, stripe, cs, ns, stream)
    failed = args.failed if args.failed is not None else 0
    racks = [list(range(r, min(r + g, n))) for r in range(0, n, g)]  # chunk i on agent i // g
    G = len(nxec.car_plan(n, k, failed, racks))
    part = nxec.DeviceBuffer(ns * G * cs)

    def unfused(i):
        ctx.rs_car_repair(n, k, failed, racks, buf.ptr, cst, stripe, part.ptr, cs, G * cs, cs, ns, stream)

    ops = [
        ("repair_fused", lambda i: ctx.rs_recover(n, k, [failed], buf.ptr, cst, stripe, cs, ns, stream),
         ns * (k + 1) * cs),
        ("repair_car_unfused", unfused, ns * (k + 1 + 2 * G) * cs),
    ]
    config = {"workload": f"RS(12,4) (n,k)=(16,12) single-failure repair of chunk {failed}, racks of {g} chunks "
                          f"({G} partials), {cs >> 10} KiB chunks, {ns} stripes per GPU",
              "stripes_per_gpu": ns, "chunk_bytes": cs, "layout": lay,
              "byte_accounting": "fused (k+1)*cs; CAR unfused (k+1+2G)*cs per stripe (SURVEY 8d)",
              "launch": json.loads(ctx.describe_launch(1, k, cs, ns))}
    kern = config["launch"]["kernel"]
    zero = lambda: _zero_chunks(buf, [failed], cst, stripe, cs, ns, stream)  # noqa: E731
    erase = [("repair_fused", zero, lambda: ops[0][1](0)), ("repair_car_unfused", zero, lambda: unfused(0))]
    return Workload("repair12", "GiB/s RS(12,4) single-failure repair, 1 MiB chunks, device-resident", config, ops,
                    [buf, part], f"{kern} K={k} rows=1 (fused recover)", ns, erase=erase)


def wl_mixed16(args, ctx, stream, rank):
    """Config 5: RS(16,4) alternating encode / 4-erasure decode at one chunk size;
    the stripe count fills ~args.gib GiB per GPU."""
    n, k, cs = 20, 16, args.chunk
    cst, stripe, lay = layout(args, n, cs, ctx, k)
    ns = max(1, int(args.gib * (1 << 30)) // stripe)
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(0xFACE + rank)
    pats = ([0, 1, 2, 3], [16, 17, 18, 19], [1, 4, 17, 19])
    ops = [
        ("encode", lambda i: ctx.rs_encode(n, k, buf.ptr, cst, stripe, cs, ns, stream), ns * n * cs),
        ("decode", lambda i: ctx.rs_recover(n, k, pats[i % 3], buf.ptr, cst, stripe, cs, ns, stream), ns * n * cs),
    ]
    config = {"workload": f"RS(16,4) (n,k)=(20,16) encode + 4-erasure recover, {cs >> 10} KiB chunks, {ns} stripes "
                          f"(~{args.gib} GiB) per GPU",
              "stripes_per_gpu": ns, "chunk_bytes": cs, "erasure_patterns": pats, "layout": lay,
              "launch": json.loads(ctx.describe_launch(4, k, cs, ns))}
    zero = lambda cl: _zero_chunks(buf, cl, cst, stripe, cs, ns, stream)  # noqa: E731
    erase = [("encode", lambda: zero(range(k, n)), lambda: ops[0][1](0))]
    erase += [(f"recover{pat}", lambda pat=pat: zero(pat), lambda i=i: ops[1][1](i)) for i, pat in enumerate(pats)]
    return Workload("mixed16", f"GiB/s RS(16,4) encode+decode, {cs >> 10} KiB chunks, device-resident", config, ops,
                    [buf], "k_mul_vec<K=16,R=8> (encode launch)", ns, erase=erase)


def wl_write14(args, ctx, stream, rank):
    """Write path of the proxy (chunk_manager.cc:99-175): RS(10,4) encode of the
    batch plus the MD5 digest of all n chunks of every stripe (Chunk::computeMD5,
    chunk.hh:136), as ONE fused kernel (nxec_rs_encode_md5_stripes ->
    k_encode_md5): the data is read from HBM once, the parity written once, and
    every chunk's MD5 chain runs on the same bytes from LDS.  MD5 is a serial
    chain per chunk (one lane each), so the kernel is bound by the chain's VALU
    issue, not by HBM."""
    n, k, cs, ns = args.n, args.k, args.chunk, args.stripes
    stripe = n * cs
    buf = nxec.DeviceBuffer(ns * stripe)
    buf.fill_random(0xC0FFEE + rank * 7919)
    dig = nxec.DeviceBuffer(ns * n * 16)
    ops = [
        ("encode_md5_fused", lambda i: ctx.rs_encode_md5(n, k, buf.ptr, cs, stripe, cs, ns, dig.ptr, stream),
         ns * n * cs),
    ]
    config = {"workload": f"RS({n},{k}) write path: encode + per-chunk MD5 of all {n} chunks in one fused kernel, "
                          f"{cs >> 10} KiB chunks, {ns} stripes per GPU", "stripes_per_gpu": ns, "chunk_bytes": cs,
              "byte_accounting": "n*cs per stripe: one HBM pass (k*cs read, (n-k)*cs written); the MD5 of all n "
                                 "chunks reads the same bytes from LDS"}
    return Workload("write14", "GiB/s RS(10,4) encode + per-chunk MD5, 1 MiB chunks, device-resident", config, ops,
                    [buf, dig], f"k_mul_md5<K={k}> (fused encode + MD5; MD5-chain-bound, not HBM-bound)", ns)


def wl_object(args, ctx, stream, rank):
    """Object-level write and read: nxec_encode_object over an
    object of `stripes` full RS(10,4) stripes (data chunks read in place,
    parity + MD5 of all n chunks per stripe, chunk_manager.cc:99-175,369-452),
    and nxec_decode_object of the stored chunks with 4 data chunks lost
    (decodeFile, chunk_manager.cc:738-800) back into a contiguous object."""
    n, k, M, ns = args.n, args.k, args.chunk, args.stripes
    p = n - k
    length = ns * k * M
    obj = nxec.DeviceBuffer(length)
    obj.fill_random(0xD00D + rank)
    par = nxec.DeviceBuffer(ns * p * M)
    md5 = nxec.DeviceBuffer(ns * n * 16)
    chunks = nxec.DeviceBuffer(ns * n * M)
    chunks.fill_random(0xF00D + rank)
    ctx.rs_encode(n, k, chunks.ptr, M, n * M, M, ns, stream)
    out = nxec.DeviceBuffer(length)
    failed = list(range(min(4, p)))
    cmd5 = nxec.DeviceBuffer(ns * n * 16)  # digests of the stored chunks, for the verified read
    ctx.md5_chunks(chunks.ptr, M, n * M, n, M, ns, cmd5.ptr, stream)
    ok = nxec.DeviceBuffer(ns * n)
    ops = [
        ("write_encode_object_md5", lambda i: ctx.encode_object(n, k, obj.ptr, length, M, par.ptr, None, md5.ptr, stream),
         ns * n * M),
        ("read_decode_object", lambda i: ctx.decode_object(n, k, failed, chunks.ptr, length, M, out.ptr, None, stream),
         2 * ns * k * M),
        ("read_verify_decode_object",
         lambda i: ctx.decode_object_verify(n, k, failed, chunks.ptr, length, M, cmd5.ptr, out.ptr, None, ok.ptr,
                                            None, stream),
         2 * ns * k * M),
    ]
    config = {"workload": f"object of {ns} RS({n},{k}) stripes ({length >> 30} GiB), {M >> 10} KiB chunks: write = "
                          f"encode_object + MD5 of all chunks, read = decode_object with chunks {failed} lost, "
                          "then the same read with every input chunk's MD5 verified (decode_object_verify)",
              "stripes_per_gpu": ns, "chunk_bytes": M,
              "byte_accounting": "write: n*cs per stripe (one fused encode + MD5 pass); read: full-output decode "
                                 "2k*cs per stripe"}
    return Workload("object", "GiB/s object write (encode+MD5) + read (decode), RS(10,4), 1 MiB chunks, device-resident",
                    config, ops, [obj, par, md5, chunks, out, cmd5, ok], "encode_object (fused k_mul_md5)", ns)


# MD5 chain of one 256-byte step of one chunk (4 blocks), measured alone with
# the fused kernel's barriers: ~9.8 ms per 4096 steps (role probes,
# profiles/r02_encode_md5_role_probes.log) -- the floor of a slot's run
MD5_STEP_US = 9.8e3 / 4096


def files_longest_slot(n, k, M, lengths, cus=256, step=256):
    """Steps of the longest slot of nxec_encode_objects' fused plan (the LPT of
    plan_files_slots, nxec_files_md5.hip, over every request: a file's full
    stripes and its last stripe), and the request count."""
    import heapq

    reqs = []
    for L in lengths:
        ns, nf, cl = nxec.object_layout(n, k, L, M)
        reqs += [M] * nf + ([cl] if ns > nf else [])
    steps = sorted(((r + step - 1) // step for r in reqs), reverse=True)
    slots = cus * min(16, 256 // n)
    if len(steps) <= slots:
        return (max(steps) if steps else 0), len(reqs)
    heap = [(0, g) for g in range(slots)]
    for st in steps:
        load, g = heapq.heappop(heap)
        heapq.heappush(heap, (load + st, g))
    return max(l for l, _ in heap), len(reqs)


def wl_files(args, ctx, stream, rank):
    """Many files per call (nxec_encode_objects): 4096 files with sizes uniform
    in [1 B, 2*k*M] (full and ragged last stripes mixed) packed in one arena,
    encode + MD5 of every chunk.  Bytes = the kernel's HBM side, the write14
    convention: data read once + parity written + the zero-padded last-stripe
    data chunks written to the tail arena (the MD5 reads come out of LDS)."""
    import numpy as np

    n, k, M = args.n, args.k, args.chunk
    p = n - k
    rng = np.random.default_rng(1234 + rank)
    lengths = [int(x) for x in rng.integers(1, 2 * k * M + 1, size=4096)]
    offs = np.concatenate([[0], np.cumsum([(L + 15) // 16 * 16 for L in lengths])])
    arena = nxec.DeviceBuffer(int(offs[-1]))
    arena.fill_random(77 + rank)
    total, tail_bytes = nxec.objects_layout(n, k, lengths, M)
    par = nxec.DeviceBuffer(total * p * M)
    tail = nxec.DeviceBuffer(max(tail_bytes, 16))
    md5 = nxec.DeviceBuffer(total * n * 16)
    ptrs = [arena.ptr + int(o) for o in offs[:-1]]
    user = sum(lengths)
    layouts = [nxec.object_layout(n, k, L, M) for L in lengths]
    parity_bytes = sum((nf * M + (ns - nf) * cl) * p for ns, nf, cl in layouts)
    # NXEC_OBJECTS_TAIL_INPLACE (a batching ChunkManager sends whole chunks
    # from the object, as it does for full stripes): of each last stripe only
    # the partial data chunk is written, zero-padded, to the tail arena
    tail_written = sum((cl + 15) // 16 * 16 for (ns, nf, cl), L in zip(layouts, lengths)
                       if ns > nf and (L - nf * k * M) % cl)
    # k_files_md5's own bytes per launch: every request's k data chunks read
    # (last stripes: in place from the object, the chunks past the data from
    # the zero line) and p parity chunks written, at the request's chunk
    # length, plus each partial chunk's zero-padded tail-slot store (tail_written)
    kernel_bytes = sum((nf * M + (ns - nf) * cl) * n for ns, nf, cl in layouts) + tail_written
    longest, nreq = files_longest_slot(n, k, M, lengths)
    # NXEC_OBJECTS_ASYNC: the host plans batch i + 1 while batch i codes (the
    # timed region ends with a stream sync)
    ops = [("encode_objects_md5",
            lambda i: ctx.encode_objects(n, k, ptrs, lengths, M, par.ptr, tail.ptr, md5.ptr, stream,
                                         flags=nxec.OBJECTS_TAIL_INPLACE | nxec.OBJECTS_ASYNC),
            user + parity_bytes + tail_written)]
    config = {"workload": f"{len(lengths)} files, sizes uniform in [1 B, {2 * k} MiB], RS({n},{k}) {M >> 10} KiB max "
                          f"chunks ({total} stripes, {user / 2**30:.1f} GiB user data): encode + MD5 of all chunks",
              "files": len(lengths), "stripes": total, "user_bytes": user, "requests": nreq,
              "tail": "nxec_encode_objects_ex(NXEC_OBJECTS_TAIL_INPLACE): whole last-stripe data chunks stay in "
                      "their objects, the partial one is written zero-padded",
              "byte_accounting": "value: HBM side of the call, the write14 convention: data read + parity "
                                 f"written + tail-arena writes ({user / 2**30:.1f} + {parity_bytes / 2**30:.1f} + "
                                 f"{tail_written / 2**30:.1f} GiB), the MD5 of every chunk reads LDS; roofline: "
                                 f"k_files_md5 alone, (k + p) x chunk length per request + the partial chunks' tail-slot "
                                 f"stores ({kernel_bytes / 2**30:.2f} "
                                 "GiB), timed by HIP events around its launch inside the library",
              "host": "nxec_encode_objects_ex(NXEC_OBJECTS_ASYNC): the host plan of step i + 1 overlaps step i",
              "md5_chain_floor": {"longest_slot_steps": longest, "us_per_step": round(MD5_STEP_US, 3),
                                  "ms": round(longest * MD5_STEP_US / 1e3, 2),
                                  "note": "one lane's MD5 chain per chunk, a slot's requests back to back: the "
                                          "longest slot's 256-byte steps x the bare chain's step time "
                                          "(profiles/r02_encode_md5_role_probes.log)"}}
    return Workload("files", "GiB/s multi-file write (encode+MD5), RS(10,4), 1 MiB max chunk, device-resident",
                    config, ops, [arena, par, tail, md5],
                    "k_files_md5<10> (encode_objects_ex(TAIL_INPLACE | ASYNC): one launch codes and hashes every "
                    "stripe, last stripes read in place with their partial chunk masked and stored to the tail arena)",
                    total, roof_bytes=kernel_bytes,
                    kernel_timer=(lambda: ctx.kernel_timing(True), ctx.kernel_time))


CONFIG1 = ((6, 4, 1 << 20, "RS(4,2) read as (n,k)=(6,4), 4 MiB file, 1 MiB chunks"),
           (4, 2, 2 << 20, "literal sample storage_class.ini (n,k)=(4,2), 4 MiB file, 2 MiB chunks"))


def wl_config1(args, ctx, stream, rank):
    """Config 1: a 4 MiB file, one stripe, in both readings of RS(4,2) (SURVEY
    §0): (n,k)=(6,4) with 1 MiB chunks and the sample's literal (4,2) with
    2 MiB chunks.  One step = per geometry one encode launch and one
    (n-k)-erasure recover launch over the single stripe (device-resident; a
    single stripe is launch-latency bound, not HBM bound).  The CPU legs of
    the same file (reference base C, SIMD port, per-stripe GPU host path) are
    in cpu_baseline.by_config."""
    ops, bufs = [], []
    for n, k, cs, _ in CONFIG1:
        buf = nxec.DeviceBuffer(n * cs)
        buf.fill_random(0x5EED + n + rank)
        lost = list(range(n - k))
        ops.append((f"encode_{n}_{k}", lambda i, b=buf, n=n, k=k, cs=cs: ctx.rs_encode(n, k, b.ptr, cs, n * cs, cs, 1,
                                                                                           stream), (n) * cs))
        ops.append((f"recover_{n}_{k}", lambda i, b=buf, n=n, k=k, cs=cs, f=lost: ctx.rs_recover(
            n, k, f, b.ptr, cs, n * cs, cs, 1, stream), (k + len(lost)) * cs))
        bufs.append(buf)
    config = {"workload": "config 1: 4 MiB file = one stripe, (n,k)=(6,4) 1 MiB chunks and literal (4,2) 2 MiB "
                          "chunks; encode + (n-k)-erasure recover per geometry",
              "geometries": [g[3] for g in CONFIG1],
              "byte_accounting": "encode n*cs + recover (k+e)*cs per stripe"}
    return Workload("config1", "GiB/s RS(4,2) 4 MiB-file encode+decode (config 1), device-resident", config, ops,
                    bufs, "k_mul_vec (single-stripe encode launch, latency bound)", 1)


def cpu_baseline_config1(args):
    """Config 1 on the host: each geometry's 4 MiB file written (RSCode::encode
    with the rs.cc:80 copy) and read back with the first n-k chunks lost
    (RSCode::decode: all k rows of the k x k inverse, rs.cc:196,228-230), one
    file per call on one thread (the proxy codes a file's stripes in
    sequence), by the reference's ISA-L base C and the SIMD port; plus the
    same per-file calls through libnxec's host-buffer entry point
    (nxec_encode_host, the path RSCode::encode/decode take) for comparison."""
    import numpy as np

    import oracle

    level = oracle.simd_level()
    ref = oracle.RefISAL() if oracle.ref_available() else None
    out = {}
    for n, k, cs, label in CONFIG1:
        e = n - k
        enc = nxec.gen_rs_matrix(n, k)[k:]
        ids, _, _ = nxec.rs_plan(n, k, list(range(e)), False)
        ids = ids[:k]
        inv = nxec.decode_matrix(n, k, ids, list(range(k)))
        data = oracle.fill_bytes(k * cs, 4242 + n).reshape(1, k, cs)
        chunks = np.zeros((1, n, cs), dtype=np.uint8)
        dec = np.zeros((1, k, cs), dtype=np.uint8)
        file_bytes = (n + 2 * k) * cs  # write n*cs + read (k survivors in, k out)

        def timed(fn, min_s=0.5):
            fn()
            reps, t0 = 0, time.perf_counter()
            while reps == 0 or time.perf_counter() - t0 < min_s:
                fn()
                reps += 1
            return (time.perf_counter() - t0) / reps

        def port():
            oracle.simd_rscode_encode_range(level, n, k, cs, 0, 1, data, chunks, enc)
            oracle.simd_rscode_decode_range(level, n, k, cs, 0, 1, chunks, ids, inv, dec)

        res = {"file_ms_port_1t": round(timed(port) * 1e3, 3)}
        if ref is not None:
            def base_c():
                ref.encode(enc, list(data[0]), list(chunks[0, k:]))
                ref.encode(inv, [chunks[0, i] for i in ids], list(dec[0]))
            res["file_ms_reference_base_c_1t"] = round(timed(base_c) * 1e3, 3)

        def gpu_host():
            nxec.encode_host(enc, list(data[0]))
            nxec.encode_host(inv, [chunks[0, i] for i in ids])
        res["file_ms_gpu_host_path"] = round(timed(gpu_host) * 1e3, 3)
        for key in list(res):
            res[key.replace("file_ms", "GiB_s")] = round(file_bytes / (res[key] * 1e-3) / GIB, 3)
        res["bytes_per_file"] = file_bytes
        out[label] = res
    return out


WORKLOADS = {"rs10_4": wl_rs10_4, "decode_full": wl_decode_full, "repair12": wl_repair12, "mixed16": wl_mixed16, "write14": wl_write14,
             "object": wl_object, "files": wl_files, "config1": wl_config1}


def launch_local_ranks(argv, world):
    """`bench.py --gpus N` outside torch.distributed.run: start N fresh rank
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, the same argv),
    one per GPU, before this process has imported the package or touched a
    GPU.  Rank 0's JSON line is forwarded; the exit status is non-zero if any
    rank fails (the others are then stopped: a rank blocked in a barrier would
    never finish)."""
    import signal
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # rank 0's stdout is the result; the others' go to stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    failed = None
    live = set(range(world))
    out0 = b""
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0 and failed is None:
                failed = (r, rc)
                for q in live:  # exact PIDs this launcher started
                    try:
                        procs[q].send_signal(signal.SIGTERM)
                    except OSError:
                        pass
        if live:
            time.sleep(0.05)
    out0 = procs[0].stdout.read()
    sys.stdout.write(out0.decode(errors="replace"))
    sys.stdout.flush()
    if failed is not None:
        print(f"bench launcher: rank {failed[0]} exited with status {failed[1]}", file=sys.stderr)
        return failed[1] if failed[1] > 0 else 1
    return 0


def group_devices(members, visible):
    """Device of each nxec_group member: member i on GPU i, round-robin when
    fewer GPUs are visible (the one-GPU box rehearses an 8-member group)."""
    return [i % max(1, visible) for i in range(members)]


def group_measure(args):
    """--group: the one-process deployment of SURVEY §8e ("one host thread +
    hipSetDevice + streams per GPU"): an nxec_group of N contexts, member i
    owning its own args.stripes-stripe batch on device i (weak scaling, as the
    ranks), each step the headline's encode + recover (rotating patterns)
    through nxec_group_rs_{encode,recover}_stripes_async -- each member's
    long-lived thread queues both launches on its stream, one nxec_group_wait
    after the timed steps (the ranks' pattern: queue every step, sync once).  Verified as the ranks' run: the
    batches' checksums survive the timed steps, and erased chunks of every
    member come back.  Aggregate user-visible GiB/s of all members."""
    n, k, cs, ns = args.n, args.k, args.chunk, args.stripes
    p, e = n - k, len(PATTERNS[0])
    devices = group_devices(args.gpus, nxec.device_count())
    # the table's layout for "tuned" too (the calibration runs on one context)
    cst, stripe, lay = layout(argparse.Namespace(**dict(vars(args), layout="auto" if args.layout == "tuned"
                                                        else args.layout)), n, cs)
    g = nxec.Group(devices)
    bufs = []
    for i, d in enumerate(devices):
        nxec.set_device(d)
        b = nxec.DeviceBuffer(ns * stripe)
        b.fill_random(0x6A0 + 7919 * i)
        bufs.append(b)
    ptrs, counts = [b.ptr for b in bufs], [ns] * len(devices)
    g.rs_encode(n, k, ptrs, cst, stripe, cs, counts)

    def sums():
        out = []
        for d, b in zip(devices, bufs):
            nxec.set_device(d)
            out.append(b.checksum())
        return out

    def step(i):  # queued on every member's thread and stream; as the ranks, one wait after the steps
        g.rs_encode_async(n, k, ptrs, cst, stripe, cs, counts)
        g.rs_recover_async(n, k, PATTERNS[i % len(PATTERNS)], ptrs, cst, stripe, cs, counts)

    for i in range(max(1, args.warmup)):
        step(i)
    g.wait()
    want = sums()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    g.wait()
    dt = time.perf_counter() - t0
    verified = sums() == want
    # erase the third pattern's chunks in every member's batch for real, rebuild them
    for d, b in zip(devices, bufs):
        nxec.set_device(d)
        for c in PATTERNS[2]:
            b.memset2d(0, c * cst, stripe, cs, ns)
    nxec.device_sync()
    destroyed = all(a != w for a, w in zip(sums(), want))
    g.rs_recover(n, k, PATTERNS[2], ptrs, cst, stripe, cs, counts)
    verified = verified and destroyed and sums() == want
    step_bytes = len(devices) * ns * ((k + p) + (k + e)) * cs
    for d, b in zip(devices, bufs):
        nxec.set_device(d)
        b.free()
    g.close()
    return {"value": round(step_bytes * args.steps / dt / GIB, 2), "unit": "GiB/s", "members": len(devices),
            "devices": devices, "stripes_per_member": ns, "steps": args.steps, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "verified": verified, "layout": lay,
            "note": "one process, nxec_group: a long-lived host thread + context per member, encode + recover "
                    "queued every step, one group wait after the steps (as the ranks sync once); "
                    "encode (k+p)*cs + recover (k+e)*cs per stripe as the headline"}


def dry_run(args):
    """Launcher/rendezvous check without a GPU: the ranks meet over gloo, take
    the same barrier + max-over-ranks + sum reductions as a real run, and rank
    0 prints the line shape a real run would (no compute, value null)."""
    from nexoedge_amd.dist import RankGroup

    if os.environ.get("RANK") == os.environ.get("NXEC_DRY_RUN_FAIL_RANK", "-"):
        sys.exit(3)  # launcher test: this rank dies before the rendezvous
    grp = RankGroup()
    grp.barrier()
    t = 0.001 * (grp.rank + 1)
    elapsed = grp.max(t)
    ranks = grp.sum(1.0)
    if grp.rank == 0:
        line = {"metric": "dry-run", "value": None, "n_gpus": grp.world, "ranks_seen": int(ranks),
                "max_elapsed_s": elapsed, "steps": args.steps, "warmup": args.warmup}
        if args.group:  # the one-process deployment's plan: member i on device i, its own stripe batch
            line["group"] = {"members": args.gpus, "devices": group_devices(args.gpus, args.gpus),
                             "stripes_per_member": args.stripes}
        print(json.dumps(line), flush=True)
    grp.close()


def main():
    global nxec
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_local_ranks(sys.argv[1:], args.gpus))
    if args.dry_run:
        return dry_run(args)
    import nexoedge_amd  # noqa: F401  (load libnxec before torch: one HIP runtime)
    from nexoedge_amd import nxec as _nxec
    from nexoedge_amd.dist import RankGroup

    nxec = _nxec
    grp = RankGroup()
    world, rank, local = grp.world, grp.rank, grp.local_rank
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one rank per GPU; more ranks than visible GPUs share them round-robin
    # (only for rehearsing the multi-rank path on a small box)
    dev = local % max(1, nxec.device_count())
    # before any pinned buffer or host worker thread exists: this rank's host
    # work runs on the CPUs (and first-touch memory) of its GPU's NUMA node
    # (the CPU baseline below runs on the process's original CPUs)
    orig_affinity = os.sched_getaffinity(0)
    try:
        numa_node = nxec.bind_thread_numa(dev)
    except nxec.NxecError:
        numa_node = -1
    ctx = nxec.Context(dev)
    stream = ctx.stream
    wl = WORKLOADS[args.workload](args, ctx, stream, rank)
    step_bytes = sum(b for _, _, b in wl.ops)
    nops = len(wl.ops)

    def step(i, evs=None):
        for oi, (_, fn, _) in enumerate(wl.ops):
            if evs is not None:
                evs[oi].record(stream)
            fn(i)
        if evs is not None:
            evs[nops].record(stream)

    for i in range(max(1, args.warmup)):
        step(i)
    ctx.sync()
    nxec.device_sync()
    # every op is idempotent on a consistent batch (re-encode / recover rewrite
    # the same bytes), so the batch checksum must not change across the timed steps
    sum_before = wl.buffers[0].checksum()

    evs = [[nxec.Event() for _ in range(nops + 1)] for _ in range(args.steps)]
    grp.barrier()
    nxec.device_sync()
    if wl.kernel_timer:
        wl.kernel_timer[0]()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, evs[i])
    ctx.sync()
    nxec.device_sync()
    t1 = time.perf_counter()
    grp.barrier()
    elapsed = grp.max(t1 - t0)
    # the union of the ranks' timed regions (one host, one monotonic clock):
    # ranks sharing a GPU start a little apart, so the first and last run
    # partly alone and max(t1 - t0) is shorter than the window they share
    window = grp.max(t1) + grp.max(-t0)
    total_bytes = grp.sum(float(step_bytes * args.steps))
    numa_nodes = [int(v) for v in grp.gather(numa_node)]
    consistent = wl.buffers[0].checksum() == sum_before and wl.expect_sum in (None, sum_before)
    verified = grp.sum(0.0 if consistent else 1.0) == 0.0
    # outside the timed region: erase chunks for real and rebuild them
    rebuilt = erase_checks(wl, ctx, sum_before)
    verified = grp.sum(0.0 if verified and all(rebuilt.values()) else 1.0) == 0.0

    # on-box copy ceiling: hipMemcpyDtoD of 16 GiB inside the
    # workload buffer, after the checksum above (it overwrites data)
    ceiling = None
    if rank == 0 and wl.buffers[0].nbytes >= (32 << 30):
        half = 16 << 30
        e0, e1 = nxec.Event(), nxec.Event()
        wl.buffers[0].copy_within(half, 0, half, stream)  # warm
        e0.record(stream)
        for _ in range(3):
            wl.buffers[0].copy_within(half, 0, half, stream)
        e1.record(stream)
        ctx.sync()
        ms = e0.elapsed_ms(e1) / 3
        ceiling = {"d2d_memcpy_GB_s": round(2 * half / (ms * 1e-3) / 1e9, 1),
                   "note": "hipMemcpyDtoD 16 GiB, read+write bytes counted"}

    # per-op event-timed durations on the launch stream
    op_ms = [sum(evs[i][oi].elapsed_ms(evs[i][oi + 1]) for i in range(args.steps)) / args.steps for oi in range(nops)]

    result = None
    if rank == 0:
        # roofline of the dominant kernel: algorithmic bytes per launch / event-timed launch duration
        # (averaged over its launches in a step when several ops run it)
        ro = wl.ops[:wl.roof_ops]
        b0 = sum(b for _, _, b in ro) // len(ro)
        ms0 = sum(op_ms[:wl.roof_ops]) / len(ro)
        kt = None
        if wl.kernel_timer:
            kms, kn = wl.kernel_timer[1]()
            kt = {"launches": kn, "source": "nxec_kernel_time: HIP events inside libnxec around the kernel's launch"}
            b0, ms0 = wl.roof_bytes, kms / max(kn, 1)
        gbs0 = b0 / (ms0 * 1e-3) / 1e9
        traffic, traffic_src = load_traffic(args, wl.name, b0)
        result = {
            "metric": wl.metric,
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
            "verified": verified,
            "verified_rebuilds": rebuilt or None,
            "config": dict(wl.config, parallelism=f"stripe-sharded x{world}, no collectives"),
            "numa_node_per_rank": numa_nodes,
            "ranks_window": None if world == 1 else {
                "value": round(total_bytes / window / GIB, 2), "ms_per_step": round(window / args.steps * 1e3, 3),
                "note": "latest end - earliest start over the ranks (one host's monotonic clock): the aggregate "
                        "over the window the ranks share; `value` is the contract's max over ranks of each one's own "
                        "timed region"},
            "roofline": {
                "bound": "hbm",
                "achieved": round(gbs0, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(gbs0 / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "lib_sha16": lib_sha16(),
                "kernel": wl.roof_kernel,
                "bytes_per_launch": b0,
                "avg_launch_ms": round(ms0, 4),
            },
            "ops": {name: {"avg_ms": round(ms, 4), "bytes": b, "GB_s": round(b / (ms * 1e-3) / 1e9, 1),
                           "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                    for (name, _, b), ms in zip(wl.ops, op_ms)},
        }
        if kt:
            result["roofline"]["kernel_timing"] = kt
        if world > nxec.device_count():
            result["roofline"]["shared_device"] = (
                f"{world} ranks on {nxec.device_count()} GPU(s), round-robin (a rehearsal of the multi-rank path): "
                "each launch ran beside the other ranks' launches, so the per-launch rate is not the kernel's")
        if ceiling:
            result["roofline"]["on_box_ceiling"] = ceiling
        if wl.name == "rs10_4":
            k, cs = args.k, args.chunk
            result["user_data_gib_s"] = round(2 * wl.stripes * k * cs * args.steps * world / elapsed / GIB, 2)
    headline_n1 = rank == 0 and world == 1 and wl.name == "rs10_4"
    if args.host_inclusive and world > 1 and wl.name == "rs10_4":
        # every rank at once: the host-resident encode over each GPU's own link
        hi = host_inclusive_ranks(ctx, grp, args.n, args.k, args.chunk)
        if rank == 0:
            result["host_inclusive"] = hi
    if args.host_inclusive and headline_n1:
        result["host_inclusive"] = host_inclusive(ctx, args.n, args.k, args.chunk)
    if args.host_inclusive and wl.name == "rs10_4":
        # the unmodified drop-in over every visible GPU (one process, the
        # default pool), rank 0 only while the other ranks wait
        grp.barrier()
        if rank == 0:
            result.setdefault("host_inclusive", {})["dropin_pool"] = dropin_pool_rate(orig_affinity)
        grp.barrier()
    if (headline_n1 or (rank == 0 and world == 1 and wl.name == "config1")) and not args.no_cpu_baseline:
        os.sched_setaffinity(0, orig_affinity)  # the host's CPUs, not only the GPU's node
    if headline_n1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, args.n, args.k, args.chunk)
        if args.host_inclusive:
            result["cpu_baseline"]["write_path_with_md5"] = cpu_write_path(args, args.n, args.k, args.chunk)
    if rank == 0 and world == 1 and wl.name == "config1" and not args.no_cpu_baseline:
        by = cpu_baseline_config1(args)
        first = by[CONFIG1[0][3]]
        ref_v = first.get("GiB_s_reference_base_c_1t")
        result["cpu_baseline"] = {
            "value": ref_v if ref_v is not None else first["GiB_s_port_1t"], "unit": "GiB/s", "cores": 1,
            "kind": "reference" if ref_v is not None else "port",
            "sample": f"one 4 MiB file written and read back, {CONFIG1[0][3]}; both readings in by_config",
            "by_config": by, "host": _host_info()}
    for b in wl.buffers:
        b.free()
    ctx.close()  # before the group leg: no rank keeps streams (hardware queues) on a shared GPU
    if args.group and wl.name == "rs10_4":
        # the one-process deployment over the same GPUs, after the ranks' buffers are gone
        grp.barrier()
        if rank == 0:
            result["group"] = group_measure(args)
        grp.barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)
    grp.close()


def host_inclusive(ctx, n, k, cs, ns=512):
    """Pinned host buffers in and out: the kernel reads the data and writes the
    parity over PCIe (zero copy), and for comparison the staged path (H2D data
    -> encode -> D2H parity, triple-buffered; NXEC_HOST_DIRECT=0)."""
    p = n - k
    hd = nxec.PinnedBuffer(ns * k * cs)
    hp = nxec.PinnedBuffer(ns * p * cs)
    import numpy as np

    hd.array[:] = np.random.default_rng(1).integers(0, 256, size=hd.nbytes, dtype=np.uint8)
    reps = 3

    def rate():
        ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
        return ns * (k + p) * cs / ((time.perf_counter() - t0) / reps) / GIB

    direct = rate()
    os.environ["NXEC_HOST_DIRECT"] = "0"
    try:
        staged = rate()
    finally:
        del os.environ["NXEC_HOST_DIRECT"]
    out = {"encode_GiB_s_(k+p)cs": round(direct, 2), "pcie_bytes_GiB_s": round(direct, 2),
           "encode_staged_GiB_s_(k+p)cs": round(staged, 2), "stripes": ns, "batch": 64,
           "note": "zero copy: the kernel reads/writes the pinned host buffers over PCIe; "
                   "staged: H2D -> kernel -> D2H on three streams (NXEC_HOST_DIRECT=0)"}
    # object write path with MD5 of every chunk (nxec_encode_object_host): the
    # proxy's writeFileStripe coding work for a host-resident object
    hm = nxec.PinnedBuffer(ns * n * 16)
    length = ns * k * cs
    ctx.encode_object_host(n, k, hd.ptr, length, cs, hp.ptr, hm.ptr)
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.encode_object_host(n, k, hd.ptr, length, cs, hp.ptr, hm.ptr)
    dt = (time.perf_counter() - t0) / reps
    out["object_write_md5_GiB_s_user_data"] = round(length / dt / GIB, 2)
    hd.free()
    hp.free()
    hm.free()
    rf = read_from_frames(ctx, n, k, cs, min(ns, 256))
    out["read_frames_decode_GiB_s_user_data"] = rf["pipelined"]
    out["read_frames_decode_legs"] = rf
    out["recover_frames_zero_copy"] = recover_frames_rate(ctx, n, k, cs, min(ns, 128))
    return out


def dropin_pool_rate(affinity, threads="16,64", secs="1.5"):
    """The per-stripe drop-in as an unmodified proxy runs it -- RSCode::decode
    (4 erasures) and CodingUtils::encode per stripe with pageable buffers from
    16 and 64 caller threads sharing one RSCode -- in a child process
    (build/dropin_rate pool, tools/dropin_rate.cc) whose default pool holds a
    context per visible GPU: on an N-GPU node the calls spread
    over N PCIe links.  GiB/s of (k+p)*cs resp. (k+e)*cs per stripe, and the
    calls each pool member served.  Host CPUs: the process's original
    affinity (not only GPU 0's node)."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "dropin_rate")
    if not os.path.exists(exe):
        return {"skipped": "build/dropin_rate not built"}
    mine = os.sched_getaffinity(0)
    os.sched_setaffinity(0, affinity)  # the child inherits it
    try:
        r = subprocess.run([exe, str(1 << 20), secs, "pool", threads], capture_output=True, text=True, timeout=180)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    finally:
        os.sched_setaffinity(0, mine)
    out = {"legs": [], "note": "per-stripe RSCode::decode / CodingUtils::encode, pageable buffers, one process, "
                               "default pool over every visible GPU (NXEC_DEFAULT_DEVICES=all)"}
    for line in r.stdout.splitlines():
        try:
            d = json.loads(line)
        except ValueError:
            continue
        if "pool_members" in d:
            out["pool_members"] = d["pool_members"]
        elif "path" in d:
            out["legs"].append({"path": d["path"], "threads": d["threads"], "GiB_s": d["GiB_s"], "ok": d["ok"]})
    if r.returncode != 0:
        out["error"] = f"rc {r.returncode}: {r.stderr[-300:]}"
    return out


def host_inclusive_ranks(ctx, grp, n, k, cs, ns=256, reps=3):
    """N > 1: every rank runs the zero-copy host-batch encode (pinned data in,
    pinned parity out, its own GPU's PCIe link) at the same time, between two
    barriers; aggregate = all ranks' (k+p)*cs / the slowest rank's time.  A
    rank whose leg fails still joins every collective (reports -1), so one
    failure cannot hang the others."""
    p = n - k
    t, bufs = -1.0, []
    try:
        bufs.append(nxec.PinnedBuffer(ns * k * cs))
        bufs.append(nxec.PinnedBuffer(ns * p * cs))
        hd, hp = bufs
        hd.array[:] = 0x5A
        ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)  # warm
        ready = True
    except Exception:  # noqa: BLE001  (reported, not raised: the ranks must stay in step)
        ready = False
    grp.barrier()
    if ready:
        try:
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.rs_encode_host_batch(n, k, hd.ptr, hp.ptr, cs, ns, 64)
            t = (time.perf_counter() - t0) / reps
        except Exception:  # noqa: BLE001
            t = -1.0
    grp.barrier()
    failed = grp.sum(1.0 if t <= 0 else 0.0)
    tmax = grp.max(t)
    for b in bufs:
        b.free()
    if failed:
        return {"error": f"{int(failed)} rank(s) failed the host-inclusive leg"}
    agg = grp.world * ns * (k + p) * cs / tmax / GIB
    return {"encode_GiB_s_(k+p)cs_all_ranks": round(agg, 2), "per_rank_GiB_s": round(agg / grp.world, 2),
            "ranks": grp.world, "stripes_per_rank": ns, "batch": 64,
            "note": "zero copy over each GPU's own PCIe link, all ranks at once (slowest rank's time)"}


def read_from_frames(ctx, n, k, cs, ns):
    """The proxy read path on received chunk frames (pageable message buffers,
    one per chunk, io.cc:209-216): the k surviving chunks of every stripe
    gathered into HBM, full-output decode of n-k erasures (chunk_manager.cc:
    738-800), the k data chunks scattered into per-chunk host frames.
    `pipelined`: one nxec_decode_frames call (gather of batch b + 1, decode of
    b, scatter of b - 1 at once); `sequential`: the same three steps one after
    the other (nxec_gather_chunks x k, nxec_rs_decode_stripes,
    nxec_scatter_chunks); `gather_only` / `scatter_only`: the two PCIe legs
    alone, to name the limit.  User-data GiB/s (k*cs per stripe)."""
    import numpy as np

    failed = list(range(k - (n - k), k))  # worst case: n-k data chunks lost
    alive = [c for c in range(n) if c not in failed]
    rx = np.random.default_rng(2).integers(0, 256, size=ns * n * cs, dtype=np.uint8)
    tx = np.empty(ns * k * cs, dtype=np.uint8)
    st, dec = nxec.DeviceBuffer(ns * n * cs), nxec.DeviceBuffer(ns * k * cs)
    in_frames = [rx.ctypes.data + (s * n + c) * cs for s in range(ns) for c in range(n)]
    out_frames = [tx.ctypes.data + i * cs for i in range(ns * k)]
    rxf = {c: [in_frames[s * n + c] for s in range(ns)] for c in alive}

    def gather():
        for cid in alive:
            ctx.gather_chunks(rxf[cid], cs, st.ptr + cid * cs, n * cs)

    def scatter():
        ctx.scatter_chunks(dec.ptr, cs, out_frames, cs)

    def sequential():
        gather()
        ctx.rs_decode(n, k, failed, st.ptr, cs, n * cs, dec.ptr, cs, k * cs, cs, ns)
        scatter()

    def pipelined():
        ctx.decode_frames(n, k, failed, in_frames, out_frames, cs, ns)

    import resource

    cpu = {}

    def rate(fn, reps=3):
        """user-data GiB/s of fn, and the process's CPU seconds (every thread:
        the calling thread, the host copy pool, the pipeline's stage threads)
        per wall second -- against the cgroup quota, the share of the box's CPU
        budget the leg used (name the bound)"""
        fn()
        r0, c0 = resource.getrusage(resource.RUSAGE_SELF), _cgroup_cpu_stat()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        ctx.sync()
        wall = time.perf_counter() - t0
        r1, c1 = resource.getrusage(resource.RUSAGE_SELF), _cgroup_cpu_stat()
        used = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
        cpu[fn.__name__] = {"cpu_s_per_call": round(used / reps, 4), "cpus_busy": round(used / wall, 2),
                            "sys_share": round((r1.ru_stime - r0.ru_stime) / max(used, 1e-9), 3)}
        if c0 and c1:  # the cgroup held the box's threads back this long (quota exhausted in a period)
            cpu[fn.__name__]["cgroup_throttled_ms"] = round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 1)
            cpu[fn.__name__]["cgroup_periods_throttled"] = c1.get("nr_throttled", 0) - c0.get("nr_throttled", 0)
            cpu[fn.__name__]["cgroup_periods"] = c1.get("nr_periods", 0) - c0.get("nr_periods", 0)
        return round(ns * k * cs / (wall / reps) / GIB, 2)

    out = {"pipelined": rate(pipelined), "sequential": rate(sequential), "gather_only": rate(gather),
           "scatter_only": rate(scatter), "stripes": ns, "erasures": failed}
    out["cpu"] = cpu
    out["cgroup_cpu_quota"] = _host_info().get("cgroup_cpu_quota")
    out["host_threads"] = int(os.environ.get("NXEC_HOST_THREADS", "8"))
    # the pipelined call wrote the original data chunks (parity-free check: the
    # survivors were random, so compare against the sequential path's output)
    want = tx.copy()
    pipelined()
    out["pipelined_equals_sequential"] = bool(np.array_equal(tx, want))
    st.free()
    dec.free()
    return out


def recover_frames_rate(ctx, n, k, cs, ns):
    """nxec_rs_recover_frames on pinned frames (a registered receive pool): one
    kernel reads the k survivors and writes the n-k lost data chunks over PCIe.
    User data = the k data chunks per stripe now complete in host memory."""
    e = n - k
    failed = list(range(k - e, k))
    buf = nxec.PinnedBuffer(ns * n * cs)
    buf.array[:] = 7
    frames = [buf.ptr + i * cs for i in range(ns * n)]
    ctx.rs_recover_frames(n, k, failed, frames, cs, ns)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.rs_recover_frames(n, k, failed, frames, cs, ns)
    dt = (time.perf_counter() - t0) / reps
    buf.free()
    return {"user_data_GiB_s": round(ns * k * cs / dt / GIB, 2), "pcie_GiB_s_(k+e)cs": round(ns * (k + e) * cs / dt / GIB, 2),
            "stripes": ns, "failed": failed}


def cpu_write_path(args, n, k, cs):
    """CPU write path of the reference per stripe: encode (SIMD stand-in) + MD5
    of all n chunks (OpenSSL via hashlib, GIL released), threads over stripes;
    user-data GiB/s, the same unit as object_write_md5_GiB_s_user_data."""
    import concurrent.futures as cf
    import hashlib

    import numpy as np

    import oracle

    threads = args.cpu_threads or len(os.sched_getaffinity(0))
    p, ns = n - k, max(min(args.cpu_stripes, 64), threads)
    enc = nxec.gen_rs_matrix(n, k)[k:]
    data = oracle.fill_bytes(ns * k * cs, 7).reshape(ns, k, cs)
    parity = np.zeros((ns, p, cs), dtype=np.uint8)

    def work(lo, hi):
        for s in range(lo, hi):
            oracle.simd_encode(enc, list(data[s]), list(parity[s]))
            for c in list(data[s]) + list(parity[s]):
                hashlib.md5(c).digest()

    bounds = [(ns * t // threads, ns * (t + 1) // threads) for t in range(threads)]
    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda b: work(*b), bounds))
        dt = time.perf_counter() - t0
    return {"value": round(ns * k * cs / dt / GIB, 3), "unit": "GiB/s user data", "cores": threads, "kind": "port",
            "sample": f"{ns} RS({n},{k}) stripes of {cs >> 10} KiB chunks: SIMD encode + hashlib MD5 of all "
                      f"{n} chunks per stripe, {threads} threads"}


if __name__ == "__main__":
    main()
