#!/usr/bin/env python3
"""Probe: where the multi-file write (nxec_encode_objects -> k_files_md5)
spends its steps.  Several 4096-file batches, each timed in one process:

  full10    every file exactly one full RS(10,4) stripe (10 MiB): no tails
  even5     every file 5 MiB: one last stripe each, 512 KiB chunks, all whole
  ragged    every file's length uniform in [1 B, 10 MiB): one ragged last stripe each
  mix       bench.py's batch: uniform in [1 B, 20 MiB] (full + ragged)
  al16/al8  last stripes of whole chunks only, chunk starts 16-byte aligned /
            all 8 bytes off (the cost of misaligned loads)

each with the tail arena written whole (default) and with
NXEC_OBJECTS_TAIL_INPLACE (only each last stripe's partial data chunk);

The slot plan is LPT over request steps (plan_files_slots, restated here on
the host to get the longest slot); ms / longest-slot-steps is the cost of one
256-byte step of a workgroup, comparable with k_mul_md5's (13.8 ms / 4096)."""
import heapq
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexoedge_amd import nxec  # noqa: E402

n, k, M = 14, 10, 1 << 20
p = n - k
STEP = 256
ctx = nxec.Context(0)
CUS, SMAX = 256, min(16, 256 // n)


def requests(lengths):
    out = []
    for L in lengths:
        ns, nf, cl = nxec.object_layout(n, k, L, M)
        out += [M] * nf + ([cl] if ns > nf else [])
    return out


def longest_slot(req_lens):
    steps = sorted(((L + STEP - 1) // STEP for L in req_lens), reverse=True)
    G = len(steps) if len(steps) <= CUS * SMAX else CUS * SMAX
    if G == len(steps):
        return max(steps)
    heap = [(0, g) for g in range(G)]
    for s in steps:
        load, g = heapq.heappop(heap)
        heapq.heappush(heap, (load + s, g))
    return max(l for l, _ in heap)


def run(name, lengths, flags=0, reps=5):
    offs = np.concatenate([[0], np.cumsum([(L + 15) // 16 * 16 for L in lengths])])
    arena = nxec.DeviceBuffer(int(offs[-1]))
    arena.fill_random(77)
    total, tail_bytes = nxec.objects_layout(n, k, lengths, M)
    par = nxec.DeviceBuffer(total * p * M)
    tail = nxec.DeviceBuffer(max(tail_bytes, 16))
    md5 = nxec.DeviceBuffer(total * n * 16)
    ptrs = [arena.ptr + int(o) for o in offs[:-1]]

    def once():
        ctx.encode_objects(n, k, ptrs, lengths, M, par.ptr, tail.ptr, md5.ptr, flags=flags)

    once()
    ctx.sync()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        once()
        ctx.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    ms = sorted(ts)[len(ts) // 2]
    req = requests(lengths)
    ls = longest_slot(req)
    print(f"{name:8s} {'inplace' if flags else 'copy   '} files {len(lengths)} requests {len(req)} tails {sum(1 for L in lengths if L % (k * M))} "
          f"longest slot {ls} steps: {ms:.3f} ms, {ms / ls * 1e3:.3f} us/step, "
          f"tail arena {tail_bytes / 2**30:.2f} GiB", flush=True)
    for b in (arena, par, tail, md5):
        b.free()


rng = np.random.default_rng(1234)
sets = {
    "full10": [k * M] * 4096,
    "even5": [k * M // 2] * 4096,
    "ragged": [int(x) for x in rng.integers(1, k * M, size=4096)],
    "mix": [int(x) for x in np.random.default_rng(1234).integers(1, 2 * k * M + 1, size=4096)],
    # whole last-stripe chunks only (length = k * cl), chunk starts 16-byte
    # aligned (cl % 16 == 0) or all misaligned by 8: the cost of misaligned loads
    "al16": [k * 16 * int(x) for x in np.random.default_rng(99).integers(1, M // 16, size=4096)],
    "al8": [k * (16 * int(x) + 8) for x in np.random.default_rng(99).integers(1, M // 16, size=4096)],
}
which = sys.argv[1:] or list(sets)
for name in which:
    for flags in (0, nxec.OBJECTS_TAIL_INPLACE):  # tail arena: every data chunk / only the partial one
        run(name, sets[name], flags)
