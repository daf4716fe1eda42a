#!/usr/bin/env python3
"""Stripe-group (tile order) sweep for RS(10,4) 4096 x 1 MiB recovers in the
packed layout: runs tools/recover_patterns.py's timing for a few patterns
under NXEC_STRIPE_GROUP = 1 .. 32 (each value in a fresh process: the env is
read per launch, but keep processes independent)."""
import os
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
code = r'''
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath("%s"))))
from nexoedge_amd import nxec
n, k, cs, ns = 14, 10, 1 << 20, 4096
ctx = nxec.Context(0); st = ctx.stream
buf = nxec.DeviceBuffer(ns * n * cs); buf.fill_random(5)
ctx.rs_encode(n, k, buf.ptr, cs, n * cs, cs, ns, st); ctx.sync()
for name, f in [("encode", None), ("1,4,11,13", [1, 4, 11, 13]), ("0,2,4,6", [0, 2, 4, 6]), ("1,2,3,4", [1, 2, 3, 4]), ("0-3", [0, 1, 2, 3])]:
    go = (lambda: ctx.rs_encode(n, k, buf.ptr, cs, n * cs, cs, ns, st)) if f is None else (lambda f=f: ctx.rs_recover(n, k, f, buf.ptr, cs, n * cs, cs, ns, st))
    go(); e0, e1 = nxec.Event(), nxec.Event(); e0.record(st)
    for _ in range(5): go()
    e1.record(st); ctx.sync(); ms = e0.elapsed_ms(e1) / 5
    b = ns * (k + (n - k if f is None else len(f))) * cs
    print(f"sg {os.environ.get('NXEC_STRIPE_GROUP', 'auto'):>4s} {os.environ.get('NXEC_TILE_ORDER', 'queue'):6s} {name:10s} {ms:7.3f} ms frac8T {b / ms / 1e6 / 8e3:.3f}", flush=True)
buf.free(); ctx.close()
''' % os.path.join(here, "x")
for sg in sys.argv[1:] or ["auto", "1", "2", "4", "16", "32"]:
    env = dict(os.environ)
    if sg == "static":
        env["NXEC_TILE_ORDER"] = "static"
    elif sg != "auto":
        env["NXEC_STRIPE_GROUP"] = sg
    r = subprocess.run([sys.executable, "-c", code], env=env, timeout=120)
    if r.returncode:
        sys.exit(r.returncode)
