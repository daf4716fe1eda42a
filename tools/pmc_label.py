#!/usr/bin/env python3
"""Per-dispatch PMC traffic (tools/pmc_dispatch.py) labelled with the bench
op of each dispatch and its algorithmic bytes, as one JSON document for
profiles/.  Usage:
  pmc_label.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR SOURCE_CMD LABEL:BYTES [LABEL:BYTES ...]
LABEL:BYTES pairs are matched to the dispatches in order (repeat the list per
step as the bench issues it)."""
import hashlib
import json
import os
import subprocess
import sys

fdir, wdir, sub, cmd = sys.argv[1:5]
labels = [(a.rsplit(":", 1)[0], a.rsplit(":", 1)[1]) for a in sys.argv[5:]]
out = subprocess.run([sys.executable, __file__.replace("pmc_label.py", "pmc_dispatch.py"), fdir, wdir, sub],
                     capture_output=True, text=True, check=True).stdout
rows = [json.loads(l) for l in out.splitlines() if l.strip()]
# one LABEL:BYTES* pair labels every dispatch the same (workloads whose every
# launch of the kernel moves the same bytes)
if len(labels) == 1 and labels[0][1].endswith("*"):
    labels = labels * len(rows)
labels = [(lab, int(b.rstrip("*"))) for lab, b in labels]
if len(labels) != len(rows):
    sys.exit(f"{len(rows)} dispatches, {len(labels)} labels")
disp = []
for r, (lab, alg) in zip(rows, labels):
    r.update(op=lab, algorithmic_bytes=alg, traffic_over_algorithmic=round(r["hbm_bytes"] / alg, 5),
             frac_of_8TBs_fetch_pass=round(alg / (r["ms_fetch_pass"] * 1e-3) / 8e12, 4))
    disp.append(r)
# the library the passes measured (labelled right after the run, before any rebuild; LIB_SHA16 overrides)
lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nexoedge_amd", "lib", "libnxec.so")
lib_sha16 = os.environ.get("LIB_SHA16") or hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
print(json.dumps({
    "source": f"rocprofv3 --pmc FETCH_SIZE --kernel-trace and --pmc WRITE_SIZE --kernel-trace, separate passes of: {cmd}",
    "lib_sha16": lib_sha16,
    "gfx950_correction": "read_bytes = 2 * FETCH_SIZE * 1024 (FETCH_SIZE counts half the bytes of 16-B/lane streaming "
                         "reads, MI355X_MICROARCH.md HBM); write_bytes = WRITE_SIZE * 1024",
    "note": "ms_fetch_pass is the kernel-trace duration inside the counter pass (profiled clocks run 2-5% lower)",
    "dispatches": disp}, indent=1))
