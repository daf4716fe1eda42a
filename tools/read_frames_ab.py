"""Same-box A/B of the pageable-frames read pipeline:
bench.py's read_from_frames (nxec_decode_frames pipelined, the sequential
calls, the gather and scatter legs alone, each with its process CPU seconds
and cgroup throttling) under the library / knobs the environment names.
usage: [NXEC_LIB=...] [NXEC_HOST_LANES=1] [NXEC_HOST_THREADS=N] [FRAMES_BIND=1] python tools/read_frames_ab.py LABEL"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from nexoedge_amd import nxec  # noqa: E402

bench.nxec = nxec
node = -1
if os.environ.get("FRAMES_BIND") == "1":  # this thread and the pools it starts on the GPU's NUMA node
    node = nxec.bind_thread_numa(0)
ctx = nxec.Context(0)
rf = bench.read_from_frames(ctx, 14, 10, 1 << 20, 256)
rf["label"] = sys.argv[1] if len(sys.argv) > 1 else ""
rf["lib"] = os.environ.get("NXEC_LIB", "product")
rf["lanes"] = os.environ.get("NXEC_HOST_LANES", "")
rf["numa_node"] = node
print(json.dumps(rf), flush=True)
ctx.close()
