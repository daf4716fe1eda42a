#!/usr/bin/env bash
# A/B of build/ab/libnxec_{new,old}.so (global-address-space streaming
# accesses in every kernel vs flat in the gather forms): the headline bench
# with its host-inclusive legs, the unfused multi-file write, and the
# per-stripe drop-in at one caller.  First failure stops.
set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
AB_CMD='python bench.py --steps 20 --warmup 2 --no-cpu-baseline | python3 -c "import json,sys; d=json.load(sys.stdin); h=d[\"host_inclusive\"]; print(\"headline\", d[\"value\"], d[\"roofline\"][\"frac\"], \"zc_encode\", h[\"encode_GiB_s_(k+p)cs\"], \"obj_md5\", h[\"object_write_md5_GiB_s_user_data\"], \"frames\", h[\"recover_frames_zero_copy\"][\"user_data_GiB_s\"])"; NXEC_FUSED_MD5=0 python bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive | python3 -c "import json,sys; d=json.load(sys.stdin); print(\"files_unfused\", d[\"ms_per_step\"])"; DROPIN_AGENT_THREADS=1 build/dropin_rate 1048576 1 all 1 | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d[\"path\"][:40], d.get(\"buffers\",\"\"), d.get(\"GiB_s\", d.get(\"GiB_s_user_data\")))"' AB_T=400 bash tools/ab_lib.sh
