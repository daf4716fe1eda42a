#!/usr/bin/env bash
# tests + drop-in write leg, then the StripeBatch layout probe and the
# multi-file write A/B (build/ab/libnxec_{new,old}.so, alternating)
set -u
SKIP_BENCH=1 DROPIN=1 DROPIN_T=1,4,16,64 bash tools/gpu_r03.sh || exit $?
timeout -k 10 300 python tools/stripe_batch_layout_probe.py > gpurun_out/stripe_batch_layout.log 2>&1 || { echo "STOP probe rc=$?"; exit 1; }
cat gpurun_out/stripe_batch_layout.log
AB_CMD="python bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive" AB_T=300 bash tools/ab_lib.sh
