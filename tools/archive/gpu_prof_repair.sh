#!/usr/bin/env bash
# per-kernel stats of the RS(12,4) CAR repair workload, work-queue vs static tile order
set -u
OUT=gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for mode in queue static; do
  if [ $mode = static ]; then export NXEC_TILE_ORDER=static; else unset NXEC_TILE_ORDER; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rep_$mode -o run --output-format csv -- \
    python3 bench.py --workload repair12 --failed ${FAILED:-0} --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_rep_$mode.json 2> $OUT/prof_rep_$mode.err || exit 1
  echo "== $mode"; f=$(find $OUT/prof_rep_$mode -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 $f | cut -c1-160
done
