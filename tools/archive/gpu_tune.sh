#!/usr/bin/env bash
# tuning probe + PMC traffic passes (separate --pmc runs, kernel-trace only)
set -u
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 ./tools/microbench/tune_mul ${TUNE_S:-4096} 5 > $OUT/tune.log 2>&1 || { echo "tune rc=$?"; cat $OUT/tune.log; exit 1; }
cat $OUT/tune.log
if [ -n "${PMC:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.err; exit 1; }
  done
  find $OUT -name "*counter_collection*" | head
fi
