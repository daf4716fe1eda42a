#!/usr/bin/env bash
# GPU-box sequence: parity tests -> smoke -> bench (+ optional rocprofv3 stats).
# Each GPU step has its own time limit; a crash/timeout/abort (rc >= 2 for
# pytest, != 0 otherwise) stops the sequence -- no retries.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
nproc > $OUT/host.txt; lscpu | grep -E "Model name|^CPU\(s\)" >> $OUT/host.txt
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_T:-700} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log
  [ $rc -le 1 ] || stop pytest $rc
fi
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || stop smoke $?
tail -1 $OUT/smoke.log
timeout -k 10 ${BENCH_T:-400} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || stop bench $?
cat $OUT/bench.json
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof_bench.json 2> $OUT/prof.err || stop rocprof $?
  find $OUT/prof -name "*stats*" | head
fi
if [ -n "${PMC:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-host-inclusive > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || stop pmc_$c $?
  done
fi
