#!/usr/bin/env bash
# Round-3 GPU sequence: parity tests -> smoke -> bench -> drop-in write leg
# (writeFileStripe per stripe: GPU digests vs host OpenSSL) -> optional
# rocprofv3 stats.  Each GPU step has its own limit; the first failure stops
# the sequence (no retries).
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
nproc > $OUT/host.txt; lscpu | grep -E "Model name|^CPU\(s\)|NUMA" >> $OUT/host.txt
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_T:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log
  [ $rc -le 1 ] || stop pytest $rc
  [ $rc -eq 0 ] || stop pytest-failures $rc
fi
timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || stop smoke $?
tail -1 $OUT/smoke.log
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 ${BENCH_T:-500} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || stop bench $?
  cat $OUT/bench.json
fi
if [ -n "${DROPIN:-}" ]; then
  for m in 1 0; do
    NXEC_CHUNK_MD5=$m timeout -k 10 300 build/dropin_rate 1048576 ${DROPIN_S:-2} write ${DROPIN_T:-1,4,16,64} \
      > $OUT/dropin_write_md5mode$m.jsonl 2> $OUT/dropin_write_md5mode$m.err || stop dropin$m $?
    cat $OUT/dropin_write_md5mode$m.jsonl
  done
fi
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive ${PROF_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err || stop rocprof $?
  find $OUT/prof -name "*stats*" | head
fi
echo ALL-DONE
