#!/usr/bin/env bash
# GPU tests (full -m gpu), smoke, then the digest-placement A/B of the
# unmodified write path in one process: host / gpu / auto in rotating order,
# 3 rounds, after a warm-up leg (tools/dropin_rate.cc DROPIN_PLACES).
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; stop pytest $?; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || stop smoke $?
  tail -1 $OUT/smoke.log
fi
DROPIN_PLACES=host,gpu,auto DROPIN_REPS=${REPS:-3} timeout -k 10 600 build/dropin_rate 1048576 ${SECS:-1.5} write ${T:-1,4,16,64} \
  > $OUT/dropin_place_ab.jsonl 2> $OUT/dropin_place_ab.err || stop dropin $?
grep summary $OUT/dropin_place_ab.jsonl
timeout -k 10 300 python tools/files_mix_probe.py > $OUT/files_mix.log 2>&1 || stop files_mix $?
cat $OUT/files_mix.log
echo ALL-DONE
