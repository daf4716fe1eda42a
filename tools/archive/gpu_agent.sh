#!/usr/bin/env bash
# Agent-service measurements (fused k_gather_md5 form): parity tests, then
# build/dropin_rate's agent leg (pageable / arena buffers, 1/4/16 callers),
# a traced single-caller run and staging-batch-size A/Bs.  Each GPU step has
# its own time limit; the first failure ends the call.
set -u
OUT=gpurun_out/agent
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_agent_fused.py \
  tests/test_gpu_parity.py -k agent > $OUT/tests.log 2>&1 || stop tests $?
tail -2 $OUT/tests.log
timeout -k 10 200 ./build/dropin_rate 1048576 3 agent > $OUT/rate.jsonl 2>&1 || stop rate $?
cat $OUT/rate.jsonl
NXEC_AGENT_TRACE=1 DROPIN_AGENT_THREADS=1 timeout -k 10 100 ./build/dropin_rate 1048576 1 agent > $OUT/trace1.log 2>&1 || stop trace1 $?
tail -4 $OUT/trace1.log
for mb in ${AGENT_MB:-64 128 512}; do
  echo "batch_mb $mb" >> $OUT/batch_ab.jsonl
  NXEC_AGENT_BATCH_MB=$mb timeout -k 10 200 ./build/dropin_rate 1048576 2 agent >> $OUT/batch_ab.jsonl 2>&1 || stop batch_$mb $?
done
cat $OUT/batch_ab.jsonl
