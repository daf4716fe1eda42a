#!/usr/bin/env bash
# World = 8 rehearsal on the one-GPU box (all 8 ranks share device 0): the
# 8-member nxec_group parity test, then bench.py --gpus 8 (the launcher
# spawns 8 ranks: gloo rendezvous, per-rank NUMA binding, erase-and-rebuild
# checks, host_inclusive_ranks) for the headline and the mixed16 stream.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "group_contexts" -x -v --timeout 240 \
  --timeout-method thread > $OUT/pytest_group8.log 2>&1 || stop pytest $?
tail -3 $OUT/pytest_group8.log
timeout -k 10 400 python bench.py --gpus 8 --stripes 512 --steps 10 --warmup 2 \
  > $OUT/bench_n8.json 2> $OUT/bench_n8.err || stop bench_n8 $?
cat $OUT/bench_n8.json
timeout -k 10 400 python bench.py --workload mixed16 --gpus 8 --gib 4 --steps 5 --warmup 1 \
  > $OUT/bench_n8_mixed16.json 2> $OUT/bench_n8_mixed16.err || stop bench_n8_mixed16 $?
cat $OUT/bench_n8_mixed16.json
echo ALL-DONE
