#!/usr/bin/env bash
# configs 2-5 on one GPU: headline bench, RS(12,4) repair, RS(16,4) chunk-size sweep
set -u
OUT=gpurun_out; mkdir -p $OUT
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline || { echo "bench $* failed rc=$?"; exit 1; }; }
{
run --steps 10 --warmup 2
run --workload repair12 --failed 0 --steps 10 --warmup 2
run --workload repair12 --failed 15 --steps 10 --warmup 2
for c in 65536 262144 1048576 4194304; do run --workload mixed16 --chunk $c --gib 32 --steps 10 --warmup 2; done
} > $OUT/configs.jsonl 2> $OUT/configs.err
python3 - <<'PY'
import json
for l in open("gpurun_out/configs.jsonl"):
    d = json.loads(l)
    print(d["metric"], d["value"], d["verified"], {k: (v["avg_ms"], v["frac"]) for k, v in d["ops"].items()})
PY
