#!/usr/bin/env bash
# Round measurement set: headline bench + rocprof stats, config sweeps.  Each
# step has its own time limit; the first failure ends the call.
set -u
OUT=gpurun_out/final
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || stop bench $?
cat $OUT/bench.json | head -c 600; echo
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof_bench.json 2> $OUT/prof.err || stop rocprof $?
for cs in 65536 262144 1048576 4194304; do
  timeout -k 10 300 python bench.py --workload mixed16 --chunk $cs --no-cpu-baseline >> $OUT/configs.jsonl 2>> $OUT/configs.err || stop mixed16_$cs $?
done
for f in 0 15; do
  timeout -k 10 300 python bench.py --workload repair12 --failed $f --no-cpu-baseline >> $OUT/configs.jsonl 2>> $OUT/configs.err || stop repair12_$f $?
done
timeout -k 10 300 python bench.py --layout recover --no-cpu-baseline --no-host-inclusive >> $OUT/configs.jsonl 2>> $OUT/configs.err || stop recover_layout $?
timeout -k 10 300 python bench.py --workload object --no-cpu-baseline >> $OUT/configs.jsonl 2>> $OUT/configs.err || stop object $?
timeout -k 10 300 python bench.py --workload files --no-cpu-baseline >> $OUT/configs.jsonl 2>> $OUT/configs.err || stop files $?
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); print(d['metric'][:60], d['value'], d['roofline']['frac'], {k:v['frac'] for k,v in d['ops'].items()})
"
