#!/usr/bin/env bash
# rocprofv3 kernel stats for BASELINE configs 4 and 5 (bench workloads)
set -u
OUT=gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$tag -o run --output-format csv -- \
    python3 bench.py "$@" --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof_$tag.json 2> $OUT/prof_$tag.err || exit 1
}
run repair12_f0 --workload repair12 --failed 0
run mixed16_1m --workload mixed16 --chunk 1048576
run mixed16_4m --workload mixed16 --chunk 4194304
for t in repair12_f0 mixed16_1m mixed16_4m; do
  echo "== $t"; python3 - "$OUT/prof_$t/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:90]:92s} {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
done
