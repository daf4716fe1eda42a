#!/usr/bin/env bash
# Round-3 state of the fused/secondary workloads: files, write14, object
# benches, the StripeBatch layout probe, and rocprofv3 kernel stats of the
# headline bench.  Each GPU step has its own limit; the first failure stops.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
for w in files write14 object; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || stop bench_$w $?
  cat $OUT/bench_$w.json
done
timeout -k 10 300 python tools/stripe_batch_layout_probe.py > $OUT/stripe_batch_layout.log 2>&1 || stop probe $?
cat $OUT/stripe_batch_layout.log
if [ -z "${SKIP_PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof_bench.json 2> $OUT/prof.err || stop rocprof $?
  python3 - "$OUT/prof/run_kernel_stats.csv" <<'PY'
import csv, glob, sys
f = sys.argv[1]
if not glob.glob(f):
    f = (glob.glob("gpurun_out/prof/**/*kernel_stats.csv", recursive=True) or [f])[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:90]:92s} {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
fi
echo ALL-DONE
