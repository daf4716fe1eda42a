#!/usr/bin/env bash
# The multi-file write with the last-stripe pad copy folded into k_files_md5:
# its parity tests (fused vs separate launches, vs the oracle / hashlib),
# then the files bench fused and unfused (NXEC_FUSED_MD5=0), then rocprofv3
# kernel stats of the fused bench.  First failure stops.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "encode_objects or encode_decode_object or objects" > $OUT/pytest_files.log 2>&1 || { tail -30 $OUT/pytest_files.log; stop pytest $?; }
tail -2 $OUT/pytest_files.log
for v in 1 0 1 T; do
  if [ $v = T ]; then export NXEC_FILES_TAIL=0; fi
  NXEC_FUSED_MD5=${v/T/1} timeout -k 10 300 python bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive \
    > $OUT/bench_files_fused$v.json 2> $OUT/bench_files_fused$v.err || stop bench$v $?
  python3 -c "import json; d=json.load(open('$OUT/bench_files_fused$v.json')); print('fused=$v', d['ms_per_step'], d['roofline']['frac'], d['verified'])"
done
unset NXEC_FILES_TAIL
if [ -z "${SKIP_PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_files -o run --output-format csv -- \
    python3 bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof_files.json 2> $OUT/prof_files.err || stop rocprof $?
  python3 - "$OUT/prof_files/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:90]:92s} {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
fi
echo ALL-DONE
