# one-off GPU call: layout calibration tests, then the tuned config-5 lines (twice)
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "layout or frames" > $OUT/pytest_layout.log 2>&1 || { tail -30 $OUT/pytest_layout.log; exit 1; }
tail -2 $OUT/pytest_layout.log
for r in 1 2; do
for c in 262144 4194304 1048576 65536; do
  timeout -k 10 300 python bench.py --workload mixed16 --chunk $c --layout tuned --steps 20 --no-cpu-baseline --no-host-inclusive > $OUT/tuned_line.json 2>> $OUT/tuned.err || { tail -20 $OUT/tuned.err; exit 1; }
  cat $OUT/tuned_line.json >> $OUT/tuned2.jsonl
  python3 -c "import json; d=json.load(open('$OUT/tuned_line.json')); print($c, d['roofline']['frac'], d['ops']['decode']['frac'], d['config']['layout'][:80])"
done
done
