# one-off GPU call: rocprofv3 kernel stats of the secondary lines (decode_full, files, write14, repair12)
set -o pipefail
OUT=gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in decode_full files write14 repair12; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2_$w -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof2_$w.json 2> $OUT/prof2_$w.err \
    || { tail -20 $OUT/prof2_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/prof2_$w.json')); print('$w', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
