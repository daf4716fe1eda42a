# one-off GPU call: decode_full spread (three runs) beside the headline
set -o pipefail
OUT=gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --workload decode_full --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive > $OUT/df.json 2>> $OUT/df.err || { tail -20 $OUT/df.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/df.json')); print('decode_full', d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --no-host-inclusive > $OUT/hl.json 2>> $OUT/df.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/hl.json')); print('headline', d['value'], d['roofline']['frac'])"
