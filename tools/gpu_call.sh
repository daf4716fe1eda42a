set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python bench.py --gpus 8 --group --stripes 512 --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive > $OUT/group8.json 2> $OUT/group8.err || { tail -20 $OUT/group8.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/group8.json')); print('group8', d['value'], d['n_gpus'], d.get('verified'), json.dumps(d.get('group'))[:400])"
for r in 1 2; do
for lay in auto recover tuned; do
  timeout -k 10 300 python bench.py --layout $lay --steps 30 --no-cpu-baseline --no-host-inclusive > $OUT/head_line.json 2>> $OUT/head.err || { tail -20 $OUT/head.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/head_line.json')); print('$lay', d['value'], d['roofline']['frac'], d['verified'], d['config']['layout'])" | tee -a $OUT/headab.log
done
done
