#!/usr/bin/env bash
# End-of-round evidence, part 2: the headline kernel's PMC traffic on this
# library, the 2-rank rehearsal of the N > 1 path (both ranks on the box's one
# GPU), and the secondary workloads.  First failure stops.
set -u
OUT=gpurun_out
mkdir -p $OUT
bash tools/gpu_r03_pmc.sh || exit 1
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 --no-host-inclusive > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo "STOP n2"; tail -20 $OUT/bench_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_n2.json')); print('n2', d['n_gpus'], d['value'], d['ms_per_step'], d['numa_node_per_rank'], d['verified'])"
for w in write14 object files repair12; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "STOP $w"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['ms_per_step'], d['roofline']['frac'], d['verified'])"
done
echo ALL-DONE
