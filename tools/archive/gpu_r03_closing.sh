#!/usr/bin/env bash
# Closing evidence on the final library: GPU tests + smoke + headline bench +
# rocprofv3 stats (tools/gpu_r03.sh), the headline PMC traffic
# (tools/gpu_r03_pmc.sh) and the secondary workloads.  First failure stops.
set -u
OUT=gpurun_out
PROFILE=1 bash tools/gpu_r03.sh || exit $?
bash tools/gpu_r03_pmc.sh || exit 1
for w in write14 object files repair12 mixed16; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "STOP $w"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['ms_per_step'], d['roofline']['frac'], d['verified'])"
done
echo ALL-DONE-CLOSING
