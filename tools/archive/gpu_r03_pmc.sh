#!/usr/bin/env bash
# HBM traffic of the headline kernel on the current library: two separate
# rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE; --kernel-trace only) of
# the default bench, each dispatch of k_mul_vec labelled with its bench op
# (tools/pmc_label.py: 1 warmup + 3 timed steps of encode + recover, then the
# 4 erase-and-rebuild checks) -> gpurun_out/pmc_rs10_4.json
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CMD="python3 bench.py --no-cpu-baseline --no-host-inclusive --steps 3 --warmup 1"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$c -o run -- \
    $CMD > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err || { echo "STOP pmc $c rc=$?"; exit 1; }
done
B=60129542144
python3 tools/pmc_label.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE "k_mul_vec<10" "$CMD" \
  encode:$B "recover[0,1,2,3]:$B" encode:$B "recover[0,1,2,3]:$B" encode:$B "recover[10,11,12,13]:$B" \
  encode:$B "recover[1,4,11,13]:$B" rebuild_encode:$B "rebuild_recover[0,1,2,3]:$B" \
  "rebuild_recover[10,11,12,13]:$B" "rebuild_recover[1,4,11,13]:$B" > $OUT/pmc_rs10_4.json || { echo "STOP label"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/pmc_rs10_4.json'))
print(d['lib_sha16'])
for x in d['dispatches']: print(x['op'], x['traffic_over_algorithmic'], x['frac_of_8TBs_fetch_pass'])"
echo ALL-DONE
