#!/usr/bin/env bash
# MD5 kernel tuning sweep on the GPU box: (ring depth D, group G blocks,
# nontemporal) variants via NXEC_MD5_CFG, each a separate bench process
# (write14 workload), one line per variant.
set -u
OUT=gpurun_out; mkdir -p $OUT
for cfg in ${MD5_CFGS:-2,1,0 4,1,0 2,2,0 3,2,0 2,4,0 3,4,0 2,8,0}; do
  tag=${cfg//,/_}
  NXEC_MD5_CFG=$cfg timeout -k 10 120 python bench.py --workload write14 --steps 3 --warmup 1 \
    --no-cpu-baseline > $OUT/md5_$tag.json 2>> $OUT/md5_tune.err || { echo "STOP cfg=$cfg rc=$?"; exit 1; }
  python3 -c "import json;r=json.load(open('$OUT/md5_$tag.json'));o=r['ops']['md5_all_chunks'];print('cfg=$cfg md5', o['avg_ms'], 'ms', o['GB_s'], 'GB/s; encode', r['ops']['encode']['GB_s'])"
done
