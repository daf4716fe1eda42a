#!/usr/bin/env bash
# MD5 kernel tuning sweep on the GPU box: prefetch depth x load cache policy,
# each a separate bench process (write14 workload), one line per variant.
set -u
OUT=gpurun_out; mkdir -p $OUT
for nt in 1 0; do
  for d in 2 3 4; do
    NXEC_MD5_DEPTH=$d NXEC_MD5_NT=$nt timeout -k 10 120 python bench.py --workload write14 --steps 3 --warmup 1 \
      --no-cpu-baseline > $OUT/md5_d${d}_nt${nt}.json 2>> $OUT/md5_tune.err || { echo "STOP d=$d nt=$nt rc=$?"; exit 1; }
    python3 -c "import json,sys;r=json.load(open('$OUT/md5_d${d}_nt${nt}.json'));o=r['ops']['md5_all_chunks'];print('d=$d nt=$nt md5', o['avg_ms'], 'ms', o['GB_s'], 'GB/s; encode', r['ops']['encode']['GB_s'])"
  done
done
