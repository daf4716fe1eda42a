#!/usr/bin/env bash
# k_mul_md5 split-nibble table A/B (NXEC_EM_TABLES=nib) + k_files_md5 role probes.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_md5.py -x -q --timeout 240 --timeout-method thread \
  > $OUT/pytest_em.log 2>&1 || { tail -30 $OUT/pytest_em.log; stop pytest $?; }
tail -2 $OUT/pytest_em.log
for i in 1 2 3; do
  for t in byte nib; do
    NXEC_EM_TABLES=$t timeout -k 10 200 python bench.py --workload write14 --steps 10 --warmup 2 --no-cpu-baseline \
      --no-host-inclusive > $OUT/w14_$t.json 2> $OUT/w14_$t.err || stop w14_$t $?
    python3 -c "import json; d=json.load(open('$OUT/w14_$t.json')); print('write14 tables=$t', d['ms_per_step'], d['roofline']['frac'], d['verified'])" | tee -a $OUT/nib_ab.log
  done
done
bash tools/gpu_r04_files_roles.sh || exit $?
