#!/usr/bin/env bash
# k_mul_md5 variant B (NXEC_EM_HASHSRC=global: hash lanes read the sources from
# L2 / MALL) against the default, write14, alternating; variant tests first.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_md5.py -x -q --timeout 240 --timeout-method thread \
  > $OUT/pytest_em.log 2>&1 || { tail -30 $OUT/pytest_em.log; stop pytest $?; }
tail -2 $OUT/pytest_em.log
for i in 1 2 3; do
  for t in lds global; do
    NXEC_EM_HASHSRC=$t timeout -k 10 200 python bench.py --workload write14 --steps 10 --warmup 2 --no-cpu-baseline \
      --no-host-inclusive > $OUT/w14_$t.json 2> $OUT/w14_$t.err || stop w14_$t $?
    python3 -c "import json; d=json.load(open('$OUT/w14_$t.json')); print('write14 hashsrc=$t', d['ms_per_step'], d['roofline']['frac'], d['verified'])" | tee -a $OUT/hg_ab.log
  done
done
echo ALL-DONE
