#!/usr/bin/env bash
# Drop-in write leg (writeFileStripe per stripe, RS(10,4) 1 MiB) under each
# digest placement of nxec_encode_host_md5, plus the host-hashed reference
# form (NXEC_CHUNK_MD5=0: Chunk::computeMD5 on the calling thread).  Then the
# placement tests.  Each GPU step has its own limit; the first failure stops.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
T=${DROPIN_T:-1,4,16,64}
for p in auto gpu host; do
  NXEC_DIGEST_PLACE=$p timeout -k 10 300 build/dropin_rate 1048576 ${DROPIN_S:-2} write $T \
    > $OUT/dropin_place_$p.jsonl 2> $OUT/dropin_place_$p.err || stop dropin_$p $?
  cat $OUT/dropin_place_$p.jsonl
done
NXEC_CHUNK_MD5=0 timeout -k 10 300 build/dropin_rate 1048576 ${DROPIN_S:-2} write $T \
  > $OUT/dropin_place_none.jsonl 2> $OUT/dropin_place_none.err || stop dropin_none $?
cat $OUT/dropin_place_none.jsonl
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin_md5.py tests/test_cpp_surface.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -s > $OUT/pytest_place.log 2>&1 || { tail -30 $OUT/pytest_place.log; stop pytest $?; }
  tail -3 $OUT/pytest_place.log
  grep "placement" $OUT/pytest_place.log || true
fi
echo ALL-DONE
