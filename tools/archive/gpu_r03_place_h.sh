#!/usr/bin/env bash
# Auto digest placement: the crossover H (NXEC_DIGEST_HOST_CALLERS) swept on
# the drop-in writeFileStripe leg.  First failure stops.
set -u
OUT=gpurun_out
mkdir -p $OUT
for h in ${HS:-16 12 8}; do
  NXEC_DIGEST_HOST_CALLERS=$h timeout -k 10 300 build/dropin_rate 1048576 2 write ${DROPIN_T:-4,8,12,16,24,32} \
    > $OUT/dropin_h$h.jsonl 2> $OUT/dropin_h$h.err || { echo "STOP h$h"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/dropin_h$h.jsonl'):
    d=json.loads(l); print('H=$h', d['threads'], d['GiB_s_user_data'], d['digest_calls_host'], d['digest_calls_gpu'])"
done
echo ALL-DONE
