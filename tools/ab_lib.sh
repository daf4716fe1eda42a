#!/usr/bin/env bash
# Same-box A/B of two libnxec builds (build/ab/libnxec_{old,new}.so): runs
# CMD with each library copied in place, alternating new/old/new/old, so box
# and clock differences cancel.  Usage: AB_CMD="python tools/encode_md5_probe.py 14 10 1048576 4096" bash tools/ab_lib.sh
set -u
OUT=gpurun_out/ab
mkdir -p $OUT
for v in new old new old; do
  cp build/ab/libnxec_$v.so nexoedge_amd/lib/libnxec.so
  echo "== $v" >> $OUT/ab.log
  timeout -k 10 ${AB_T:-200} bash -c "$AB_CMD" >> $OUT/ab.log 2>&1 || { echo "STOP $v rc=$?"; cat $OUT/ab.log; exit 1; }
done
cp build/ab/libnxec_new.so nexoedge_amd/lib/libnxec.so
cat $OUT/ab.log
