# one-off GPU call: the >= 2 MiB chunk pad (2 KiB today) against 3 / 5 / 6 / 7 KiB over geometries, twice
set -o pipefail
OUT=gpurun_out
PROBE_GIB=32 PROBE_REPEAT=2 PROBE_CPADS=2048,3072,5120,6144,7168 PROBE_SPADS=0 PROBE_SG=1 \
  timeout -k 10 700 python3 -u tools/layout_probe.py 20,16,2048 20,16,8192 14,10,2048 14,10,4096 16,12,4096 12,8,4096 20,16,3072 \
  > $OUT/bigpads.log 2>&1 || { tail -5 $OUT/bigpads.log; exit 1; }
grep -c enc $OUT/bigpads.log
