# one-off GPU call: chunk pads 0-48 KiB (and odd stripe) for the headline geometry RS(10,4) 1 MiB, twice
set -o pipefail
OUT=gpurun_out
PROBE_GIB=32 PROBE_REPEAT=2 PROBE_CPADS=0,512,1024,1536,2560,3072,3584,5120,6144,7168,10240,12288,20480,24576,40960,49152 PROBE_SPADS=0,1 PROBE_SG=1 \
  timeout -k 10 900 python3 -u tools/layout_probe.py 14,10,1024 > $OUT/headline_pads.log 2>&1 || { tail -5 $OUT/headline_pads.log; exit 1; }
grep -c enc $OUT/headline_pads.log
