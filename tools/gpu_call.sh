# one-off GPU call: finer chunk pads at 128 / 256 / 512 KiB chunks over (14,10) and (20,16), twice
set -o pipefail
OUT=gpurun_out
PROBE_GIB=32 PROBE_REPEAT=2 PROBE_CPADS=0,1536,2560,3072,3584,4096,4608,5120,6144,7168,10240,12288 PROBE_SPADS=0 PROBE_SG=1 \
  timeout -k 10 800 python3 -u tools/layout_probe.py 20,16,256 14,10,256 14,10,128 20,16,128 14,10,512 \
  > $OUT/smallchunk_pads.log 2>&1 || { tail -5 $OUT/smallchunk_pads.log; exit 1; }
grep -c enc $OUT/smallchunk_pads.log
