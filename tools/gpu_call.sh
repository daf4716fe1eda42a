# one-off GPU call: L2 -> fabric latency / DRAM-credit counters for the headline geometry's recover
# patterns (packed: contiguous vs scattered; odd stripe: scattered), 32 GiB passes
set -o pipefail
export PROBE_GIB=32
STEPS="lat5" TCC_LAYOUTS="r10_packed_enc:14:10:1024:0:0:enc;r10_packed_rec0123:14:10:1024:0:0:0,1,2,3;r10_packed_rec_scat:14:10:1024:0:0:1,4,11,13;r10_odd_rec_scat:14:10:1024:0:1:1,4,11,13" \
  bash tools/gpu_r05.sh
