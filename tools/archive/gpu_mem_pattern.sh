#!/usr/bin/env bash
# memory-pattern probe on one box; output tagged with the host name
set -u
OUT=gpurun_out; mkdir -p $OUT
tag=${1:-run}
{ echo "host $(hostname)"; timeout -k 10 200 ./tools/microbench/mem_pattern ${REPS:-10} ${FILTER:-}; } > $OUT/mem_pattern_$tag.log 2>&1
rc=$?; cat $OUT/mem_pattern_$tag.log; exit $rc
