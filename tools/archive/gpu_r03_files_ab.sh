#!/usr/bin/env bash
# files-path tests, then an alternating A/B of build/ab/libnxec_{new,old}.so on
# the files bench and the full-stripe probe, then FETCH_SIZE / WRITE_SIZE
# counter passes of the files bench on the new library
set -u
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "encode_objects or encode_decode_object or objects" > $OUT/pytest_files.log 2>&1 || { tail -30 $OUT/pytest_files.log; exit 1; }
tail -1 $OUT/pytest_files.log
AB_CMD="python bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive | python3 -c \"import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'])\"; python tools/files_probe.py 2>&1 | tail -1" AB_T=300 bash tools/ab_lib.sh || exit 1
if [ -n "${PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmcf_$c -o run -- \
      python3 bench.py --workload files --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/pmcf_$c.json 2> $OUT/pmcf_$c.err || { echo "STOP pmc $c"; exit 1; }
  done
  python3 tools/pmc_dispatch.py $OUT/pmcf_FETCH_SIZE $OUT/pmcf_WRITE_SIZE "k_files_md5" > $OUT/pmcf_dispatch.jsonl || exit 1
  cat $OUT/pmcf_dispatch.jsonl
fi
echo ALL-DONE
