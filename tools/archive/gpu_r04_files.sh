#!/usr/bin/env bash
# Multi-file write: encode_objects tests (incl. the in-place tail mode), the
# files mix probe (copy vs in-place tails) and bench --workload files.
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "encode_objects" -x -q --timeout 300 \
  --timeout-method thread > $OUT/pytest_files.log 2>&1 || { tail -30 $OUT/pytest_files.log; stop pytest $?; }
tail -2 $OUT/pytest_files.log
timeout -k 10 300 python tools/files_mix_probe.py ${PROBE_SETS:-} > $OUT/files_mix.log 2>&1 || stop files_mix $?
cat $OUT/files_mix.log
timeout -k 10 300 python bench.py --workload files --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive \
  > $OUT/bench_files.json 2> $OUT/bench_files.err || stop bench_files $?
python3 -c "import json; d=json.load(open('$OUT/bench_files.json')); print('files', d['ms_per_step'], d['roofline']['frac'], d['verified'], d['config']['md5_chain_floor'])"
echo ALL-DONE
