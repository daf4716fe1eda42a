#!/usr/bin/env bash
# GPU-box sequence, each step under its own time limit; the first failing step
# ends the call (no retries).  Select steps with STEPS="tests smoke bench ..."
#   tests   python -m pytest tests -m gpu            -> gpurun_out/pytest_gpu.log
#   smoke   __graft_entry__.smoke()                  -> gpurun_out/smoke.log
#   bench   python bench.py $BENCH_ARGS              -> gpurun_out/bench.json
#   bench2  python bench.py --gpus 2 (1-GPU rehearsal of the rank launcher)
#   prof    rocprofv3 --kernel-trace --stats of bench.py $PROF_ARGS -> gpurun_out/prof/
#   pmc     rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py $PROF_ARGS
#   dropin  build/dropin_rate $DROPIN_ARGS           -> gpurun_out/dropin.jsonl
set -u
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-"tests smoke bench"}
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
bash tools/host_probe.sh > $OUT/host.txt 2>&1
if has tests; then
  timeout -k 10 ${PYTEST_T:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || stop pytest $rc
fi
if has smoke; then
  timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || stop smoke $?
  tail -1 $OUT/smoke.log
fi
if has bench; then
  timeout -k 10 ${BENCH_T:-600} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || stop bench $?
  cat $OUT/bench.json
fi
if has bench2; then
  timeout -k 10 ${BENCH_T:-600} python bench.py --gpus 2 --no-cpu-baseline ${BENCH2_ARGS:-} > $OUT/bench2.json 2> $OUT/bench2.err || stop bench2 $?
  cat $OUT/bench2.json
fi
if has prof; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive ${PROF_ARGS:-} \
    > $OUT/prof_bench.json 2> $OUT/prof.err || stop rocprof $?
  find $OUT/prof -name "*stats*"
fi
if has pmc; then
  # PMC_SETS: ";"-separated "tag:bench args" (default: the headline workload)
  export TMPDIR=/tmp
  IFS=';' read -ra SETS <<< "${PMC_SETS:-rs10_4:--steps 2 --warmup 0}"
  for set in "${SETS[@]}"; do
    tag=${set%%:*}; args=${set#*:}
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${tag}_$c -o run -- \
        python3 bench.py --no-cpu-baseline --no-host-inclusive $args \
        > $OUT/pmc_${tag}_$c.json 2> $OUT/pmc_${tag}_$c.err || stop pmc_${tag}_$c $?
    done
    echo "pmc $tag done"
  done
fi
if has dropin; then
  timeout -k 10 300 ./build/dropin_rate ${DROPIN_ARGS:-} > $OUT/dropin.jsonl 2> $OUT/dropin.err || stop dropin $?
  cat $OUT/dropin.jsonl
fi
exit 0
