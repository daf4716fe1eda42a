#!/usr/bin/env bash
# Round-6 closing evidence on the final library, every step under its own
# limit, the first failure ends the call (no retries):
#   tests  -m gpu + smoke                         -> pytest_gpu_final.log, smoke.log
#   bench  headline (defaults)                    -> bench_final.json
#   prof   rocprofv3 --kernel-trace --stats       -> prof/ + prof_bench.json
#   pmc    FETCH_SIZE / WRITE_SIZE passes per workload, dispatches labelled
#          with the bench line's bytes per launch -> pmc_<w>.json
#   cfg    secondary workloads                    -> configs_final.jsonl
#   group  8-member nxec_group rehearsal on one GPU -> group8.json
#   dropin the drop-in per-stripe rates (build/dropin_rate, default pool) -> dropin_final.jsonl
# STEPS selects (default: all).
set -u
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-"tests bench prof pmc cfg group dropin"}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu_final.log 2>&1 || { tail -30 $OUT/pytest_gpu_final.log; stop pytest $?; }
  tail -2 $OUT/pytest_gpu_final.log
  timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || stop smoke $?
  tail -1 $OUT/smoke.log
fi
if has bench; then
  timeout -k 10 500 python bench.py > $OUT/bench_final.json 2> $OUT/bench_final.err || stop bench $?
  python3 -c "import json; d=json.load(open('$OUT/bench_final.json')); print('headline', d['value'], d['roofline']['frac'], d['verified'])"
fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive > $OUT/prof_bench.json 2> $OUT/prof.err \
    || stop rocprof $?
  find $OUT/prof -name "*stats*"
fi
if has pmc; then
  # workload | extra bench args | kernel substring | op label (bench.py PMC_SUMMARIES)
  for spec in "rs10_4||k_mul_vec<10|encode_recover" "decode_full||k_mul_vec<10,8,false,true|decode_full" \
              "write14||k_mul_md5<10|encode_md5_fused" "repair12||k_mul_perm<12|repair_fused_perm12" \
              "files||k_files_md5<10|encode_objects_md5" "mixed16|--chunk 4194304 --gib 16|k_mul_vec<16|encode_recover"; do
    IFS='|' read -r w extra ksub op <<< "$spec"
    CMD="python3 bench.py --workload $w $extra --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_${w}_$c -o run -- \
        $CMD > $OUT/pmc_${w}_$c.json 2> $OUT/pmc_${w}_$c.err || stop pmc_${w}_$c $?
    done
    B=$(python3 -c "import json; print(json.load(open('$OUT/pmc_${w}_FETCH_SIZE.json'))['roofline']['bytes_per_launch'])")
    python3 tools/pmc_label.py $OUT/pmc_${w}_FETCH_SIZE $OUT/pmc_${w}_WRITE_SIZE "$ksub" "$CMD" "$op:$B*" \
      > $OUT/pmc_$w.json || stop label_$w $?
    python3 -c "
import json; d=json.load(open('$OUT/pmc_$w.json')); r=[x['traffic_over_algorithmic'] for x in d['dispatches']]
print('pmc $w', d['lib_sha16'], len(r), 'dispatches, traffic/algorithmic', min(r), max(r))"
  done
fi
if has cfg; then
  rm -f $OUT/configs_final.jsonl
  for spec in "decode_full|" "write14|" "object|" "files|" "repair12|" "repair12|--failed 15" "mixed16|--chunk 65536" \
              "mixed16|--chunk 262144" "mixed16|--chunk 1048576" "mixed16|--chunk 4194304" "rs10_4|--layout recover" \
              "mixed16|--chunk 262144 --layout tuned" "mixed16|--chunk 4194304 --layout tuned" \
              "mixed16|--chunk 65536 --layout tuned" "mixed16|--chunk 1048576 --layout tuned"; do
    IFS='|' read -r w extra <<< "$spec"
    timeout -k 10 300 python bench.py --workload $w $extra --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive \
      > $OUT/cfg.json 2> $OUT/cfg.err || stop cfg_$w $?
    cat $OUT/cfg.json >> $OUT/configs_final.jsonl
    python3 -c "import json; d=json.load(open('$OUT/cfg.json')); print('$w $extra', d['ms_per_step'], d['roofline']['frac'], d['verified'])"
  done
fi
if has group; then
  timeout -k 10 300 python bench.py --gpus 8 --group --stripes 512 --steps 10 --warmup 2 --no-cpu-baseline \
    --no-host-inclusive > $OUT/group8.json 2> $OUT/group8.err || stop group $?
  python3 -c "import json; d=json.load(open('$OUT/group8.json')); print('group8', d['value'], d['verified'], d['group']['value'], d['group']['verified'])"
fi
if has dropin; then
  timeout -k 10 300 build/dropin_rate 1048576 1.5 all 1,4,16 > $OUT/dropin_final.jsonl 2> $OUT/dropin_final.err || stop dropin $?
  tail -3 $OUT/dropin_final.jsonl
fi
echo ALL-DONE
