#!/usr/bin/env bash
# Round-6 GPU steps (one gpurun call runs the STEPS it is given; every GPU
# step under its own limit, the first failure ends the call, no retries):
#   tests    pytest -m gpu (PYTEST_K narrows it)          -> pytest_gpu.log
#   smoke    __graft_entry__.py smoke                       -> smoke.log
#   bench    bench.py defaults                              -> bench.json
#   cfg      secondary workloads (CFG_LIST)                 -> configs.jsonl
#   frames   read-frames pipeline A/B: product / host lanes (probe build) x2 -> frames_ab.jsonl
#   group    bench.py --gpus 8 --group, HW queues 4 and 8   -> group_hwq.jsonl
#   dropin   build/dropin_rate 1/4/16 callers, pool all vs current -> dropin_ab.jsonl
set -u
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-"tests"}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; stop pytest $?; }
  tail -3 $OUT/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 180 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; stop smoke $?; }
  tail -1 $OUT/smoke.log
fi
if has bench; then
  timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; stop bench $?; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('headline', d['value'], d['roofline']['frac'], d['verified'])"
fi
if has cfg; then
  CFG_LIST=${CFG_LIST:-"decode_full;files;write14;repair12;mixed16:--chunk 262144;mixed16:--chunk 4194304;mixed16:--chunk 65536;mixed16:--chunk 1048576"}
  IFS=';' read -ra CFGS <<< "$CFG_LIST"
  for c in "${CFGS[@]}"; do
    w=${c%%:*}; extra=""; [ "$c" != "$w" ] && extra=${c#*:}
    timeout -k 10 300 python bench.py --workload $w $extra --steps ${CFG_STEPS:-20} --no-cpu-baseline --no-host-inclusive \
      >> $OUT/configs.jsonl 2>> $OUT/configs.err || { tail -20 $OUT/configs.err; stop "cfg $c" $?; }
    tail -1 $OUT/configs.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'][:60], d['value'], d['roofline']['frac'], d['ms_per_step'], d['verified'])"
  done
fi
if has frames; then
  for r in 1 2 3; do
    for v in ${FRAMES_VARIANTS:-product bound lanes_bound}; do
      case $v in
        product) env="";;
        dma) env="FRAMES_DMA=1";;
        bound) env="FRAMES_BIND=1";;
        lanes) env="NXEC_LIB=build/ab/lanes/libnxec.so NXEC_HOST_LANES=1";;
        lanes_bound) env="NXEC_LIB=build/ab/lanes/libnxec.so NXEC_HOST_LANES=1 FRAMES_BIND=1";;
        lanes7) env="NXEC_LIB=build/ab/lanes/libnxec.so NXEC_HOST_LANES=1 NXEC_HOST_THREADS=7";;
        threads12) env="NXEC_HOST_THREADS=12";;
        nt) env="NXEC_LIB=build/ab/lanes/libnxec.so NXEC_NT_STAGING=1";;
        probe) env="NXEC_LIB=build/ab/lanes/libnxec.so";;
      esac
      env $env timeout -k 10 200 python tools/read_frames_ab.py $v >> $OUT/frames_ab.jsonl 2>> $OUT/frames_ab.err \
        || { tail -20 $OUT/frames_ab.err; stop "frames $v" $?; }
      tail -1 $OUT/frames_ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['label'], d['pipelined'], d['gather_only'], d['scatter_only'], {k: v.get('cpus_busy') for k, v in d['cpu'].items()})"
    done
  done
fi
if has ring; then
  # k_mul_md5 with a barrier per step (NXEC_EM_RING=0, rounds 2-5) vs the ring
  # hand-off, one probe build, alternating: write14, the verified read, repair12
  RING_LIST=${RING_LIST:-"write14;decode_full;repair12"}
  IFS=';' read -ra RW <<< "$RING_LIST"
  for r in 1 2; do
    for v in 1 0; do
      for w in "${RW[@]}"; do
        NXEC_LIB=build/ab/lanes/libnxec.so NXEC_EM_RING=$v timeout -k 10 300 python bench.py --workload $w --steps 20 \
          --no-cpu-baseline --no-host-inclusive | sed "s/^{/{\"em_ring\": $v, /" >> $OUT/ring_ab.jsonl 2>> $OUT/ring_ab.err \
          || { tail -20 $OUT/ring_ab.err; stop "ring $w $v" $?; }
        tail -1 $OUT/ring_ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ring', d['em_ring'], d['config'].get('workload'), d['ms_per_step'], {k: v['avg_ms'] for k, v in d['ops'].items()})"
      done
    done
  done
fi
if has ringsq; then
  # one SQ + GRBM pass per form (counters in their own runs, MI355X_MICROARCH.md)
  ROOT=$(pwd)
  for v in 0 1; do
    (cd /tmp && export TMPDIR=/tmp && NXEC_LIB=$ROOT/build/ab/lanes/libnxec.so NXEC_EM_RING=$v timeout -s KILL 90 rocprofv3 \
      --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
      SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/sq_ring$v -o run -- \
      python3 $ROOT/tools/ring_probe.py) > $OUT/sq_ring$v.log 2>&1 || { tail -20 $OUT/sq_ring$v.log; stop "ringsq $v" $?; }
    python3 tools/sq_summary.py $OUT/sq_ring$v k_mul_md5 em_ring=$v | tee -a $OUT/sq_ring.jsonl
  done
fi
if has group; then
  for q in ${GROUP_HWQ:-4 8}; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --gpus 8 --group --stripes 512 --steps 10 --warmup 2 \
      --no-cpu-baseline --no-host-inclusive > $OUT/group_q$q.json 2> $OUT/group_q$q.err || { tail -20 $OUT/group_q$q.err; stop "group q$q" $?; }
    python3 -c "import json; d=json.load(open('$OUT/group_q$q.json')); print('hwq $q ranks', d['value'], d['ms_per_step'], 'group', d['group']['value'], d['group']['ms_per_step'])"
  done
fi
if has gstreams; then
  # streams per device of the 8-member one-GPU group (probe build, NXEC_GROUP_STREAMS)
  for r in 1 2; do
    for gs in ${GSTREAMS:-1 2 4}; do
      NXEC_LIB=build/ab/lanes/libnxec.so NXEC_GROUP_STREAMS=$gs timeout -k 10 400 python bench.py --gpus 8 --group \
        --stripes 512 --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive > $OUT/gs_$gs.json 2> $OUT/gs_$gs.err \
        || { tail -20 $OUT/gs_$gs.err; stop "gstreams $gs" $?; }
      python3 -c "import json; d=json.load(open('$OUT/gs_$gs.json')); print('group_streams $gs ranks', d['value'], d['ms_per_step'], 'group', d['group']['value'], d['group']['ms_per_step'])" | tee -a $OUT/gstreams.log
    done
  done
fi
if has admit; then
  # per-device admission of drop-in calls (probe build, NXEC_POOL_ADMIT; 0 = none), 16 / 64 callers
  for r in 1 2; do
    for a in ${ADMIT:-0 8 16}; do
      LD_LIBRARY_PATH=$(pwd)/build/ab/lanes NXEC_POOL_ADMIT=$a timeout -k 10 200 build/dropin_rate 1048576 1.5 pool ${ADMIT_THREADS:-16,64} \
        | sed "s/^{/{\"admit\": $a, /" >> $OUT/admit_ab.jsonl 2>> $OUT/admit_ab.err || { tail -20 $OUT/admit_ab.err; stop "admit $a" $?; }
    done
  done
  grep GiB_s $OUT/admit_ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('admit', d['admit'], d['path'][:22], d['threads'], d['GiB_s'])"
fi
if has admitw; then
  # the admission gate on the write legs (RSCode::encode with the digests, writeFileStripe), 16 / 64 callers:
  # no gate / gate on every call (build/ab/lanes_noex) / gate except zero-copy digest calls (build/ab/lanes)
  for r in 1 2; do
    for v in "noex 0" "noex 8" "lanes 8"; do
      set -- $v
      for mode in write all; do
        LD_LIBRARY_PATH=$(pwd)/build/ab/$1 NXEC_POOL_ADMIT=$2 timeout -k 10 200 build/dropin_rate 1048576 1.5 $mode ${ADMIT_THREADS:-16,64} \
          | sed "s/^{/{\"variant\": \"$1\", \"admit\": $2, /" >> $OUT/admitw_ab.jsonl 2>> $OUT/admitw_ab.err || { tail -20 $OUT/admitw_ab.err; stop "admitw $v $mode" $?; }
      done
    done
  done
  grep -h GiB_s $OUT/admitw_ab.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if 'path' in d and 'threads' in d: print('admitw', d['variant'], d['admit'], d['path'][:26], d.get('buffers',''), d['threads'], d.get('GiB_s', d.get('GiB_s_user_data')), d.get('digest_calls_host'), d.get('digest_calls_gpu'))"
fi
if has tunedab; then
  # config 5: --layout auto and --layout tuned interleaved (same strides chosen; does the calibration's
  # 24 GiB scratch, freed before the batch is allocated, change the batch's speed?)
  for r in 1 2; do
    for c in 262144 4194304; do
      for lay in auto tuned; do
        timeout -k 10 300 python bench.py --workload mixed16 --chunk $c --layout $lay --steps 10 --warmup 2 --no-cpu-baseline \
          --no-host-inclusive > $OUT/tab.json 2> $OUT/tab.err || stop tunedab $?
        python3 -c "import json; d=json.load(open('$OUT/tab.json')); print('tunedab', $r, $c, '$lay', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['config']['layout'][:60])" | tee -a $OUT/tunedab.log
      done
    done
  done
fi
if has dropin; then
  for r in 1 2; do
    for v in all current; do
      NXEC_DEFAULT_DEVICES=$v timeout -k 10 300 build/dropin_rate 1048576 1.5 all 1,4,16 | sed "s/^{/{\"pool\": \"$v\", /" \
        >> $OUT/dropin_ab.jsonl 2>> $OUT/dropin_ab.err || { tail -20 $OUT/dropin_ab.err; stop "dropin $v" $?; }
    done
  done
  tail -4 $OUT/dropin_ab.jsonl
fi
