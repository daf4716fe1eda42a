#!/usr/bin/env bash
# Round-5 GPU steps (one gpurun call runs the STEPS it is given; every GPU
# step under its own limit, the first failure ends the call, no retries):
#   sweep5   config-5 layout A/B: chunk pads 0-16 KiB x odd stripe stride x
#            stripe groups, RS(16,4) 256 KiB / 1 MiB / 4 MiB, twice -> config5_layout_ab.log
#   tccval   one per-L2-channel counter pass (tools/tcc_instances.yaml) -> tcc/val
#   tcc5     per-L2-channel read/write request passes, default vs candidate
#            layouts (TCC_LAYOUTS) -> tcc5.jsonl
set -u
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-"sweep5"}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
ROOT=$(pwd)
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
  timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; stop bench $?; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('headline', d['value'], d['roofline']['frac'], d['verified'])"
fi
if has cfg; then
  # secondary workloads, one JSON line each (CFG_LIST: "workload[:extra args]" ;-separated)
  CFG_LIST=${CFG_LIST:-"decode_full;files;write14;repair12;mixed16:--chunk 262144;mixed16:--chunk 4194304;mixed16:--chunk 65536;mixed16:--chunk 1048576"}
  IFS=';' read -ra CFGS <<< "$CFG_LIST"
  for c in "${CFGS[@]}"; do
    w=${c%%:*}; extra=""; [ "$c" != "$w" ] && extra=${c#*:}
    timeout -k 10 300 python bench.py --workload $w $extra --steps ${CFG_STEPS:-20} --no-cpu-baseline --no-host-inclusive \
      >> $OUT/configs.jsonl 2>> $OUT/configs.err || { tail -20 $OUT/configs.err; stop "cfg $c" $?; }
    tail -1 $OUT/configs.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'][:60], d['value'], d['roofline']['frac'], d['ms_per_step'], d['verified'])"
  done
fi
if has sweep5; then
  PROBE_GIB=32 PROBE_REPEAT=2 PROBE_CPADS=0,2048,4096,8192,16384 PROBE_SPADS=0,1 PROBE_SG=1,8 PROBE_SG_ALL=1 \
    timeout -k 10 400 python3 -u tools/layout_probe.py 20,16,256 20,16,4096 20,16,1024 \
    > $OUT/config5_layout_ab.log 2>&1 || { tail -5 $OUT/config5_layout_ab.log; stop sweep5 $?; }
  tail -3 $OUT/config5_layout_ab.log
fi
if has tccval; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 60 rocprofv3 -E $ROOT/tools/tcc_instances.yaml --pmc NXEC_TCC_RD_I0 NXEC_TCC_RD_I1 NXEC_TCC_RD_I2 \
    NXEC_TCC_RD_I3 --kernel-trace --output-format csv -d $ROOT/$OUT/tcc/val -o run -- \
    python3 $ROOT/tools/tcc_channels.py 20 16 256 0 0 enc 2 > $ROOT/$OUT/tcc_val.log 2>&1 \
    || { tail -20 $ROOT/$OUT/tcc_val.log; stop tccval $?; }
  cd $ROOT
  tail -3 $OUT/tcc_val.log
  python3 tools/tcc_summary.py val $OUT/tcc/val || true
fi
if has tcc5; then
  # TCC_LAYOUTS: "label:n:k:cs_kib:cpad:spad:op;..."
  TCC_LAYOUTS=${TCC_LAYOUTS:-"256k_packed:20:16:256:0:0:enc;256k_packed_rec:20:16:256:0:0:1,4,17,19"}
  IFS=';' read -ra LAY <<< "$TCC_LAYOUTS"
  cd /tmp && export TMPDIR=/tmp
  for L in "${LAY[@]}"; do
    IFS=':' read -r lab n k cs cpad spad op <<< "$L"
    dirs=""
    for tag in RD WR; do
      for q in 0 4 8 12; do
        d=$ROOT/$OUT/tcc/$lab/${tag}$q
        timeout -s KILL 60 rocprofv3 -E $ROOT/tools/tcc_instances.yaml --pmc NXEC_TCC_${tag}_I$q \
          NXEC_TCC_${tag}_I$((q+1)) NXEC_TCC_${tag}_I$((q+2)) NXEC_TCC_${tag}_I$((q+3)) --kernel-trace \
          --output-format csv -d $d -o run -- python3 $ROOT/tools/tcc_channels.py $n $k $cs $cpad $spad $op 2 \
          > $ROOT/$OUT/tcc_$lab.log 2>&1 || { tail -20 $ROOT/$OUT/tcc_$lab.log; stop "tcc5 $lab $tag$q" $?; }
        dirs="$dirs $d"
      done
    done
    python3 $ROOT/tools/tcc_summary.py $lab $dirs >> $ROOT/$OUT/tcc5.jsonl || stop "tcc_summary $lab" $?
  done
  cd $ROOT
  wc -l $OUT/tcc5.jsonl
fi
if has lat5; then
  # per-request latency and credit stalls at the L2 -> fabric interface (same
  # TCC_LAYOUTS): LEVEL_sum / REQ_sum = average requests' cycles in flight
  IFS=';' read -ra LAY <<< "$TCC_LAYOUTS"
  cd /tmp && export TMPDIR=/tmp
  for L in "${LAY[@]}"; do
    IFS=':' read -r lab n k cs cpad spad op <<< "$L"
    for pass in "RD:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
                "WR:TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum" \
                "BUSY:TCC_BUSY_avr TCC_CYCLE_sum TCC_TAG_STALL_sum"; do
      tag=${pass%%:*}; ctrs=${pass#*:}
      timeout -s KILL 60 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $ROOT/$OUT/lat/$lab/$tag -o run -- \
        python3 $ROOT/tools/tcc_channels.py $n $k $cs $cpad $spad $op 2 > $ROOT/$OUT/lat_$lab.log 2>&1 \
        || { tail -20 $ROOT/$OUT/lat_$lab.log; stop "lat5 $lab $tag" $?; }
    done
    python3 $ROOT/tools/tcc_summary.py --lat $lab $ROOT/$OUT/lat/$lab >> $ROOT/$OUT/lat5.jsonl || stop "lat_summary $lab" $?
  done
  cd $ROOT
  cat $OUT/lat5.jsonl
fi
if has sweep5b; then
  PROBE_GIB=32 PROBE_REPEAT=2 PROBE_CPADS=0,4096 PROBE_SPADS=0 PROBE_SG=1 \
    timeout -k 10 400 python3 -u tools/layout_probe.py 20,16,128 20,16,256 20,16,512 14,10,128 14,10,256 14,10,512 \
    20,16,64 14,10,64 > $OUT/config5_layout_ab_b.log 2>&1 || { tail -5 $OUT/config5_layout_ab_b.log; stop sweep5b $?; }
  tail -3 $OUT/config5_layout_ab_b.log
fi
if has filesab; then
  # same-box A/B of the multi-file write: product (the fold), the probe build
  # with the fold off (round 4: pad copy + plain kernel); alternating, twice
  for r in 1 2; do
    for v in prod nofold; do
      case $v in
        prod) lib=""; env="";;
        nofold) lib=build/ab/probes/libnxec.so; env="NXEC_FILES_FOLD=0";;
        probes) lib=build/ab/probes/libnxec.so; env="";;
      esac
      env $env ${lib:+NXEC_LIB=$ROOT/$lib} timeout -k 10 300 python bench.py --workload files --steps 30 --no-cpu-baseline \
        --no-host-inclusive > $OUT/filesab_line.json 2>> $OUT/filesab.err || { tail -20 $OUT/filesab.err; stop "filesab $v" $?; }
      python3 -c "import json; d=json.load(open('$OUT/filesab_line.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['verified'], d['roofline']['lib_sha16'])" | tee -a $OUT/filesab.log
    done
  done
fi
if has filesalign; then
  # the fold's cost split: aligned in-place reads vs masked chunks vs raw sizes
  for v in prod nofold; do
    case $v in
      prod) lib=""; env="";;
      nofold) lib=build/ab/probes/libnxec.so; env="NXEC_FILES_FOLD=0";;
    esac
    echo "== $v" >> $OUT/files_align.log
    env $env ${lib:+NXEC_LIB=$ROOT/$lib} timeout -k 10 300 python3 -u tools/files_align_probe.py >> $OUT/files_align.log 2>&1 \
      || { tail -20 $OUT/files_align.log; stop "filesalign $v" $?; }
  done
  cat $OUT/files_align.log
fi
echo "DONE $STEPS"
