#!/usr/bin/env bash
# SQ counters of k_mul_md5 vs k_files_md5 on identical full stripes
# (tools/files_probe.py): one --pmc pass, 8 SQ counters, --kernel-trace only.
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 tools/files_probe.py > $OUT/sq_probe.log 2>&1 || { echo "STOP sq rc=$?"; tail -5 $OUT/sq_probe.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/sq/**/run_counter_collection.csv', recursive=True) or glob.glob('gpurun_out/sq/run_counter_collection.csv')
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(f[0])):
    name = r.get('Kernel_Name', '')
    if 'k_mul_md5' not in name and 'k_files_md5' not in name: continue
    key = 'k_mul_md5' if 'k_mul_md5' in name else 'k_files_md5'
    agg[key][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(key, r['Dispatch_Id'])] += 1
nd = collections.Counter(k for k, _ in cnt)
for key, d in agg.items():
    print(key, 'dispatches', nd[key], ' '.join(f"{c}={v / nd[key]:.4g}" for c, v in sorted(d.items())))
PY
echo ALL-DONE
