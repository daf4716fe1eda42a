#!/usr/bin/env bash
# rocprofv3 kernel trace of the files mix probe: kernel durations of
# k_files_md5 per batch against the probe's wall time per call (host planning
# + table upload + the kernel).
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_files -o run --output-format csv -- \
  python3 tools/files_mix_probe.py ${PROBE_SETS:-} > $OUT/files_mix_prof.log 2>&1 || stop rocprof $?
cat $OUT/files_mix_prof.log | grep -v "^\[" | tail -12
f=$(find $OUT/prof_files -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "files_md5" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print("k_files_md5 launches", len(d))
for i in range(0, len(d), 6):
    print(" ".join(f"{x:.3f}" for x in d[i:i + 6]))
PY
echo ALL-DONE
