#!/usr/bin/env bash
# k_files_md5 role probes (tools/files_role_probe.py) under rocprofv3 --kernel-trace
set -u
OUT=gpurun_out
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
NXEC_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_roles -o run --output-format csv -- \
  python3 tools/files_role_probe.py > $OUT/files_roles.log 2>&1 || stop rocprof $?
grep -E "^probe|plan" $OUT/files_roles.log | head -60
f=$(find $OUT/prof_roles -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "files_md5" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print("k_files_md5 launches", len(d))
i = 0
for probe in range(8):
    for name in ("full10", "mix"):
        print(f"probe {probe} {name:6s} kernel ms", " ".join(f"{x:.3f}" for x in d[i:i + 3]))
        i += 3
PY
echo ALL-DONE
