#!/usr/bin/env bash
# End of session: full GPU tests + smoke + headline bench (tools/gpu_r03.sh),
# then the files-kernel load-policy A/B (NXEC_FILES_LOADS=1 cached, 0 streaming)
set -u
bash tools/gpu_r03.sh || exit $?
for v in 1 0 1 0; do
  echo "== NXEC_FILES_LOADS=$v"
  NXEC_FILES_LOADS=$v timeout -k 10 300 python bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline --no-host-inclusive \
    | python3 -c "import json,sys; d=json.load(sys.stdin); print('files', d['ms_per_step'])" || exit 1
  NXEC_FILES_LOADS=$v timeout -k 10 200 python tools/files_probe.py 2>&1 | tail -1 || exit 1
done
echo ALL-DONE-END
