# one-off GPU call: objects/files tests, then the files A/Bs
set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "objects or files or md5" > $OUT/pytest_files.log 2>&1 || { tail -30 $OUT/pytest_files.log; exit 1; }
tail -2 $OUT/pytest_files.log
STEPS="filesalign filesab" bash tools/gpu_r05.sh || exit 1
