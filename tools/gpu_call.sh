# one-off GPU call: read-path pool-size A/B, then the decode_frames tests
set -o pipefail
OUT=gpurun_out
for t in 8 16 12 8 16; do
  NXEC_HOST_THREADS=$t FRAMES_READ=1 timeout -k 10 240 python3 -u tools/frames_rate.py >> $OUT/frames_read.log 2>&1 || { tail -20 $OUT/frames_read.log; exit 1; }
done
cat $OUT/frames_read.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "frames" > $OUT/pytest_frames.log 2>&1 || { tail -30 $OUT/pytest_frames.log; exit 1; }
tail -2 $OUT/pytest_frames.log
