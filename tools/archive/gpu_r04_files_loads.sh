# k_files_md5 on whole stripes: cached vs streaming loads, against k_mul_md5 (write14) on the same box
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/files_mix_probe.py full10 mix > gpurun_out/fl_cached.log 2>&1 || exit 1
NXEC_FILES_LOADS=0 timeout -k 10 200 python3 tools/files_mix_probe.py full10 mix > gpurun_out/fl_stream.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload write14 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/w14.json 2>&1 || exit 1
cat gpurun_out/fl_cached.log gpurun_out/fl_stream.log
python3 -c "import json; d=json.load(open('gpurun_out/w14.json')); print('write14', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
