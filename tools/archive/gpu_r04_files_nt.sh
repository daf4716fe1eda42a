mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "encode_objects" > gpurun_out/t_nt.log 2>&1 || { tail -20 gpurun_out/t_nt.log; exit 1; }
tail -1 gpurun_out/t_nt.log
timeout -k 10 200 python bench.py --workload files --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/files_nt.json 2>&1 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/files_nt.json')); print(d['ms_per_step'], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['verified'])"
timeout -k 10 300 python3 tools/files_mix_probe.py full10 ragged mix > gpurun_out/files_mix_nt.log 2>&1 || exit 1
cat gpurun_out/files_mix_nt.log
