# k_mul_md5 A/B: one 512-lane workgroup per CU (default) vs two 256-lane workgroups per CU
# with their own step barriers (NXEC_EM_HALF=1), write14, alternating
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_md5.py -x -q --timeout 120 --timeout-method thread -k "variants_ab" > gpurun_out/t_half.log 2>&1 || { tail -20 gpurun_out/t_half.log; exit 1; }
tail -1 gpurun_out/t_half.log
for round in 1 2; do
  for h in 0 1; do
    NXEC_EM_HALF=$h timeout -k 10 200 python bench.py --workload write14 --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/half_$h.json 2> gpurun_out/half_$h.err || { tail -5 gpurun_out/half_$h.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/half_$h.json')); print('half=$h', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified'])"
  done
done
