# k_mul_md5 ring depth A/B (write14): in-tree build (D = 4) vs separate builds with -DNXEC_EM_DEPTH=5, 6
mkdir -p gpurun_out
for round in 1 2; do
  for v in default d5 d6; do
    if [ $v = default ]; then L=; else L=build/var/$v/libnxec.so; fi
    NXEC_LIB=$L timeout -k 10 200 python bench.py --workload write14 --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/emd_$v.json 2> gpurun_out/emd_$v.err || { tail -5 gpurun_out/emd_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/emd_$v.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified'])"
  done
done
