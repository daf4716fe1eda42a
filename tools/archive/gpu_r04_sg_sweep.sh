# config 5 stripe-group sweep of the work-queue kernels (NXEC_STRIPE_GROUP overrides the
# heuristic): RS(16,4) 256 KiB and 4 MiB chunks, encode + recover, auto layout
mkdir -p gpurun_out
for cs in 262144 4194304 1048576; do
  for sg in def 1 2 4 8 16; do
    if [ $sg = def ]; then E=; else E="NXEC_STRIPE_GROUP=$sg"; fi
    env $E timeout -k 10 200 python bench.py --workload mixed16 --chunk $cs --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/sg.json 2> gpurun_out/sg.err || { tail -5 gpurun_out/sg.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/sg.json')); o=d['ops']; print('cs $cs sg $sg', o['encode']['frac'], o['decode']['frac'], d['roofline']['frac'], d['verified'])"
  done
done
