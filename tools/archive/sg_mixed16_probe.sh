mkdir -p gpurun_out
for cs in 262144 4194304; do
  for sg in 1 2 4 8; do
    NXEC_STRIPE_GROUP=$sg timeout -k 10 200 python bench.py --workload mixed16 --chunk $cs --no-cpu-baseline --steps 6 > gpurun_out/sg_tmp.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/sg_tmp.json')); print('cs', $cs, 'sg', $sg, {k: v['frac'] for k, v in d['ops'].items()})" | tee -a gpurun_out/sg_mixed16.log
  done
done
