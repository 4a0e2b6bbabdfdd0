#!/bin/bash
# In-step timing of the fused aggregation kernel variants (FLSIM_AGG_VARIANT="G,NT"): the bench's
# live probe over the training step, where theta/m/v/S come cold from HBM.
set -u
mkdir -p gpurun_out
for V in 1,0 2,0 1,1 4,0; do
  FLSIM_AGG_VARIANT=$V timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline \
      > gpurun_out/agg_instep_$V.json 2> gpurun_out/agg_instep_$V.err || { echo "bench $V failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/agg_instep_$V.json')); a=d['aggregation']; print('$V', d['value'], a['avg_launch_us'], a['achieved'], a['frac'])"
done
