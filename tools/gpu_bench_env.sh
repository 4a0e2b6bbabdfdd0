#!/bin/bash
# bench.py (no CPU baseline) without and with an environment setting, e.g.
#   bash tools/gpu_bench_env.sh <tag> FLSIM_WGRAD_STREAM=1 [bench args...]
set -u
TAG=$1; SETTING=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_${TAG}_off.json 2> gpurun_out/bench_${TAG}_off.err \
    || { echo "bench off failed"; tail -5 gpurun_out/bench_${TAG}_off.err; exit 1; }
env $SETTING timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_${TAG}_on.json 2> gpurun_out/bench_${TAG}_on.err \
    || { echo "bench on failed"; tail -5 gpurun_out/bench_${TAG}_on.err; exit 1; }
for V in off on; do
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$V.json')); print('$V', d['value'], d['ms_per_step'], d['roofline']['frac'], d['aggregation']['frac'])"
done
