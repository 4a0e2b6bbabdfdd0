#!/bin/bash
# The BASELINE configs beyond the headline line, one MI355X (bench.py, no CPU baseline):
#   configs[1] n=10 d=50 throttle warm start | configs[2] n=1024 d=500 | configs[3] 16k workers,
#   heterogeneous delays (reference + independent entries) | configs[4] vgg11 n=4096 d=1000
# Usage (repo root, GPU box):  bash tools/gpu_configs_all.sh <tag>
set -u
TAG=${1:-cfg}
mkdir -p gpurun_out
run() {   # name, timeout, bench args...
    local name=$1 to=$2; shift 2
    timeout -k 10 $to python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_${TAG}_$name.json \
        2> gpurun_out/bench_${TAG}_$name.err || { echo "$name failed $?"; tail -5 gpurun_out/bench_${TAG}_$name.err; return 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$name.json')); a=d.get('aggregation') or {}; print('$name', d['value'], 'ws/s', d['ms_per_step'], 'ms/epoch', 'agg', a.get('probe'), a.get('frac'), a.get('avg_launch_us'))"
}
# configs[1]'s warm start: the sha-pinned fixture of the trajectory test (tests/golden/warm_n10.npz)
timeout -k 10 120 python -u tools/warm_start_file.py --out gpurun_out/warm_start.pt \
    > gpurun_out/make_warm_start_$TAG.log 2>&1 || { echo "warm start failed"; exit 1; }
run configs1_warm 300 --n_workers 10 --delay 50 --model_file gpurun_out/warm_start.pt --steps 200 --warmup 10 || exit 1
run configs2_d500 300 --n_workers 1024 --delay 500 --steps 8 --warmup 2 || exit 1
run configs3 600 --n_workers 16384 --delays heterogeneous --steps 3 --warmup 1 || exit 1
run configs3_indep 600 --n_workers 16384 --delays heterogeneous --semantics independent --steps 3 --warmup 1 || exit 1
run configs4_vgg11 400 --model vgg11 --n_workers 4096 --delay 1000 --steps 4 --warmup 1 || exit 1
