#!/bin/bash
# configs[3] bench lines (reference and independent entries), one MI355X.
# Usage (repo root, GPU box): bash tools/gpu_configs3.sh <tag>
set -u
TAG=${1:-c3}
mkdir -p gpurun_out
for SEM in reference independent; do
    timeout -k 10 600 python -u bench.py --no-cpu-baseline --n_workers 16384 --delays heterogeneous \
        --semantics $SEM --steps 3 --warmup 1 > gpurun_out/bench_${TAG}_$SEM.json 2> gpurun_out/bench_${TAG}_$SEM.err \
        || { echo "$SEM failed $?"; tail -5 gpurun_out/bench_${TAG}_$SEM.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$SEM.json')); a=d['aggregation']; print('$SEM', d['value'], a['probe'], a['frac'], a['avg_launch_us'])"
done
