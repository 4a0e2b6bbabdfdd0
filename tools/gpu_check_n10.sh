#!/bin/bash
# full GPU test suite, then the n = 10 and headline bench lines (no CPU baseline)
set -u
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" gpurun_out/pytest_gpu_$TAG.log | head -20; tail -5 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --n_workers 10 --delay 50 --steps 200 --warmup 10 \
    > gpurun_out/bench_${TAG}_n10.json 2> gpurun_out/bench_${TAG}_n10.err || { echo "n10 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_head.json 2> gpurun_out/bench_${TAG}_head.err || { echo "head failed"; exit 1; }
for V in n10 head; do
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$V.json')); a=d['aggregation']; print('$V', d['value'], d['ms_per_step'], 'agg', a['frac'], a['avg_launch_us'], a['alg_bytes_per_launch'])"
done
