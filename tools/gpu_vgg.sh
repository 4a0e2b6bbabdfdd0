#!/bin/bash
# One GPU call for the VGG-11 engine: its parity tests, the PerformantNet1 tests (shared kernels),
# then a short configs[4] bench line.  Usage (repo root, GPU box): bash tools/gpu_vgg.sh <tag>
set -u
TAG=${1:-vgg}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_vgg.py tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 \
    || { echo "pytest failed $?"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench.py --model vgg11 --n_workers 4096 --delay 1000 --steps 2 \
    --warmup 1 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
