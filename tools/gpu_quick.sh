#!/bin/bash
# Quick GPU check after a kernel change: the gradient parity tests of both networks, then the
# headline bench line without the CPU baseline.  Usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -u
TAG=${1:-quick}
K=${2:-"gradient or aggregate or trajectory"}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vgg.py -m gpu -x -q \
    -k "$K" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 \
    || { echo "pytest failed $?"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err || { echo "bench failed $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
