#!/bin/bash
# One GPU call: parity tests, rocprofv3 trace + PMC passes, HBM traffic table, then the bench line
# (which reads the traffic table).  Usage (repo root, on the GPU box):  bash tools/gpu_round.sh <tag>
set -u
TAG=${1:-r01}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${K:+-k "$K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_profile.sh $TAG || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_$TAG gpurun_out/prof_$TAG/traffic.json profiles/traffic.json || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
