#!/bin/bash
# Interpreter lab + server-step micro-benchmarks (+ optionally the server-step GPU tests).
# Usage (repo root, GPU box): bash tools/gpu_seq.sh <tag> [pytest -k expression]
set -u
TAG=${1:-seq}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/lab/casc_lab > gpurun_out/lab_casc_$TAG.txt 2>&1 || { echo "lab failed"; tail -5 gpurun_out/lab_casc_$TAG.txt; exit 1; }
cat gpurun_out/lab_casc_$TAG.txt
for M in seq ref; do
    timeout -k 10 180 python -u tools/step_bench.py $M > gpurun_out/step_${TAG}_$M.txt 2>&1 \
        || { echo "step_bench $M failed"; tail -5 gpurun_out/step_${TAG}_$M.txt; exit 1; }
    echo "== $M"; sed -n 2,6p gpurun_out/step_${TAG}_$M.txt
done
[ -z "${2:-}" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1; s=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
exit $s
