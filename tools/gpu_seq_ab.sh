#!/bin/bash
# Server-step micro-benchmarks for two library builds (A: in-tree, B: flsim/_lib_b), then the GPU
# tests on A.  Usage (repo root, GPU box): bash tools/gpu_seq_ab.sh <tag> [skip-tests]
set -u
TAG=${1:-seq}
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in A B; do
    if [ $V = B ]; then export FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so; fi
    for M in seq ref; do
        timeout -k 10 180 python -u tools/step_bench.py $M > gpurun_out/step_${TAG}_${V}_$M.txt 2>&1 \
            || { echo "step_bench $V $M failed"; tail -5 gpurun_out/step_${TAG}_${V}_$M.txt; exit 1; }
        echo "== $V $M"; head -4 gpurun_out/step_${TAG}_${V}_$M.txt
    done
done
unset FLSIM_LIB
[ "${2:-}" = skip-tests ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1; s=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
exit $s
