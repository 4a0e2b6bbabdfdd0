#!/bin/bash
# Server-step micro-benchmarks (tools/step_bench.py seq|ref) for library builds A (in-tree) and
# B (flsim/_lib_b).  Usage (repo root, GPU box): bash tools/gpu_step_ab.sh <tag>
set -u
TAG=${1:-ab}
mkdir -p gpurun_out
for V in A B; do
    if [ $V = B ]; then export FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so; fi
    for M in seq ref; do
        timeout -k 10 180 python -u tools/step_bench.py $M > gpurun_out/step_${TAG}_${V}_$M.txt 2>&1 \
            || { echo "step_bench $V $M failed"; tail -5 gpurun_out/step_${TAG}_${V}_$M.txt; exit 1; }
        echo "== $V $M"; sed -n 3,6p gpurun_out/step_${TAG}_${V}_$M.txt
    done
done
