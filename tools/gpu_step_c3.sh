#!/bin/bash
# Server step on configs[3]'s own rule programs (epochs 1..6) + the seq/ref micro-benchmarks.
# Usage (repo root, GPU box): bash tools/gpu_step_c3.sh <tag>
set -u
TAG=${1:-c3}
mkdir -p gpurun_out
for T in 1 3 6; do
    timeout -k 10 180 python -u tools/step_bench.py c3 $T > gpurun_out/step_${TAG}_c3_$T.txt 2>&1 \
        || { echo "step_bench c3 $T failed"; tail -5 gpurun_out/step_${TAG}_c3_$T.txt; exit 1; }
    echo "== c3 $T"; sed -n 2,6p gpurun_out/step_${TAG}_c3_$T.txt
done
