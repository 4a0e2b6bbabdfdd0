#!/bin/bash
# configs[3] server-step programs for library builds A (in-tree) and B (flsim/_lib_b)
set -u
TAG=${1:-c3ab}
mkdir -p gpurun_out
for V in A B; do
    if [ $V = B ]; then export FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so; fi
    for T in 1 3 6; do
        timeout -k 10 180 python -u tools/step_bench.py c3 $T > gpurun_out/step_${TAG}_${V}_$T.txt 2>&1 \
            || { echo "step_bench $V c3 $T failed"; tail -5 gpurun_out/step_${TAG}_${V}_$T.txt; exit 1; }
        echo "== $V c3 $T $(sed -n 5p gpurun_out/step_${TAG}_${V}_$T.txt)"
    done
done
