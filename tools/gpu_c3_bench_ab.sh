#!/bin/bash
# configs[3] reference-semantics bench line for build A, A without unit interleave, and build B
# (flsim/_lib_b): the general-order server step's probe.  Usage: bash tools/gpu_c3_bench_ab.sh <tag>
set -u
TAG=${1:-c3ab}
mkdir -p gpurun_out
run() {
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --n_workers 16384 --delays heterogeneous \
        --steps 3 --warmup 1 > gpurun_out/bench_${TAG}_$1.json 2> gpurun_out/bench_${TAG}_$1.err \
        || { echo "$1 failed"; tail -5 gpurun_out/bench_${TAG}_$1.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$1.json')); a=d['aggregation']; print('$1', d['value'], a['frac'], a['avg_launch_us'])"
}
run A
FLSIM_STEP_NO_INTERLEAVE=1 run A_noil
FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so run B
