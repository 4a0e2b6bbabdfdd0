#!/bin/bash
# Per-rank load probe on one MI355X: the bench at the worker counts one rank of an N-GPU job
# computes (n=1024/N active-equivalent) and configs[1] (n=10).  Usage: bash tools/gpu_sizes.sh <tag>
set -u
TAG=${1:-sizes}
mkdir -p gpurun_out/sizes_$TAG
export TMPDIR=/tmp
for spec in "10 50 40" "128 50 8" "256 50 8" "512 50 8"; do
    set -- $spec
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --n_workers $1 --delay $2 --steps $3 \
        > gpurun_out/sizes_$TAG/n$1.json 2> gpurun_out/sizes_$TAG/n$1.err \
        || { echo "bench n=$1 failed $?"; tail -20 gpurun_out/sizes_$TAG/n$1.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['all_gemms'])" gpurun_out/sizes_$TAG/n$1.json n=$1
done
