#!/bin/bash
# SQ counter passes over one chunk of the worker-batched GEMMs (n_workers 64 -> 32 computing
# workers = one chunk).  Usage (repo root, GPU box): bash tools/gemm_pmc.sh <tag> "<pass1>" "<pass2>" ...
set -u
TAG=$1; shift
OUT=gpurun_out/gemmpmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for PASS in "$@"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o run \
        --kernel-include-regex "gemm_kernel|aggregate_adam|k_pool" \
        -- python3 bench.py --n_workers 64 --steps 1 --warmup 0 --no-cpu-baseline --no-probe \
        > $OUT/p$i.log 2>&1 || { echo "pass $i ($PASS) failed $?"; tail -5 $OUT/p$i.log; exit 1; }
    echo "pass $i ok: $PASS"
done
