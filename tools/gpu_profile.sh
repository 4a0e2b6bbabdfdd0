#!/bin/bash
# Profiles bench.py on one MI355X: kernel-trace stats + separate PMC passes for HBM traffic.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}
shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline --no-probe}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1 || { echo "trace pass failed $?"; exit 1; }
echo "trace pass ok"
# HBM bytes of the aggregation kernel and the heaviest GEMMs, one counter group per pass
for PMC in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $PMC --output-format csv -d "$OUT/pmc_$PMC" -o run \
        --kernel-include-regex "k_slab_step|k_agg_stream|gemm_kernel|k_conv1_fwd|k_pool_scatter" \
        -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-probe \
        > "$OUT/bench_$PMC.log" 2>&1 || { echo "pmc $PMC failed $?"; exit 1; }
    echo "pmc $PMC ok"
done
