#!/bin/bash
# A/B of one environment toggle on configs[1] (n = 10, d = 50, throttle, warm start): A, B, A, B.
# Usage (repo root, GPU box):  bash tools/gpu_ab_c1.sh <tag> <VAR> <valueA> <valueB>
set -u
TAG=$1; VAR=$2; A=$3; B=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/warm_start_file.py --out $OUT/warm_start_n10.pt > $OUT/warm.log 2>&1 \
    || { echo "warm start failed"; exit 1; }
run() {
    local name=$1 val=$2
    env $VAR=$val timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-stream --n_workers 10 \
        --delay 50 --model_file $OUT/warm_start_n10.pt --steps 200 --warmup 10 \
        > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed $?"; tail -5 $OUT/$name.err; return 1; }
    python3 tools/bench_summary.py $OUT/$name.json > $OUT/$name.txt; echo "== $name ($VAR=$val)"; head -3 $OUT/$name.txt
}
run c1_A $A && run c1_B $B && run c1_A2 $A && run c1_B2 $B && echo done
