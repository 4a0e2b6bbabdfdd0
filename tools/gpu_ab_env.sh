#!/bin/bash
# A/B of one environment toggle on the headline bench and on configs[1], same box, interleaved.
# Usage (repo root, GPU box):  bash tools/gpu_ab_env.sh <tag> <VAR> <valueA> <valueB>
set -u
TAG=$1; VAR=$2; A=$3; B=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/warm_start_file.py --out $OUT/warm_start_n10.pt > $OUT/warm.log 2>&1 \
    || { echo "warm start failed"; exit 1; }
run() {   # name value args...
    local name=$1 val=$2; shift 2
    env $VAR=$val timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-stream "$@" \
        > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed $?"; tail -5 $OUT/$name.err; return 1; }
    python3 tools/bench_summary.py $OUT/$name.json > $OUT/$name.txt; echo "== $name ($VAR=$val)"; head -2 $OUT/$name.txt
}
C1="--n_workers 10 --delay 50 --model_file $OUT/warm_start_n10.pt --steps 200 --warmup 10"
run head_A $A || exit 1
run head_B $B || exit 1
run c1_A $A $C1 || exit 1
run c1_B $B $C1 || exit 1
run head_A2 $A || exit 1
run head_B2 $B || exit 1
echo done
