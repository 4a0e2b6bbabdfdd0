#!/bin/bash
# A/B of one environment toggle on the headline bench only (A, B, A, B on one box).
# Usage (repo root, GPU box):  bash tools/gpu_ab_head.sh <tag> <VAR> <valueA> <valueB> [bench args]
set -u
TAG=$1; VAR=$2; A=$3; B=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1 val=$2
    env $VAR=$val timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-stream "${@:3}" \
        > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed $?"; tail -5 $OUT/$name.err; return 1; }
    python3 tools/bench_summary.py $OUT/$name.json > $OUT/$name.txt; echo "== $name ($VAR=$val)"; head -2 $OUT/$name.txt
}
run head_A "$A" "$@" || exit 1
run head_B "$B" "$@" || exit 1
run head_A2 "$A" "$@" || exit 1
run head_B2 "$B" "$@" || exit 1
echo done
