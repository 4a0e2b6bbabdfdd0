#!/bin/bash
# configs[1] A/B: small-chunk 128-row tiles (FLSIM_SMALL_S) and the round-filling weight-gradient
# split (FLSIM_WSPLIT_FILL), then the headline bench (the 128-worker chunk must be unchanged).
# Usage (repo root, GPU box):  bash tools/gpu_r03e.sh <tag>
set -u
TAG=${1:-r03e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/warm_start_file.py --out $OUT/warm_start_n10.pt > $OUT/warm.log 2>&1 \
    || { echo "warm start failed"; tail -5 $OUT/warm.log; exit 1; }
c1() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-stream \
        --n_workers 10 --delay 50 --model_file $OUT/warm_start_n10.pt --steps 200 --warmup 10 \
        > $OUT/bench_c1_$name.json 2> $OUT/bench_c1_$name.err \
        || { echo "configs1 $name failed $?"; tail -5 $OUT/bench_c1_$name.err; return 1; }
    echo "== $name"; python3 tools/bench_summary.py $OUT/bench_c1_$name.json > $OUT/sum_c1_$name.txt
    head -3 $OUT/sum_c1_$name.txt
}
c1 base FLSIM_SMALL_S=0 FLSIM_WSPLIT_FILL=0 || exit 1
c1 small FLSIM_SMALL_S=2048 FLSIM_WSPLIT_FILL=0 || exit 1
c1 fill FLSIM_SMALL_S=0 FLSIM_WSPLIT_FILL=1 || exit 1
c1 both FLSIM_SMALL_S=2048 FLSIM_WSPLIT_FILL=1 || exit 1
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench_head.json 2> $OUT/bench_head.err \
    || { echo "headline failed $?"; tail -5 $OUT/bench_head.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench_head.json > $OUT/sum_head.txt; head -3 $OUT/sum_head.txt
echo done
