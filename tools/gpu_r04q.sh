#!/bin/bash
# round 4: stream concurrency on the 16k-sample chunks, same box: default, weight gradients on the
# side stream (FLSIM_CONCURRENT_BWD=16384), and that plus pipelined chunks (FLSIM_PIPELINE=1).
# Usage (repo root, GPU box): bash tools/gpu_r04q.sh <tag>
set -u
TAG=${1:-r04q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1; shift
    env "$@" timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-stream > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { echo "bench $name failed $?"; tail -5 $OUT/bench_$name.err; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); print('$name', b['value'], b['ms_per_step'])"
}
run base FLSIM_X=0
run cbwd FLSIM_CONCURRENT_BWD=16384
run cbwd_pipe FLSIM_CONCURRENT_BWD=16384 FLSIM_PIPELINE=1
run base2 FLSIM_X=0
echo r04q-ok
