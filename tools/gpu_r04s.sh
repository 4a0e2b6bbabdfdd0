#!/bin/bash
# round 4: the fused conv1 test, and the conv6 weight-gradient tile A/B on one box (A B A B): 192x96 of 4 waves (default) against
# 192x192 of 8 waves (FLSIM_WG6_WIDE=1).  Usage (repo root, GPU box): bash tools/gpu_r04s.sh <tag>
set -u
TAG=${1:-r04s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread \
    -k "conv1_wgrad_fused" > $OUT/pytest.txt 2>&1
echo "pytest rc $?"; tail -2 $OUT/pytest.txt
run() {
    local name=$1; shift
    env "$@" timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-stream > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { echo "bench $name failed $?"; tail -5 $OUT/bench_$name.err; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); k=b['roofline']['per_kernel']['conv6_wgrad']; print('$name', b['value'], k)"
}
run a1 FLSIM_WG6_WIDE=0
run b1 FLSIM_WG6_WIDE=1
run a2 FLSIM_WG6_WIDE=0
run b2 FLSIM_WG6_WIDE=1
echo r04s-ok
