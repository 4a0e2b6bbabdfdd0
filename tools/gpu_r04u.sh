#!/bin/bash
# round 4: the general-order interpreter with consecutive words overlapped (casc_run_macro_pipe,
# default; FLSIM_CASC_PIPE=0 = word at a time): bit-exact tests, then configs[3]'s bench line both ways.
# (historical: the interpreter was removed after this run, profiles/r04/r04u; the script no longer applies)
# Usage (repo root, GPU box): bash tools/gpu_r04u.sh <tag>
set -u
TAG=${1:-r04u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_server_step.py tests/test_gpu_configs.py \
    -v --timeout 300 --timeout-method thread -k "general_order or aggregate or fused or stream or heterogeneous or configs3" \
    > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest.txt; grep -E "^FAILED" $OUT/pytest.txt | head
[ $rc -eq 0 ] || exit 1
run() {
    local name=$1; shift
    env "$@" timeout -k 10 600 python3 -u bench.py --n_workers 16384 --delays heterogeneous --no-cpu-baseline \
        --no-stream --steps 3 --warmup 1 > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { echo "bench $name failed $?"; tail -5 $OUT/bench_$name.err; exit 1; }
    python3 -c "import json; b=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); a=b['aggregation']; print('$name', b['value'], a['avg_launch_us'], a['frac'])"
}
run pipe FLSIM_CASC_PIPE=1
run word FLSIM_CASC_PIPE=0
run pipe2 FLSIM_CASC_PIPE=1
echo r04u-ok
