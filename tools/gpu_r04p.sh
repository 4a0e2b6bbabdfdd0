#!/bin/bash
# round 4: the persistent pipelined stream after the all-reduce (FLSIM_AGG_PIPE=1): its bit-exact
# tests, the stream micro-benchmark (all forms, same box) and the bench line's stream probe with it.
# Usage (repo root, GPU box): bash tools/gpu_r04p.sh <tag>
set -u
TAG=${1:-r04p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_server_step.py tests/test_gpu_parity.py -v \
    --timeout 300 --timeout-method thread -k "stream or aggregate or fused" > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest.txt; grep -E "^FAILED" $OUT/pytest.txt | head
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/agg_bench.py > $OUT/agg_bench.txt 2>&1 \
    || { echo "agg_bench failed $?"; tail -5 $OUT/agg_bench.txt; exit 1; }
cat $OUT/agg_bench.txt
FLSIM_AGG_PIPE=1 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench_pipe.json 2> $OUT/bench_pipe.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench_pipe.err; exit 1; }
python3 -c "import json; b=json.loads(open('$OUT/bench_pipe.json').read().strip().splitlines()[-1]); print(b['value'], json.dumps(b['aggregation_stream']))"
echo r04p-ok
