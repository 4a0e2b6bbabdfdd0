#!/bin/bash
# round 4: conv2-4 inputs (a1, d1, a3) stored channel-slice-major: smoke, every GPU test, then the
# default bench line with its per-kernel times.  Usage (repo root, GPU box): bash tools/gpu_r04z.sh <tag>
set -u
TAG=${1:-r04z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
    || { echo "smoke failed $?"; tail -5 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt && head -30 $OUT/bench.txt
echo r04z-ok
