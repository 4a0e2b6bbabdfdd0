#!/bin/bash
# round 4: split-form operand lab, then the split-operand product: smoke, every GPU test (error
# census logged), the default bench line.  Usage (repo root, GPU box): bash tools/gpu_r04b.sh <tag>
set -u
TAG=${1:-r04b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ "${LAB:-1}" = 0 ] || timeout -k 10 300 tools/lab/xs_lab > $OUT/lab_xs.txt 2>&1 || { echo "lab failed $?"; tail -5 $OUT/lab_xs.txt; exit 1; }
[ "${LAB:-1}" = 0 ] || cat $OUT/lab_xs.txt
FLSIM_CONCURRENT_BWD=0 timeout -k 10 200 python3 -u tools/dbg_split.py 1 0 > $OUT/dbg.txt 2>&1 && grep grad $OUT/dbg.txt | head -12
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
    || { echo "smoke failed $?"; tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.txt
grep -E "FAILED|ERROR" $OUT/pytest_gpu.txt | head -20
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt
cat $OUT/bench.txt
