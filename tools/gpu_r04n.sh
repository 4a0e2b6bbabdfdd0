#!/bin/bash
# round 4: conv1's weight gradient fused into conv2's data gradient (c1fuse.h): every GPU test,
# the bench line fused and unfused (FLSIM_C1_FUSE=0).  Usage (repo root, GPU box): bash tools/gpu_r04n.sh <tag>
set -u
TAG=${1:-r04n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# (run when the fused path was the default; since then FLSIM_C1_FUSE=1 selects it)
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt; head -9 $OUT/bench.txt
FLSIM_C1_FUSE=0 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench_unfused.json 2> $OUT/bench_unfused.err \
    || { echo "bench unfused failed $?"; tail -5 $OUT/bench_unfused.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench_unfused.json > $OUT/bench_unfused.txt; head -9 $OUT/bench_unfused.txt
echo r04n-ok
