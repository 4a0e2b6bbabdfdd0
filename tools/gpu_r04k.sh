#!/bin/bash
# round 4: conv2 forward on 4-wave 64-row blocks, conv3 weight gradient on 96x96 tiles (every GPU test,
# the bench line) and the lab's direct-kernel sweeps.  Usage (repo root, GPU box): bash tools/gpu_r04k.sh <tag>
set -u
TAG=${1:-r04k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt; cat $OUT/bench.txt
for T in fwd2v fwd3v fwd4v; do
    timeout -k 10 300 tools/lab/xs_lab $T > $OUT/lab_$T.txt 2>&1 || { echo "lab $T failed $?"; tail -5 $OUT/lab_$T.txt; exit 1; }
    cat $OUT/lab_$T.txt
done
echo r04k-ok
