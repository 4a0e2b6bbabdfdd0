#!/bin/bash
# round 4: GPU tests with the precision census, bench line, rocprofv3 profile + counters, then the
# planar-LDS lab.  Usage (repo root, GPU box): bash tools/gpu_r04e.sh <tag>
set -u
TAG=${1:-r04e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest.txt; grep -E "^FAILED" $OUT/pytest.txt | head
[ $rc -le 1 ] || exit $rc
bash tools/gpu_prof_r04.sh $TAG || exit 1
timeout -k 10 300 tools/lab/xq_lab > $OUT/lab_xq.txt 2>&1 || { echo "xq lab failed $?"; tail -5 $OUT/lab_xq.txt; exit 1; }
cat $OUT/lab_xq.txt
