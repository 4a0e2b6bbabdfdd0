#!/bin/bash
# A/B of the split-bf16 accumulation (gemm_x6.h FLSIM_X6_FRESH): the precision tests with error
# census logs on both libraries, the lab (fresh build) and the default bench line.
set -u
OUT=gpurun_out/${1:-fresh_ab}
mkdir -p $OUT
export TMPDIR=/tmp
K="teacher_forced or flip or worker_step or tf_ or trajectory_drift"
FLSIM_LIB=build/nofresh/libflsim.so FLSIM_FLIP_LOG=$OUT/flips_nofresh.jsonl FLSIM_TOL_LOG=$OUT/tol_nofresh.jsonl \
    timeout -k 10 700 python3 -u -m pytest tests -m gpu -k "$K" -v -s --timeout 300 --timeout-method thread > $OUT/pytest_nofresh.txt 2>&1
echo "nofresh rc $?"; tail -2 $OUT/pytest_nofresh.txt
FLSIM_FLIP_LOG=$OUT/flips_fresh.jsonl FLSIM_TOL_LOG=$OUT/tol_fresh.jsonl \
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_fresh.txt 2>&1
rc=$?
echo "fresh rc $rc"; tail -2 $OUT/pytest_fresh.txt; grep -E "^FAILED" $OUT/pytest_fresh.txt | head
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 tools/lab/xs_lab > $OUT/lab_xs_fresh.txt 2>&1 || { echo "lab failed $?"; exit 1; }
cat $OUT/lab_xs_fresh.txt
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json | head -30
timeout -k 10 300 tools/lab/xp_lab > $OUT/lab_xp.txt 2>&1 || { echo "xp lab failed $?"; tail -5 $OUT/lab_xp.txt; exit 1; }
cat $OUT/lab_xp.txt
timeout -k 10 300 tools/lab/xq_lab > $OUT/lab_xq.txt 2>&1 || { echo "xq lab failed $?"; tail -5 $OUT/lab_xq.txt; exit 1; }
cat $OUT/lab_xq.txt
bash tools/gpu_prof_r04.sh r04d || exit 1
