#!/bin/bash
# round 4: the k-major LDS stride fix: bench line, weight-gradient lab, GPU tests, and the LDS
# conflict counters of the weight gradients.  Usage (repo root, GPU box): bash tools/gpu_r04f.sh <tag>
set -u
TAG=${1:-r04f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt; head -30 $OUT/bench.txt
timeout -k 10 300 tools/lab/xs_lab wg > $OUT/lab_wg.txt 2>&1 || { echo "lab failed $?"; tail -5 $OUT/lab_wg.txt; exit 1; }
cat $OUT/lab_wg.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p_lds -o run \
    --kernel-include-regex "gemm_x6_kernel" -- python3 bench.py --n_workers 128 --no-throttle --steps 1 --warmup 0 \
    --no-cpu-baseline --no-probe --no-stream > $OUT/p_lds.log 2>&1 || { echo "pmc failed $?"; tail -5 $OUT/p_lds.log; exit 1; }
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest.txt; grep -E "^FAILED" $OUT/pytest.txt | head
