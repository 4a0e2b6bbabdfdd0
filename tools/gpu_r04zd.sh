#!/bin/bash
# round 4: slice-order stores in the slice-major producer epilogues (conv2's pool epilogue -> d1,
# conv3's bias/ReLU epilogue -> a3) against row-order stores (tools/ab_sm/libflsim_rowstore.so, the
# previous commit), A B A B on one box, then every GPU test on the tree's library.  (Measured: conv3 2.66 -> 2.57 ms,
# conv2 5.64 -> 5.80; r04ze, with only conv3's epilogue in slice order, was flat: both reverted)
# Usage (repo root, GPU box): bash tools/gpu_r04zd.sh <tag>
set -u
TAG=${1:-r04zd}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1; shift
    env "$@" timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-stream > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { echo "bench $name failed $?"; tail -5 $OUT/bench_$name.err; exit 1; }
    python3 - "$OUT/bench_$name.json" "$name" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk = b["roofline"]["per_kernel"]
ks = ["conv2_fwd", "conv3_fwd", "conv4_fwd", "conv2_dgrad", "conv3_dgrad", "conv4_dgrad"]
print(sys.argv[2], round(b["value"], 1), " ".join(f"{k} {pk[k]['avg_ms']:.3f}" for k in ks if k in pk))
PY
}
run row1 FLSIM_LIB=tools/ab_sm/libflsim_rowstore.so
run sl1 FLSIM_X=0
run row2 FLSIM_LIB=tools/ab_sm/libflsim_rowstore.so
run sl2 FLSIM_X=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
echo r04zd-ok
