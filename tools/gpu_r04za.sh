#!/bin/bash
# round 4: A B A B on one box, pixel-major conv2-4 inputs (tools/abx/libflsim_pm.so, built from the
# previous commit plus a stub of flsim_pn1_workspace_slice_major returning 0) against channel-slice-major (the tree's libflsim.so, dgrad masks applied in LDS),
# then every GPU test on the tree's library.  Usage (repo root, GPU box): bash tools/gpu_r04za.sh <tag>
# (tools/abx is listed in .gpurunignore since the round-4 A/B runs: copy the library back in to rerun)
set -u
TAG=${1:-r04za}
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
ks = ["conv2_fwd", "conv3_fwd", "conv4_fwd", "conv2_dgrad", "conv3_dgrad", "conv4_dgrad", "conv2_wgrad", "conv3_wgrad", "conv4_wgrad"]
print(sys.argv[2], round(b["value"], 1), " ".join(f"{k} {pk[k]['avg_ms']:.3f}" for k in ks if k in pk))
PY
}
run pm1 FLSIM_LIB=tools/abx/libflsim_pm.so
run sm1 FLSIM_X=0
run pm2 FLSIM_LIB=tools/abx/libflsim_pm.so
run sm2 FLSIM_X=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
echo r04za-ok
