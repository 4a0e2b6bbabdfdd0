#!/bin/bash
# Per-tensor gradient error census of the VGG teacher-forced tests under two libraries.
# Usage (repo root, GPU box):  bash tools/gpu_tol_ab.sh <tag> <libA> <libB>
set -u
TAG=$1; A=$2; B=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for side in A B; do
    lib=$A; [ $side = B ] && lib=$B
    FLSIM_LIB=$lib FLSIM_TOL_LOG=$OUT/tol_$side.jsonl timeout -k 10 400 python3 -u -m pytest \
        tests/test_gpu_vgg.py tests/test_gpu_vgg_bn.py -q -k teacher_forced \
        --timeout 300 --timeout-method thread > $OUT/pytest_$side.log 2>&1
    rc=$?
    echo "side $side ($lib): pytest rc $rc"; tail -2 $OUT/pytest_$side.log
    [ $rc -ge 2 ] && exit $rc
done
python3 - $OUT <<'PY'
import json, sys
out = sys.argv[1]
for side in "AB":
    for l in open(f"{out}/tol_{side}.jsonl"):
        r = json.loads(l)
        w = r["worst"]
        k = max(w, key=w.get)
        print(side, r["test"].split("::")[-1][:60], "max %.3e (%s)" % (w[k], k))
PY
echo done
