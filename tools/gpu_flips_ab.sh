#!/bin/bash
# Decision-flip census (tests/_flips.py) of the GPU parity tests under two libraries.
# Usage (repo root, GPU box):  bash tools/gpu_flips_ab.sh <tag> <libA> <libB>
set -u
TAG=$1; A=$2; B=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for side in A B; do
    lib=$A; [ $side = B ] && lib=$B
    FLSIM_LIB=$lib FLSIM_FLIP_LOG=$OUT/flips_$side.jsonl timeout -k 10 500 python3 -u -m pytest \
        tests/test_gpu_parity.py tests/test_gpu_facade.py tests/test_gpu_configs.py -q \
        --timeout 300 --timeout-method thread > $OUT/pytest_$side.log 2>&1
    rc=$?
    echo "side $side ($lib): pytest rc $rc"; tail -3 $OUT/pytest_$side.log
    [ $rc -ge 2 ] && exit $rc
done
python3 - $OUT <<'PY'
import json, sys
out = sys.argv[1]
for side in "AB":
    try:
        rows = [json.loads(l) for l in open(f"{out}/flips_{side}.jsonl")]
    except FileNotFoundError:
        rows = []
    for r in rows:
        print(side, r["test"].split("::")[-1][:60], "tf %.2e" % r["tf"], "gpu", sum(r["flips_gpu"].values()),
              "cpu32", sum(r["flips_cpu32"].values()))
PY
echo done
