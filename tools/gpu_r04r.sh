#!/bin/bash
# round 4: the fused conv1 weight-gradient test (FLSIM_C1_FUSE switched in-process).
# Usage (repo root, GPU box): bash tools/gpu_r04r.sh <tag>
set -u
TAG=${1:-r04r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread \
    -k "conv1_wgrad_fused or chunk_of_workers" > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -3 $OUT/pytest.txt; grep -E "^FAILED|Error" $OUT/pytest.txt | head
exit $rc
