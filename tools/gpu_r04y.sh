#!/bin/bash
# round 4: the direct split GEMM over a channel-slice-major input ([img][CI/16][H][W][16]: the
# 16 rows of a fragment read whole cache lines) against the product's pixel-major input, on the
# conv2 / conv3 / conv4 forward shapes (r04x: the texture path is 84-89 % busy there).
# Usage (repo root, GPU box): bash tools/gpu_r04y.sh <tag>
set -u
TAG=${1:-r04y}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for t in "fwd2v e" "fwd3" "fwd4"; do
    LAB_SM=1 timeout -k 10 300 tools/lab/xs_lab "$t" >> $OUT/lab_sm.txt 2>&1 || { echo "lab $t failed $?"; tail -5 $OUT/lab_sm.txt; exit 1; }
done
cat $OUT/lab_sm.txt
echo r04y-ok
