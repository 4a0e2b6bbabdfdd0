#!/bin/bash
# round 4: the direct split GEMM with the LH A ring (gemm_dx6.h: [l|h|m] registers, A[l|h] x B[h|l])
# against the product's form, on the forward shapes of conv2 / conv3 / conv4, B's third plane from
# LDS (p3) or swapped in registers.  Usage (repo root, GPU box): bash tools/gpu_r04w.sh <tag>
# (historical: the LH ring was removed after this run, profiles/r04/r04w; LAB_LH no longer exists)
set -u
TAG=${1:-r04w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for t in "fwd2v e" "fwd2 p3" "fwd3" "fwd4"; do
    LAB_LH=1 timeout -k 10 300 tools/lab/xs_lab "$t" >> $OUT/lab_lh.txt 2>&1 || { echo "lab $t failed $?"; tail -5 $OUT/lab_lh.txt; exit 1; }
done
cat $OUT/lab_lh.txt
echo r04w-ok
