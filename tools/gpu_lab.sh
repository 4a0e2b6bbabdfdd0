#!/bin/bash
# Run a lab binary, then one FETCH_SIZE pass and one clock/MFMA-busy pass over it (GPU box).
# Usage: bash tools/gpu_lab.sh <tag> <binary> [filter]
set -u
TAG=$1; BIN=$2; FILT=${3:-}
OUT=gpurun_out/lab_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 $BIN $FILT > $OUT/time.txt 2>&1 || { echo "lab failed $?"; tail -5 $OUT/time.txt; exit 1; }
cat $OUT/time.txt
export LAB_ITERS=1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $BIN $FILT \
    > $OUT/fetch.log 2>&1 || { echo "fetch pass failed $?"; tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/clk -o run -- $BIN $FILT \
    > $OUT/clk.log 2>&1 || { echo "clk pass failed $?"; tail -5 $OUT/clk.log; exit 1; }
echo done
