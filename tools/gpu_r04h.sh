#!/bin/bash
# round 4: the bias column sum on the matrix cores (weight-gradient lab A/B), the counters of the
# N = 48 data-gradient variants (lab dg3), and the general-order server step's VALU counters on
# configs[3]'s own epochs.  Usage (repo root, GPU box): bash tools/gpu_r04h.sh <tag>
set -u
TAG=${1:-r04h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 tools/lab/xs_lab wg > $OUT/lab_wg.txt 2>&1 || { echo "lab failed $?"; tail -5 $OUT/lab_wg.txt; exit 1; }
cat $OUT/lab_wg.txt
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
LAB_ITERS=1 timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/p_dg3 -o run \
    -- tools/lab/xs_lab dg3 > $OUT/p_dg3.log 2>&1 || { echo "pmc dg3 failed $?"; tail -5 $OUT/p_dg3.log; exit 1; }
VALU="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $VALU --output-format csv -d $OUT/p_c3 -o run \
    --kernel-include-regex "k_slab_step" -- python3 bench.py --n_workers 16384 --delays heterogeneous \
    --steps 2 --warmup 0 --no-cpu-baseline --no-stream --no-probe > $OUT/p_c3.log 2>&1 \
    || { echo "pmc c3 failed $?"; tail -5 $OUT/p_c3.log; exit 1; }
echo r04h-ok
