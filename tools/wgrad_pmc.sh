#!/bin/bash
# PMC characterisation of the worker-batched GEMMs on ONE 128-worker chunk (16,384 samples):
# bench.py --n_workers 128 --no-throttle, one epoch = 127 fast + the slow worker = one chunk.
# Each counter set is its own rocprofv3 pass (gfx950 slot limits: 8 SQ, 4 TCC with FETCH_SIZE = 3
# and WRITE_SIZE = 2).  Usage (repo root, GPU box):  bash tools/wgrad_pmc.sh <tag>
set -u
TAG=${1:-r03}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_available.txt 2>&1 || true
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
  "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for PASS in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o run \
        --kernel-include-regex "gemm_kernel|gemm_direct|k_conv1_fwd" \
        -- python3 bench.py --n_workers 128 --no-throttle --steps 1 --warmup 0 \
        --no-cpu-baseline --no-probe --no-stream > $OUT/p$i.log 2>&1 \
        || { echo "pass $i ($PASS) failed $?"; tail -5 $OUT/p$i.log; exit 1; }
    echo "pass $i ok: $PASS"
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
