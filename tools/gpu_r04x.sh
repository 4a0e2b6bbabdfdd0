#!/bin/bash
# round 4: texture-address / texture-data / vector-L1 counters of the GEMMs on one 128-worker chunk
# (what bounds the direct-A forward kernels).  One counter group per run (gfx950 limits: 2 TA, 2 TD,
# 4 TCP, 2 GRBM per pass).  Usage (repo root, GPU box): bash tools/gpu_r04x.sh <tag>
set -u
TAG=${1:-r04x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || { echo "list-avail failed $?"; }
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" $OUT/avail.txt | sort -u > $OUT/avail_tatdtcp.txt || true
KREGEX="gemm_kernel|gemm_x6_kernel|gemm_dx6_kernel|gemm_direct_kernel|k_conv1_fwd"
PASSES=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
  "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
  "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
)
i=0
for PASS in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o run \
        --kernel-include-regex "$KREGEX" \
        -- python3 bench.py --n_workers 128 --no-throttle --steps 1 --warmup 0 \
        --no-cpu-baseline --no-probe --no-stream > $OUT/p$i.log 2>&1 \
        || { echo "pass $i ($PASS) failed $?"; tail -5 $OUT/p$i.log; exit 1; }
    echo "pass $i ok: $PASS"
done
python3 tools/pmc_summary_ta.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
echo r04x-ok
