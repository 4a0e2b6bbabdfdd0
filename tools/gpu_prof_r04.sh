#!/bin/bash
# Round-4 profile of the shipped tree on one MI355X:
#   1. the default bench line (no CPU baseline);
#   2. rocprofv3 --kernel-trace --stats of the default bench (every GEMM, split-bf16 ones included);
#   3. PMC passes, one counter group per run, on ONE 128-worker chunk (bench.py --n_workers 128
#      --no-throttle, one epoch = 16,384 samples): FETCH_SIZE, WRITE_SIZE, and the SQ groups that
#      say where the GEMMs spend their cycles (MFMA busy, LDS instructions / conflicts / stalls,
#      VALU and VMEM instruction counts).  gfx950 slot limits: 8 SQ, 4 TCC (FETCH_SIZE 3,
#      WRITE_SIZE 2), 2 GRBM per pass.
#   4. tools/pmc_traffic.py (traffic table, math-tagged) and tools/pmc_summary.py.
# Usage (repo root, GPU box):  bash tools/gpu_prof_r04.sh <tag>
set -u
TAG=${1:-r04}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt
head -3 $OUT/bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > $OUT/trace.log 2>&1 \
    || { echo "trace failed $?"; tail -5 $OUT/trace.log; exit 1; }
echo "trace ok"
KREGEX="gemm_kernel|gemm_x6_kernel|gemm_dx6_kernel|gemm_direct_kernel|k_conv1_fwd|k_slab_step|k_pool_scatter"
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
  "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
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
TR=$OUT/traffic_in
mkdir -p $TR/pmc_FETCH_SIZE $TR/pmc_WRITE_SIZE $TR/trace
cp $(find $OUT/p1 -name "*counter_collection.csv" | head -1) $TR/pmc_FETCH_SIZE/run_counter_collection.csv
cp $(find $OUT/p2 -name "*counter_collection.csv" | head -1) $TR/pmc_WRITE_SIZE/run_counter_collection.csv
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
cp $OUT/kernel_stats.csv $TR/trace/run_kernel_stats.csv
python3 tools/pmc_traffic.py $TR $OUT/traffic.json > $OUT/traffic.txt && cat $OUT/traffic.txt
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
echo prof-ok
