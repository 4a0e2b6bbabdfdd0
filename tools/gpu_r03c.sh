#!/bin/bash
# Round-3 measurement call: configs[1] (n = 10, d = 50, throttle, warm start) kernel trace and
# GPU idle share, the conv2 weight-gradient tile sweep after the k-major LDS store remap, and the
# LDS bank-conflict counter of the product's weight gradients.
# Usage (repo root, GPU box):  bash tools/gpu_r03c.sh <tag>
set -u
TAG=${1:-r03c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 tools/lab/direct_lab rfwd2 > $OUT/lab_resident.txt 2>&1 && \
    timeout -k 10 300 tools/lab/direct_lab rdg2 >> $OUT/lab_resident.txt 2>&1 \
    || { echo "resident lab failed $?"; tail -5 $OUT/lab_resident.txt; exit 1; }
cat $OUT/lab_resident.txt
timeout -k 10 120 python3 tools/warm_start_file.py --out $OUT/warm_start_n10.pt > $OUT/warm.log 2>&1 \
    || { echo "warm start failed"; tail -5 $OUT/warm.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --n_workers 10 --delay 50 \
    --model_file $OUT/warm_start_n10.pt --steps 200 --warmup 10 > $OUT/bench_configs1.json \
    2> $OUT/bench_configs1.err || { echo "configs1 bench failed $?"; tail -5 $OUT/bench_configs1.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench_configs1.json || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c1 -o run \
    -- python3 bench.py --no-cpu-baseline --no-probe --no-stream --n_workers 10 --delay 50 \
    --model_file $OUT/warm_start_n10.pt --steps 100 --warmup 10 > $OUT/trace_c1.log 2>&1 \
    || { echo "configs1 trace failed $?"; tail -5 $OUT/trace_c1.log; exit 1; }
python3 tools/trace_gaps.py $OUT/trace_c1 0.5 > $OUT/gaps_c1.txt 2>&1; head -40 $OUT/gaps_c1.txt
bash tools/gpu_lab.sh ${TAG}_wgx2 tools/lab/tile_lab wgx2 || exit 1
timeout -k 10 300 tools/lab/tile_lab "wg2 " > $OUT/lab_wg2.txt 2>&1 || { echo "lab2 failed $?"; exit 1; }
cat $OUT/lab_wg2.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv \
    -d $OUT/pmc_lds -o run --kernel-include-regex "gemm_kernel|gemm_direct|k_conv1_fwd" \
    -- python3 bench.py --n_workers 128 --no-throttle --steps 1 --warmup 0 --no-cpu-baseline \
    --no-probe --no-stream > $OUT/pmc_lds.log 2>&1 || { echo "pmc failed $?"; tail -5 $OUT/pmc_lds.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace_facade -o run \
    -- python3 tools/facade_bench.py --n_workers 256 --epochs 3 > $OUT/trace_facade.log 2>&1 \
    || { echo "facade trace failed $?"; tail -5 $OUT/trace_facade.log; exit 1; }
python3 tools/trace_gaps.py $OUT/trace_facade 0.5 > $OUT/gaps_facade.txt 2>&1; head -40 $OUT/gaps_facade.txt
echo done
