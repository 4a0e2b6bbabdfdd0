#!/bin/bash
# configs[1] (n = 10: 640-sample chunks) tuning data: the weight-gradient split floor
# (FLSIM_WSPLIT_KMIN) swept on the bench, and the forward / data-gradient tile variants at S = 640
# in the labs.  Usage (repo root, GPU box):  bash tools/gpu_r03d.sh <tag>
set -u
TAG=${1:-r03d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/warm_start_file.py --out $OUT/warm_start_n10.pt > $OUT/warm.log 2>&1 \
    || { echo "warm start failed"; tail -5 $OUT/warm.log; exit 1; }
for KMIN in 32 64 128 256; do
    FLSIM_WSPLIT_KMIN=$KMIN timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-stream \
        --n_workers 10 --delay 50 --model_file $OUT/warm_start_n10.pt --steps 200 --warmup 10 \
        > $OUT/bench_c1_kmin$KMIN.json 2> $OUT/bench_c1_kmin$KMIN.err \
        || { echo "configs1 kmin $KMIN failed $?"; tail -5 $OUT/bench_c1_kmin$KMIN.err; exit 1; }
    echo "kmin $KMIN"; python3 tools/bench_summary.py $OUT/bench_c1_kmin$KMIN.json | head -8
done
FLSIM_LAB_S=640 timeout -k 10 300 tools/lab/direct_lab > $OUT/lab_direct_s640.txt 2>&1 \
    || { echo "direct lab failed $?"; tail -5 $OUT/lab_direct_s640.txt; exit 1; }
FLSIM_LAB_S=640 timeout -k 10 300 tools/lab/tile_lab > $OUT/lab_tile_s640.txt 2>&1 \
    || { echo "tile lab failed $?"; tail -5 $OUT/lab_tile_s640.txt; exit 1; }
grep -E "TF/s" $OUT/lab_direct_s640.txt | head -80
echo done
