#!/bin/bash
# round 4: the weight-gradient main loop chosen per wave (with / without the bias column sum):
# lab A/B and the bench line.  Usage (repo root, GPU box): bash tools/gpu_r04i.sh <tag>
set -u
TAG=${1:-r04i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 tools/lab/xs_lab wg > $OUT/lab_wg.txt 2>&1 || { echo "lab failed $?"; tail -5 $OUT/lab_wg.txt; exit 1; }
cat $OUT/lab_wg.txt
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt; cat $OUT/bench.txt
echo r04i-ok
