#!/bin/bash
# round 4: conv6 weight gradient on 192x192 tiles, conv1 stores reverted (parity subset, bench line) and the
# staged-tile sweep of the N = 192 / 96 forward and data-gradient GEMMs.  Usage (repo root, GPU box): bash tools/gpu_r04m.sh <tag>
set -u
TAG=${1:-r04m}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread \
    -k "single_worker or chunk_of_workers or teacher_forced or max_chunk" > $OUT/pytest_parity.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_parity.txt; grep -E "^FAILED" $OUT/pytest_parity.txt | head
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt; head -8 $OUT/bench.txt
for T in fwd6 dg6 fwd5 dg5 dg4; do
    timeout -k 10 300 tools/lab/xs_lab "$T" > $OUT/lab_$T.txt 2>&1 || { echo "lab $T failed $?"; tail -5 $OUT/lab_$T.txt; exit 1; }
    cat $OUT/lab_$T.txt
done
echo r04m-ok
