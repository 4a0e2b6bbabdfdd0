#!/bin/bash
# Round-4 closing run on one MI355X: smoke, every GPU test (error census logged), the default
# bench line (CPU baseline included), a rocprofv3 kernel trace of the bench, and the 2-rank gloo
# rehearsal of the sharded path.  Usage (repo root, GPU box):  bash tools/gpu_final_r04.sh <tag>
set -u
OUT=gpurun_out/${1:-final_r04}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
    || { echo "smoke failed $?"; tail -5 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.txt
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt
head -3 $OUT/bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 \
    || { echo "trace failed $?"; exit 1; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --n_workers 256 \
    --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err \
    || { echo "gloo rehearsal failed $?"; tail -5 $OUT/bench_n2_gloo.err; exit 1; }
cut -c1-200 $OUT/bench_n2_gloo.json
echo final-ok
