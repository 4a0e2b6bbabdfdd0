#!/bin/bash
# round 4: bounds at 1.5x the split build's measured errors (every GPU test), the in-slot tick
# (bench stream probe), configs[3]'s general-order step, and the VALU-issue counters of the server
# step kernels.  Usage (repo root, GPU box): bash tools/gpu_r04g.sh <tag>
set -u
TAG=${1:-r04g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FLSIM_FLIP_LOG=$OUT/flips.jsonl FLSIM_TOL_LOG=$OUT/tol.jsonl timeout -k 10 900 python3 -u -m pytest \
    tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc $rc"; tail -2 $OUT/pytest_gpu.txt; grep -E "^FAILED" $OUT/pytest_gpu.txt | head
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json > $OUT/bench.txt; head -4 $OUT/bench.txt
python3 -c "import json,sys; b=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(json.dumps(b['aggregation_stream']))"
timeout -k 10 400 python3 -u bench.py --n_workers 16384 --delays heterogeneous --no-cpu-baseline \
    --no-stream > $OUT/bench_configs3.json 2> $OUT/bench_configs3.err \
    || { echo "configs3 bench failed $?"; tail -5 $OUT/bench_configs3.err; exit 1; }
python3 -c "import json,sys; b=json.loads(open('$OUT/bench_configs3.json').read().strip().splitlines()[-1]); print(b['value'], json.dumps(b['aggregation']))"
timeout -k 10 180 python3 -u tools/agg_bench.py > $OUT/agg_bench.txt 2>&1 \
    || { echo "agg_bench failed $?"; tail -5 $OUT/agg_bench.txt; exit 1; }
cat $OUT/agg_bench.txt
VALU="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $VALU --output-format csv -d $OUT/p_seq -o run \
    --kernel-include-regex "k_slab_step" -- python3 tools/step_bench.py c3 3 > $OUT/p_seq.log 2>&1 \
    || { echo "pmc seq failed $?"; tail -5 $OUT/p_seq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $VALU --output-format csv -d $OUT/p_agg -o run \
    --kernel-include-regex "k_agg_stream" -- python3 tools/agg_bench.py --iters 5 > $OUT/p_agg.log 2>&1 \
    || { echo "pmc agg failed $?"; tail -5 $OUT/p_agg.log; exit 1; }
echo r04g-ok
