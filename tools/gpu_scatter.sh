#!/bin/bash
# PerformantNet1 parity tests, then bench + rocprofv3 kernel stats of the pool scatters.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_scatter.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_scatter.log; exit 1; }
tail -1 gpurun_out/pytest_scatter.log
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_scatter.json \
    2> gpurun_out/bench_scatter.err || { echo "bench failed"; exit 1; }
cut -c1-330 gpurun_out/bench_scatter.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scatter -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe > gpurun_out/prof_scatter.log 2>&1 \
    || { echo "trace failed"; exit 1; }
grep -h pool_scatter gpurun_out/prof_scatter/run_kernel_stats.csv | cut -c1-160
