#!/bin/bash
# configs[1]: warm-start test, synthesise warm_start.pt on the GPU, bench n = 10, d = 50,
# --throttle, --model_file warm_start.pt (one MI355X).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "warm_start or trajectory" -x -v \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_warm.log 2>&1 \
    || { echo "pytest failed"; tail -30 gpurun_out/pytest_warm.log; exit 1; }
tail -2 gpurun_out/pytest_warm.log
timeout -k 10 300 python -u tools/make_warm_start.py --epochs 500 --out gpurun_out/warm_start.pt \
    > gpurun_out/make_warm_start.log 2>&1 || { echo "warm start failed"; tail -20 gpurun_out/make_warm_start.log; exit 1; }
tail -3 gpurun_out/make_warm_start.log
timeout -k 10 300 python -u bench.py --n_workers 10 --delay 50 --model_file gpurun_out/warm_start.pt \
    --steps 200 --warmup 10 > gpurun_out/bench_configs1_warm.json 2> gpurun_out/bench_configs1_warm.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_configs1_warm.err; exit 1; }
cat gpurun_out/bench_configs1_warm.json
