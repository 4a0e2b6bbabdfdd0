#!/bin/bash
# PerformantNet1 parity tests, then the headline bench (weight-gradient split change).
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_zw.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_zw.log; exit 1; }
tail -1 gpurun_out/pytest_zw.log
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_zw.json \
    2> gpurun_out/bench_zw.err || { echo "bench failed"; tail -5 gpurun_out/bench_zw.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_zw.json')); print(d['value'], d['roofline']['all_gemms'], d['mfma_efficiency_whole_step'])"
