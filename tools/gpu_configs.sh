#!/bin/bash
# configs[3] (16k workers, heterogeneous delays) and configs[4] (vgg11, 4096 workers, d = 1000)
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --n_workers 16384 --delays heterogeneous --steps 4 --warmup 1 \
    --no-cpu-baseline > gpurun_out/bench_configs3.json 2> gpurun_out/bench_configs3.err \
    || { echo "configs3 failed"; tail -5 gpurun_out/bench_configs3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_configs3.json')); print('configs3', d['value'], d['ms_per_step'])"
timeout -k 10 500 python -u bench.py --model vgg11 --n_workers 4096 --delay 1000 --steps 4 --warmup 1 \
    --no-cpu-baseline > gpurun_out/bench_configs4.json 2> gpurun_out/bench_configs4.err \
    || { echo "configs4 failed"; tail -5 gpurun_out/bench_configs4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_configs4.json')); print('configs4', d['value'], d['ms_per_step'])"
