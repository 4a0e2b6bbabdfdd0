#!/bin/bash
# VGG parity tests, then vgg11 / vgg11_bn benches (weight-gradient split change).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vgg.py tests/test_gpu_vgg_bn.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_vggzw.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_vggzw.log; exit 1; }
tail -1 gpurun_out/pytest_vggzw.log
for M in vgg11 vgg11_bn; do
  timeout -k 10 300 python -u bench.py --model $M --steps 4 --warmup 1 --no-cpu-baseline \
      > gpurun_out/bench_${M}_zw.json 2> gpurun_out/bench_${M}_zw.err || { echo "$M failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${M}_zw.json')); print('$M', d['value'])"
done
