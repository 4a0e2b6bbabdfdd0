#!/bin/bash
# Max-chunk parity test, then vgg11 / vgg11_bn bench at chunk 32 vs 128.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k max_chunk -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_chunk.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_chunk.log; exit 1; }
tail -1 gpurun_out/pytest_chunk.log
for M in vgg11 vgg11_bn; do for C in 32 128; do
  timeout -k 10 300 python -u bench.py --model $M --chunk $C --steps 4 --warmup 1 --no-cpu-baseline \
      > gpurun_out/bench_${M}_chunk_$C.json 2> gpurun_out/bench_${M}_chunk_$C.err || { echo "$M chunk $C failed"; tail -5 gpurun_out/bench_${M}_chunk_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${M}_chunk_$C.json')); print('$M', $C, d['value'])"
done; done
