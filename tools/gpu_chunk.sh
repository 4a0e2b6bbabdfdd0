#!/bin/bash
# Headline bench at several worker-chunk sizes (workers per worker-batched launch).
set -u
mkdir -p gpurun_out
for C in 32 64 128 16; do
  timeout -k 10 300 python -u bench.py --chunk $C --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/bench_chunk_$C.json 2> gpurun_out/bench_chunk_$C.err || { echo "chunk $C failed"; tail -5 gpurun_out/bench_chunk_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_chunk_$C.json')); print($C, d['value'], d['roofline']['all_gemms'])"
done
