#!/bin/bash
# weight-gradient split floor (FLSIM_WSPLIT_KMIN) on configs[1]-sized chunks and the headline
set -u
TAG=${1:-ws}
mkdir -p gpurun_out
for K in 0 16 32 64; do
    FLSIM_WSPLIT_KMIN=$K timeout -k 10 300 python -u bench.py --no-cpu-baseline --n_workers 10 --delay 50 --steps 200 --warmup 10 \
        > gpurun_out/bench_${TAG}_n10_k$K.json 2> gpurun_out/bench_${TAG}_n10_k$K.err || { echo "n10 k$K failed"; tail -5 gpurun_out/bench_${TAG}_n10_k$K.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_n10_k$K.json')); pk=d['roofline']['per_kernel']; print('n10 kmin $K', d['value'], d['ms_per_step'], ' '.join(f\"{k}:{v['avg_ms']:.3f}\" for k,v in sorted(pk.items()) if 'wgrad' in k))"
done
for K in 0 32; do
    FLSIM_WSPLIT_KMIN=$K timeout -k 10 300 python -u bench.py --no-cpu-baseline \
        > gpurun_out/bench_${TAG}_head_k$K.json 2> gpurun_out/bench_${TAG}_head_k$K.err || { echo "head k$K failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_head_k$K.json')); print('headline kmin $K', d['value'], d['ms_per_step'])"
done
