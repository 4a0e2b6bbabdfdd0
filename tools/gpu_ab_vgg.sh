#!/bin/bash
# VGG correctness tests on build A, then the configs[4] bench for builds A (in-tree) and B (flsim/_lib_b)
set -u
TAG=${1:-abv}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vgg.py tests/test_gpu_vgg_bn.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for V in A B; do
    if [ $V = B ]; then export FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --model vgg11 --n_workers 4096 --delay 1000 --steps 4 --warmup 1 \
        > gpurun_out/bench_${TAG}_$V.json 2> gpurun_out/bench_${TAG}_$V.err || { echo "bench $V failed"; tail -5 gpurun_out/bench_${TAG}_$V.err; exit 1; }
done
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
a = json.load(open(f"gpurun_out/bench_{t}_A.json")); b = json.load(open(f"gpurun_out/bench_{t}_B.json"))
print("A", a["value"], "B", b["value"])
pa, pb = a["roofline"]["per_kernel"], b["roofline"]["per_kernel"]
for k in sorted(pa):
    print(f"{k:18s} A {pa[k]['avg_ms']:8.3f} {pa[k]['tflops']:6.1f}   B {pb[k]['avg_ms']:8.3f} {pb[k]['tflops']:6.1f}")
PY
