#!/bin/bash
# correctness subset on build A, then bench.py for builds A (in-tree) and B (flsim/_lib_b)
set -u
TAG=${1:-ab}; K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
        > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_$TAG.log
fi
for V in A B; do
    if [ $V = B ]; then export FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$V.json 2> gpurun_out/bench_${TAG}_$V.err \
        || { echo "bench $V failed"; tail -5 gpurun_out/bench_${TAG}_$V.err; exit 1; }
done
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
a = json.load(open(f"gpurun_out/bench_{t}_A.json")); b = json.load(open(f"gpurun_out/bench_{t}_B.json"))
print("A", a["value"], "B", b["value"])
pa, pb = a["roofline"]["per_kernel"], b["roofline"]["per_kernel"]
for k in sorted(pa):
    print(f"{k:16s} A {pa[k]['avg_ms']:8.3f} {pa[k]['tflops']:6.1f}   B {pb[k]['avg_ms']:8.3f} {pb[k]['tflops']:6.1f}")
PY
