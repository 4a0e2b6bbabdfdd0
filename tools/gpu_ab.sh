#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_ntA.json 2> gpurun_out/bench_ntA.err || { echo "bench A failed"; tail -5 gpurun_out/bench_ntA.err; exit 1; }
FLSIM_LIB=$PWD/fl-distributed-delay_amd/flsim/_lib_b/libflsim.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_ntB.json 2> gpurun_out/bench_ntB.err || { echo "bench B failed"; tail -5 gpurun_out/bench_ntB.err; exit 1; }
python3 - <<'PY'
import json
for t in "AB":
    d = json.load(open(f"gpurun_out/bench_nt{t}.json"))
    pk = d["roofline"]["per_kernel"]
    print(t, d["value"], " ".join(f"{k}:{v['avg_ms']:.3f}" for k, v in sorted(pk.items())))
PY
