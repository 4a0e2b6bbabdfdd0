#!/bin/bash
# One GPU call: host facts, the GPU tests (optionally a -k filter), one bench line.
# Usage (repo root, on the GPU box):  bash tools/gpu_check.sh <tag> [pytest -k expression]
set -u
TAG=${1:-check}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
python3 - > gpurun_out/host_$TAG.txt 2>&1 <<'PY'
import os
print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"):
    try: print(f, open(f).read().strip())
    except OSError as e: print(f, e)
print("OMP_NUM_THREADS", os.environ.get("OMP_NUM_THREADS"))
m = [l for l in open("/proc/cpuinfo") if l.startswith("model name")]
print(m[0].strip() if m else "no model name", len(m))
PY
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
      > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
fi
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed $?"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
