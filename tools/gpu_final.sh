#!/bin/bash
# Round-closing GPU call: the full round (tests, rocprofv3 trace + PMC passes, traffic table,
# headline bench), smoke(), and the configs[2] delay-500 bench line.
set -u
TAG=${1:-r01e}
bash tools/gpu_round.sh $TAG || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py --delay 500 --steps 8 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_d500_$TAG.json 2> gpurun_out/bench_d500_$TAG.err \
    || { echo "bench d500 failed"; tail -20 gpurun_out/bench_d500_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_d500_$TAG.json
