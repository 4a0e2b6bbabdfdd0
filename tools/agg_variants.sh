#!/bin/bash
set -u
mkdir -p gpurun_out
for V in 1,0 1,1 2,0 2,1 4,0 4,1; do
  echo "variant $V"
  FLSIM_AGG_VARIANT=$V timeout -k 10 120 python -u tools/agg_bench.py || exit 1
done 2>&1 | tee gpurun_out/aggvar.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "aggregate" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
FLSIM_AGG_VARIANT=2,1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "aggregate" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
FLSIM_AGG_VARIANT=4,0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "aggregate" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
