#!/bin/bash
# debug: conv6's data gradient dz5 against fp64 (tools/dbg_split.py with the backward stopped)
set -u
mkdir -p gpurun_out/dbg
export TMPDIR=/tmp
FLSIM_DEBUG_BWD_STOP=6 FLSIM_CONCURRENT_BWD=0 timeout -k 10 200 python3 -u tools/dbg_split.py 1 0 > gpurun_out/dbg/stop6.txt 2>&1 || { echo "dbg failed $?"; tail -5 gpurun_out/dbg/stop6.txt; exit 1; }
cat gpurun_out/dbg/stop6.txt


FLSIM_CONCURRENT_BWD=0 timeout -k 10 200 python3 -u tools/dbg_split.py 2 1 > gpurun_out/dbg/full.txt 2>&1 || { echo "dbg failed $?"; tail -5 gpurun_out/dbg/full.txt; exit 1; }
cat gpurun_out/dbg/full.txt
