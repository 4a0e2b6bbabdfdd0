#!/bin/bash
# round-4 first GPU call: the shipped tree's profile (tools/gpu_prof_r04.sh), then the split-form
# operand lab (tools/lab/xs_lab.hip) under its own limit
set -u
bash tools/gpu_prof_r04.sh r04a || exit 1
mkdir -p gpurun_out/lab_xs
timeout -k 10 300 tools/lab/xs_lab > gpurun_out/lab_xs/time.txt 2>&1 || { echo "lab failed $?"; tail -5 gpurun_out/lab_xs/time.txt; exit 1; }
cat gpurun_out/lab_xs/time.txt
