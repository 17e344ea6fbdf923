#!/bin/bash
# suite + pass plans on the rank-block shapes + chain traces
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/r5_suite.sh r5d || exit 1
timeout -k 10 400 python tools/plan_ab.py --shapes 8192x16384,16384x8192,16384x16384,16384x32768,32768x16384 --iters 20,100 --rounds 3 > gpurun_out/r5d_plan_ab.txt 2>&1 || { tail gpurun_out/r5d_plan_ab.txt; exit 1; }
cat gpurun_out/r5d_plan_ab.txt
timeout -k 10 200 python tools/chain_trace.py --shape 8192x16384 --T 10 --variant 13 > gpurun_out/r5d_trace_8192x16384_t10.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_trace.py --shape 16384x8192 --T 10 --variant 13 > gpurun_out/r5d_trace_16384x8192_t10.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_trace.py --shape 32768x32768 --T 10 --variant 13 --passes 2 > gpurun_out/r5d_trace_32768_t10.txt 2>&1 || exit 1
head -30 gpurun_out/r5d_trace_*.txt
