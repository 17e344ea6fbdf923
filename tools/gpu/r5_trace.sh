#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/chain_trace.py --shape 32768x32768 --T 10 --variant 13 --passes 2 > gpurun_out/r5_trace_32768_t10.txt 2>&1 || { tail gpurun_out/r5_trace_32768_t10.txt; exit 1; }
timeout -k 10 200 python tools/chain_trace.py --shape 8192x16384 --T 10 --variant 13 > gpurun_out/r5_trace_8192_t10.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_trace.py --shape 8192x16384 --T 8 > gpurun_out/r5_trace_8192_t8.txt 2>&1 || exit 1
cat gpurun_out/r5_trace_*.txt
