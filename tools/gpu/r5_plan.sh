#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/plan_ab.py --shapes 32768x32768,16384x32768,16384x16384,8192x16384,4096x4096 --iters 20,100 > gpurun_out/r5_plan_ab.txt 2>&1 || { tail gpurun_out/r5_plan_ab.txt; exit 1; }
cat gpurun_out/r5_plan_ab.txt
timeout -k 10 300 python tools/plan_ab.py --shapes 16384x32768,16384x16384,8192x16384 --iters 20,100 --comm > gpurun_out/r5_plan_ab_comm.txt 2>&1 || { tail gpurun_out/r5_plan_ab_comm.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib" gpurun_out/r5_plan_ab_comm.txt
