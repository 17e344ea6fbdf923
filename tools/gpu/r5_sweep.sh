#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/hr_chain_sweep.py --shape 32768x32768 --rings 4,8,16 --edge 2,3.5,5 > gpurun_out/r5_hrsweep_32768.txt 2>&1 || { tail gpurun_out/r5_hrsweep_32768.txt; exit 1; }
cat gpurun_out/r5_hrsweep_32768.txt
timeout -k 10 400 python tools/hr_chain_sweep.py --shape 8192x16384 --rings 2,4,8 --edge 2,3.5,5 > gpurun_out/r5_hrsweep_8192.txt 2>&1 || exit 1
cat gpurun_out/r5_hrsweep_8192.txt
