#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tb_variants_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_hrc_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r5_hrc_tests.log; exit 1; }
tail -2 gpurun_out/r5_hrc_tests.log
timeout -k 10 400 python tools/hr_chain_sweep.py --shape 32768x32768 --rings 4,8 --edge 1.5,2,3 > gpurun_out/r5_hrsweep2_32768.txt 2>&1 || { tail gpurun_out/r5_hrsweep2_32768.txt; exit 1; }
cat gpurun_out/r5_hrsweep2_32768.txt
timeout -k 10 400 python tools/hr_chain_sweep.py --shape 8192x16384 --rings 2,4,8 --edge 1.5,2,3 > gpurun_out/r5_hrsweep2_8192.txt 2>&1 || exit 1
cat gpurun_out/r5_hrsweep2_8192.txt
timeout -k 10 200 python tools/chain_trace.py --shape 32768x32768 --T 10 --variant 13 --passes 2 > gpurun_out/r5_trace2_32768_t10.txt 2>&1 || exit 1
head -12 gpurun_out/r5_trace2_32768_t10.txt
