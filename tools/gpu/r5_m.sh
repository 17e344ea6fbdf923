#!/bin/bash
# kernel timeline of the decomposed rank's pipelined loop (proxy, sides LB)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5m
MISOR_PROXY_SIDES=LB timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m -o trace --output-format csv -- python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 2 --shapes 8192x16384:8 --comm > gpurun_out/r5m/run.log 2>&1 || { tail gpurun_out/r5m/run.log; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib" gpurun_out/r5m/run.log | tail -3
timeout -k 10 300 python -u -m pytest tests/test_host_programs_gpu.py tests/test_ns_gpu.py -x -q --durations=5 --timeout 250 --timeout-method thread > gpurun_out/r5m_tests.log 2>&1 || { tail -30 gpurun_out/r5m_tests.log; exit 1; }
tail -8 gpurun_out/r5m_tests.log
