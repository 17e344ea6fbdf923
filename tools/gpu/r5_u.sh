#!/bin/bash
# the part-2 stream forms test and the decomposed suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5u
timeout -k 10 600 python -u -m pytest tests/test_decomposed_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r5u/tests.log 2>&1 || { tail -30 gpurun_out/r5u/tests.log; exit 1; }
tail -1 gpurun_out/r5u/tests.log
