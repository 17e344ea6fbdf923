#!/bin/bash
# round 5 start: FP64 issue microbenchmark + the driver's bench setting
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/fp64_issue.bin > gpurun_out/r5_fp64_issue.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench_start.json 2> gpurun_out/r5_bench_start.err
