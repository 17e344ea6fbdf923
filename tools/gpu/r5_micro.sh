#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 tools/micro/fp64_issue.bin > gpurun_out/r5_fp64_issue2.txt 2>&1
