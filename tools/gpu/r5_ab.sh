#!/bin/bash
# A/B of an experiment build against the in-tree library at the headline pass
# (variant 13, T = 10, 32768^2) and the 8-GPU rank block (bash tools/gpu/r5_ab.sh <tag> <lib dir>)
set -o pipefail
export TMPDIR=/tmp
tag=$1; lib=$2
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_libs.py --size 32768 --passes 4 --rounds 3 main::13:10 x:practical-parallel-algorithms-with-mpi_amd/$lib/libmisor.so:13:10 > gpurun_out/ab_$tag.txt 2>&1 || { tail -20 gpurun_out/ab_$tag.txt; exit 1; }
cat gpurun_out/ab_$tag.txt
timeout -k 10 300 python tools/ab_libs.py --size 32768 --ni 8192 --nj 16384 --passes 4 --rounds 3 main::13:10 x:practical-parallel-algorithms-with-mpi_amd/$lib/libmisor.so:13:10 > gpurun_out/ab8_$tag.txt 2>&1 || { tail -20 gpurun_out/ab8_$tag.txt; exit 1; }
cat gpurun_out/ab8_$tag.txt
