#!/bin/bash
# decomposed blocks: 162 / 180 / 198-row chained blocks (MISOR_TB_CHAIN_RINGS
# 9 / 10 / 11) on the 8- and 4-GPU rank proxies, alternated
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5z
o=gpurun_out/r5z/ab.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4"
for rep in 1 2; do
for rr in 10 9 11; do
  for sh in "8192x16384:8 --sides LB" "8192x16384:8 --sides B" "16384x16384:4 --sides LB"; do
    MISOR_TB_CHAIN_RINGS=$rr timeout -k 10 200 $P --shapes $sh > gpurun_out/r5z/tmp.txt 2>&1 || { tail gpurun_out/r5z/tmp.txt; exit 1; }
    grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5z/tmp.txt | sed "s/^/R=$rr $sh: /" | tee -a $o
  done
done
done
