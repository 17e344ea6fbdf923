#!/bin/bash
# edge-column cost in the chained plan (MISOR_CHAIN_EDGE_COST) and block height
# (MISOR_TB_CHAIN_RINGS) on the 8-GPU rank block, through the pipelined loop
# (sides L+B) and compute-only, alternated
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5w
o=gpurun_out/r5w/ab.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4 --shapes 8192x16384:8"
for rep in 1 2; do
for cfg in "E=2.5 R=8" "E=1.8 R=8" "E=2.1 R=8" "E=2.5 R=10" "E=2.5 R=6"; do
  ec=${cfg#E=}; ec=${ec% R=*}; rr=${cfg#*R=}
  for sd in "--sides LB" ""; do
    MISOR_CHAIN_EDGE_COST=$ec MISOR_TB_CHAIN_RINGS=$rr timeout -k 10 200 $P $sd > gpurun_out/r5w/tmp.txt 2>&1 || { tail gpurun_out/r5w/tmp.txt; exit 1; }
    grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5w/tmp.txt | sed "s/^/$cfg ${sd:-compute}: /" | tee -a $o
  done
done
done
