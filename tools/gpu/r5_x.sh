#!/bin/bash
# block height (MISOR_TB_CHAIN_RINGS) and edge-column cost on the 8-GPU rank
# block's pipelined loop: sides L+B (corner rank) and B (middle rank), alternated
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5x
o=gpurun_out/r5x/ab.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4 --shapes 8192x16384:8"
for rep in 1 2; do
for cfg in "E=2.5 R=8" "E=2.5 R=10" "E=2.5 R=12" "E=3.0 R=10" "E=3.5 R=10"; do
  ec=${cfg#E=}; ec=${ec% R=*}; rr=${cfg#*R=}
  for sd in LB B; do
    MISOR_CHAIN_EDGE_COST=$ec MISOR_TB_CHAIN_RINGS=$rr timeout -k 10 200 $P --sides $sd > gpurun_out/r5x/tmp.txt 2>&1 || { tail gpurun_out/r5x/tmp.txt; exit 1; }
    grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5x/tmp.txt | sed "s/^/$cfg $sd: /" | tee -a $o
  done
done
done
