#!/bin/bash
# block height (ring lengths per chained block) and edge cost of the split
# ring's chain plan: the decomposed-rank proxy (sides LB / B) and N = 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r5i_rings.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4 --shapes 8192x16384:8"
for rep in 1 2; do
for rg in 8 4 6; do
for ec in 2.5 1.8; do
for sd in LB B; do
MISOR_TB_CHAIN_RINGS=$rg MISOR_CHAIN_EDGE_COST=$ec timeout -k 10 200 $P --sides $sd > gpurun_out/r5i_tmp.txt 2>&1 || { tail gpurun_out/r5i_tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5i_tmp.txt | sed "s/^/rings $rg edge $ec sides $sd: /" | tee -a $o
done
done
done
done
for rg in 8 4 8 4; do
MISOR_TB_CHAIN_RINGS=$rg timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5i_bench.json')); print('N=1 bench rings $rg', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $o
done
