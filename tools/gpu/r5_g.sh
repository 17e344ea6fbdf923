#!/bin/bash
# part-2 slot sizing (MISOR_HR_PLAN=2) against the default plan on the decomposed
# rank proxy (MISOR_PROXY_SIDES), interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r5g_reserve.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5 --shapes 8192x16384:8"
for r in 1 2; do
for sd in LB B; do
for v in 0 2; do
echo "== plan $v sides $sd" | tee -a $o
MISOR_HR_PLAN=$v timeout -k 10 200 $P --sides $sd > gpurun_out/r5g_tmp.txt 2>&1 || { tail gpurun_out/r5g_tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5g_tmp.txt | tee -a $o
done
done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5g_bench.json 2> gpurun_out/r5g_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5g_bench.json')); print('N=1 bench', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $o
