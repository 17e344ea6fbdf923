#!/bin/bash
# strong-scaling proxy of the 8-GPU rank block: compute-only, one-rank pipelined
# loop, and the decomposed rank's loop (MISOR_PROXY_SIDES) for the 4 x 2 and
# 2 x 4 splits, beside the same box's N = 1 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r5e_proxy.txt
: > $o
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5e_bench.json 2> gpurun_out/r5e_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5e_bench.json')); print('N=1 bench', d['ms_per_step'])" | tee -a $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5"
for c in "--shapes 8192x16384:8" "--shapes 8192x16384:8 --comm" "--shapes 8192x16384:8 --sides LB" "--shapes 8192x16384:8 --sides B" "--shapes 16384x8192:8 --sides LB" "--shapes 16384x8192:8 --sides L"; do
echo "== $c" | tee -a $o
timeout -k 10 200 $P $c > gpurun_out/r5e_tmp.txt 2>&1 || { tail gpurun_out/r5e_tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib" gpurun_out/r5e_tmp.txt | tee -a $o
done
