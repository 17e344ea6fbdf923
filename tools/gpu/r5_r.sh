#!/bin/bash
# T = 8 (variant 0) against T = 10 (split ring) on the 2- and 4-GPU rank blocks
# through the decomposed loop (proxy with the rank's physical sides)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5r
o=gpurun_out/r5r/t.txt
: > $o
for rep in 1 2; do
for c in "--tsteps 8 --variants 0" "--tsteps 10 --variants 13"; do
for sh in "16384x16384:4 --sides LB" "16384x32768:2 --sides LBT"; do
timeout -k 10 300 python tools/scale_proxy.py --sweeps 20 --rows 0 --rounds 4 --shapes $sh $c > gpurun_out/r5r/tmp.txt 2>&1 || { tail gpurun_out/r5r/tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5r/tmp.txt | sed "s/^/$c: /" | tee -a $o
done
done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5r/bench.json 2> gpurun_out/r5r/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5r/bench.json')); print('N=1 bench', d['ms_per_step'])" | tee -a $o
for pre in 1 0 1 0; do
MISOR_FG_PREFETCH=$pre timeout -k 10 300 python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/r5r/ns.json 2> gpurun_out/r5r/ns.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5r/ns.json')); print('NS prefetch $pre', d['ms_per_step'], d['solve_kernel_ms_per_step'], d['other_ms_per_step'])" | tee -a $o
done
