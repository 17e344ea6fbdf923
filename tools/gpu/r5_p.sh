#!/bin/bash
# host API + kernel timeline of the decomposed rank's loop (proxy, sides LB), and
# the proxy with the plans kept between solves
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
MISOR_PROXY_SIDES=LB timeout -s KILL 240 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/r5p -o trace --output-format csv -- python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 3 --shapes 8192x16384:8 --comm > gpurun_out/r5p/run.log 2>&1 || exit 1
o=gpurun_out/r5p/proxy.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 6 --shapes 8192x16384:8"
for sd in LB B; do
timeout -k 10 200 $P --sides $sd > gpurun_out/r5p/tmp.txt 2>&1 || { tail gpurun_out/r5p/tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5p/tmp.txt | sed "s/^/sides $sd: /" | tee -a $o
done
timeout -k 10 200 $P > gpurun_out/r5p/tmp.txt 2>&1 || exit 1
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5p/tmp.txt | sed "s/^/compute-only: /" | tee -a $o
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5p/bench.json 2> gpurun_out/r5p/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5p/bench.json')); print('N=1 bench', d['ms_per_step'])" | tee -a $o
