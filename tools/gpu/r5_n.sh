#!/bin/bash
# hardware queues for the decomposed rank's streams: proxy (sides LB / B) at
# GPU_MAX_HW_QUEUES 4 (default) / 8, alternated, and a timeline at 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5n
o=gpurun_out/r5n/q.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4 --shapes 8192x16384:8"
for rep in 1 2; do
for q in 4 8 16; do
for sd in LB B; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 $P --sides $sd > gpurun_out/r5n/tmp.txt 2>&1 || { tail gpurun_out/r5n/tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5n/tmp.txt | sed "s/^/queues $q sides $sd: /" | tee -a $o
done
done
done
MISOR_PROXY_SIDES=LB GPU_MAX_HW_QUEUES=8 timeout -s KILL 240 rocprofv3 --kernel-trace -d gpurun_out/r5n -o trace8 --output-format csv -- python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 2 --shapes 8192x16384:8 --comm > gpurun_out/r5n/run8.log 2>&1 || exit 1
for q in 4 8; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5n/bench$q.json 2> gpurun_out/r5n/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5n/bench$q.json')); print('N=1 bench queues $q', d['ms_per_step'])" | tee -a $o
done
timeout -k 10 300 python -u -m pytest tests/test_lex_gpu.py -x -q --durations=3 --timeout 250 --timeout-method thread > gpurun_out/r5n/lex.log 2>&1 || { tail -20 gpurun_out/r5n/lex.log; exit 1; }
tail -5 gpurun_out/r5n/lex.log
