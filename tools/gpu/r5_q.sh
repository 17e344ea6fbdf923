#!/bin/bash
# part 2 on the comm stream: parity, the proxy A/B and a timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5q
timeout -k 10 600 python -u -m pytest tests/test_decomposed_gpu.py tests/test_fullfield_gpu.py tests/test_near_threshold_gpu.py tests/test_ns_gpu.py tests/test_bench_local_gpu.py tests/test_host_programs_gpu.py -x -q --durations=5 --timeout 300 --timeout-method thread > gpurun_out/r5q/tests.log 2>&1 || { tail -30 gpurun_out/r5q/tests.log; exit 1; }
tail -3 gpurun_out/r5q/tests.log
o=gpurun_out/r5q/proxy.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 6 --shapes 8192x16384:8"
for rep in 1 2; do
for m in 1 0; do
for sd in LB B; do
MISOR_P2_CSTREAM=$m timeout -k 10 200 $P --sides $sd > gpurun_out/r5q/tmp.txt 2>&1 || { tail gpurun_out/r5q/tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5q/tmp.txt | sed "s/^/p2c $m sides $sd: /" | tee -a $o
done
done
done
MISOR_PROXY_SIDES=LB timeout -s KILL 240 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/r5q -o trace --output-format csv -- python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 3 --shapes 8192x16384:8 --comm > gpurun_out/r5q/run.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5q/bench.json 2> gpurun_out/r5q/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5q/bench.json')); print('N=1 bench', d['ms_per_step'])" | tee -a $o
