#!/bin/bash
# parity of the self-resetting queue, the one-launch loop test and plan 2, then
# the bench, NS line, decomposed-rank proxy and A/B of the loop-test launches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_sor_gpu.py tests/test_tb_variants_gpu.py tests/test_decomposed_gpu.py tests/test_fullfield_gpu.py tests/test_near_threshold_gpu.py tests/test_chain_gpu.py -x -q --durations=5 --timeout 300 --timeout-method thread > gpurun_out/r5h_tests.log 2>&1 || { tail -30 gpurun_out/r5h_tests.log; exit 1; }
tail -2 gpurun_out/r5h_tests.log
o=gpurun_out/r5h.txt
: > $o
for m in 1 0 1 0; do
MISOR_FINISH_MERGE=$m timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5h_bench_m$m.json 2> gpurun_out/r5h_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5h_bench_m$m.json')); print('N=1 bench merge=$m', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $o
done
for m in 1 0; do
MISOR_FINISH_MERGE=$m timeout -k 10 300 python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/r5h_ns_m$m.json 2> gpurun_out/r5h_ns.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5h_ns_m$m.json')); print('NS merge=$m', d['ms_per_step'], d['solve_kernel_ms_per_step'], d['other_ms_per_step'])" | tee -a $o
done
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5 --shapes 8192x16384:8"
for sd in LB B; do
timeout -k 10 200 $P --sides $sd > gpurun_out/r5h_tmp.txt 2>&1 || { tail gpurun_out/r5h_tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5h_tmp.txt | sed "s/^/sides $sd: /" | tee -a $o
done
timeout -k 10 200 $P > gpurun_out/r5h_tmp.txt 2>&1 || exit 1
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5h_tmp.txt | sed "s/^/compute-only: /" | tee -a $o
