#!/bin/bash
# chained split ring: parity (variants test file), the driver's bench chained vs
# unchained, traces, and the 8-rank block (compute-only and the pipelined loop) at T = 8 / 10
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tb_variants_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5_hrc_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r5_hrc_tests.log; exit 1; }
tail -2 gpurun_out/r5_hrc_tests.log
for k in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_hrc_bench_chain$k.json 2> gpurun_out/r5_hrc_bench_chain$k.err || exit 1
MISOR_HR_CHAIN=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_hrc_bench_nochain$k.json 2> gpurun_out/r5_hrc_bench_nochain$k.err || exit 1
done
for f in gpurun_out/r5_hrc_bench_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline']['kernel_ms'])"; done
timeout -k 10 200 python tools/chain_trace.py --shape 32768x32768 --T 10 --variant 13 --passes 2 > gpurun_out/r5_trace_32768_t10.txt 2>&1 || exit 1
timeout -k 10 200 python tools/chain_trace.py --shape 8192x16384 --T 10 --variant 13 > gpurun_out/r5_trace_8192_t10.txt 2>&1 || exit 1
head -12 gpurun_out/r5_trace_32768_t10.txt gpurun_out/r5_trace_8192_t10.txt
for c in "--tsteps 8 --variants 0" "--tsteps 10 --variants 13"; do
for m in "" "--comm"; do
timeout -k 10 300 python tools/scale_proxy.py --shapes 8192x16384:8 --sweeps 20 --rows 0 $c --rounds 3 $m 2>&1 | grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib" | tee -a gpurun_out/r5_proxy8.txt || exit 1
done
done
