#!/bin/bash
# the one-list chain plan of the split ring against the two-list one
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/r5f_plan.txt
: > $o
timeout -k 10 400 python -u -m pytest tests/test_lex_gpu.py tests/test_tb_variants_gpu.py tests/test_fullfield_gpu.py tests/test_decomposed_gpu.py -x -q --durations=5 --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1 || { tail -30 gpurun_out/r5f_tests.log; exit 1; }
tail -2 gpurun_out/r5f_tests.log
for sh in "--ni 8192 --nj 16384" "--ni 16384 --nj 8192" "--ni 16384 --nj 16384" ""; do
echo "== $sh" | tee -a $o
timeout -k 10 300 python tools/ab_env.py --var MISOR_HR_PLAN --values 0,1 --size 32768 $sh --tsteps 10 --variant 13 --passes 2 --rounds 3 2>/dev/null | tee -a $o || exit 1
done
for v in 0 1; do
MISOR_HR_PLAN=$v timeout -k 10 200 python tools/chain_trace.py --shape 8192x16384 --T 10 --variant 13 > gpurun_out/r5f_trace_8192_plan$v.txt 2>&1 || exit 1
head -12 gpurun_out/r5f_trace_8192_plan$v.txt
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5f_bench.json')); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'])"
timeout -k 10 300 python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/r5f_ns.json 2> gpurun_out/r5f_ns.err || exit 1
cat gpurun_out/r5f_ns.json
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_nsprof -o trace --output-format csv -- python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/r5f_nsprof.log 2>&1 || exit 1
