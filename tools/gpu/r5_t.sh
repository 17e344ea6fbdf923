#!/bin/bash
# NS config 5 with nontemporal stores in fg_rhs / adapt_absmax (MISOR_NS_NT=1)
# against the plain stores, alternated; the NS tests on the NT build; kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
o=gpurun_out/r5t/ab.txt
: > $o
for nt in 1 0 1 0 1 0; do
MISOR_NS_NT=$nt timeout -k 10 300 python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/r5t/ns.json 2> gpurun_out/r5t/ns.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5t/ns.json')); print('NS nt $nt', d['ms_per_step'], d['solve_kernel_ms_per_step'], d['other_ms_per_step'])" | tee -a $o
done
MISOR_NS_NT=1 timeout -k 10 600 python -u -m pytest tests/test_ns_gpu.py tests/test_bench_configs_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r5t/tests.log 2>&1 || { tail -30 gpurun_out/r5t/tests.log; exit 1; }
tail -1 gpurun_out/r5t/tests.log | tee -a $o
for nt in 0 1; do
MISOR_NS_NT=$nt timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5t/prof$nt -o trace --output-format csv -- python bench.py --workload ns --steps 10 --warmup 2 > gpurun_out/r5t/prof$nt.log 2>&1 || exit 1
done
