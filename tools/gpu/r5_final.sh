#!/bin/bash
# round-5 final evidence: smoke, the whole -m gpu suite, the driver's bench line,
# its kernel trace and PMC passes, the NS / 3D lines and the decomposed-rank proxy
set -o pipefail
export TMPDIR=/tmp
tag=${1:-final}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --durations=30 --timeout 250 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_$tag.json')); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['bound'])"
out=gpurun_out/prof_$tag
mkdir -p $out
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $out -o trace --output-format csv -- $B > $out/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out -o fetch --output-format csv -- $B > $out/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out -o write --output-format csv -- $B > $out/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $out -o sq --output-format csv -- $B > $out/sq.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/ns_$tag.json 2> gpurun_out/ns_$tag.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/ns_$tag.json')); print('NS', d['ms_per_step'], d['solve_kernel_ms_per_step'], d['other_ms_per_step'])"
timeout -k 10 300 python bench.py --workload ns3d --steps 5 --warmup 2 > gpurun_out/ns3d_$tag.json 2> gpurun_out/ns3d_$tag.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/ns3d_$tag.json')); print('NS3D', d['ms_per_step'], d['roofline'].get('solve_ms_per_iteration'))"
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5 --shapes 8192x16384:8"
o=gpurun_out/proxy_$tag.txt
: > $o
for sd in LB B; do
timeout -k 10 200 $P --sides $sd > gpurun_out/proxy_tmp.txt 2>&1 || { tail gpurun_out/proxy_tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/proxy_tmp.txt | sed "s/^/sides $sd: /" | tee -a $o
done
Q="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5"
for sh in "16384x16384:4 --sides LB" "16384x32768:2 --sides LBT"; do
timeout -k 10 200 $Q --shapes $sh > gpurun_out/proxy_tmp.txt 2>&1 || { tail gpurun_out/proxy_tmp.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/proxy_tmp.txt | sed "s/^/$sh: /" | tee -a $o
done
timeout -k 10 200 $P > gpurun_out/proxy_tmp.txt 2>&1 || exit 1
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/proxy_tmp.txt | sed "s/^/compute-only: /" | tee -a $o
timeout -k 10 200 $B > gpurun_out/bench2_$tag.json 2> gpurun_out/bench2_$tag.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench2_$tag.json')); print('N=1 bench (same box)', d['ms_per_step'])" | tee -a $o
