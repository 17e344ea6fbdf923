#!/bin/bash
# end of round: smoke, the driver's bench line and the rank proxies on the final tree
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5end
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5end/smoke.log 2>&1 || { tail -20 gpurun_out/r5end/smoke.log; exit 1; }
tail -1 gpurun_out/r5end/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5end/bench.json 2> gpurun_out/r5end/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5end/bench.json')); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['bound'])"
o=gpurun_out/r5end/proxy.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5"
for sh in "8192x16384:8 --sides LB" "8192x16384:8 --sides B" "8192x16384:8" "16384x16384:4 --sides LB" "16384x32768:2 --sides LBT"; do
  timeout -k 10 200 $P --shapes $sh > gpurun_out/r5end/tmp.txt 2>&1 || { tail gpurun_out/r5end/tmp.txt; exit 1; }
  grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5end/tmp.txt | sed "s/^/$sh: /" | tee -a $o
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5end/bench2.json 2> gpurun_out/r5end/bench2.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5end/bench2.json')); print('N=1 bench (same box)', d['ms_per_step'])" | tee -a $o
