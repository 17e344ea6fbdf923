#!/bin/bash
# the whole -m gpu suite on the decomposed blocks' new chain geometry (180-row
# blocks, edge cost 3), then the rank proxies: new defaults against the old
# (MISOR_TB_CHAIN_RINGS=8 MISOR_CHAIN_EDGE_COST=2.5), alternated
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5y
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --durations=30 --timeout 250 --timeout-method thread \
    > gpurun_out/r5y/tests.log 2>&1 || { tail -40 gpurun_out/r5y/tests.log; exit 1; }
tail -1 gpurun_out/r5y/tests.log
o=gpurun_out/r5y/ab.txt
: > $o
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4"
for rep in 1 2; do
for cfg in new old; do
  for sh in "8192x16384:8 --sides LB" "8192x16384:8 --sides B" "16384x16384:4 --sides LB" "16384x32768:2 --sides LBT"; do
    if [ $cfg = old ]; then
      MISOR_TB_CHAIN_RINGS=8 MISOR_CHAIN_EDGE_COST=2.5 timeout -k 10 200 $P --shapes $sh > gpurun_out/r5y/tmp.txt 2>&1 || { tail gpurun_out/r5y/tmp.txt; exit 1; }
    else
      timeout -k 10 200 $P --shapes $sh > gpurun_out/r5y/tmp.txt 2>&1 || { tail gpurun_out/r5y/tmp.txt; exit 1; }
    fi
    grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5y/tmp.txt | sed "s/^/$cfg $sh: /" | tee -a $o
  done
done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5y/bench.json 2> gpurun_out/r5y/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5y/bench.json')); print('N=1 bench', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $o
