#!/bin/bash
# the whole -m gpu suite on the wave-uniform ghost copies, then an A/B of them
# (lib_x: -DMISOR_GHOST_ALL, both shifts in every edge-mode wave) on the
# 8-GPU rank block (proxy, sides L+B and compute-only) and the 32768^2 grid
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --durations=30 --timeout 250 --timeout-method thread \
    > gpurun_out/r5s/tests.log 2>&1 || { tail -40 gpurun_out/r5s/tests.log; exit 1; }
tail -1 gpurun_out/r5s/tests.log
o=gpurun_out/r5s/ab.txt
: > $o
X=practical-parallel-algorithms-with-mpi_amd/lib_x/libmisor.so
P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 4"
for rep in 1 2; do
for lib in main $X; do
  L=""; [ $lib != main ] && L="--lib $lib"
  for sh in "8192x16384:8 --sides LB" "8192x16384:8" "32768x32768:1"; do
    timeout -k 10 200 $P $L --shapes $sh > gpurun_out/r5s/tmp.txt 2>&1 || { tail gpurun_out/r5s/tmp.txt; exit 1; }
    grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " gpurun_out/r5s/tmp.txt | sed "s|^|${lib##*/lib_} $sh: |" | tee -a $o
  done
done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5s/bench.json 2> gpurun_out/r5s/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5s/bench.json')); print('N=1 bench', d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $o
