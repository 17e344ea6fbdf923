#!/bin/bash
# the driver's bench setting: bench line, kernel trace and the PMC passes of the
# same command, then the 8-GPU rank block (8192 x 16384) compute-only and in the
# pipelined loop (bash tools/gpu/r5_prof.sh <tag>)
set -o pipefail
export TMPDIR=/tmp
tag=$1
out=gpurun_out/prof_$tag
mkdir -p $out
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 $B > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $out -o trace --output-format csv -- $B > $out/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out -o fetch --output-format csv -- $B > $out/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out -o write --output-format csv -- $B > $out/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $out -o sq --output-format csv -- $B > $out/sq.log 2>&1 || exit 1
for m in "" "--comm"; do
timeout -k 10 300 python tools/scale_proxy.py --shapes 8192x16384:8 --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5 $m > $out/proxy8$m.txt 2>&1 || { tail $out/proxy8$m.txt; exit 1; }
grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib" $out/proxy8$m.txt
done
timeout -k 10 200 $B > $out/bench2.json 2> $out/bench2.err || exit 1
python3 -c "import json; d=json.load(open('$out/bench2.json')); print('bench2', d['ms_per_step'], d['roofline']['kernel_ms'])"
