# Round-end evidence on one MI355X (bash tools/gpu_final.sh <tag>):
# smoke, the -m gpu suite, the default and the driver-length benches with
# their kernel traces and PMC passes (per pass length), NS per-kernel
# traffic, the strong-scaling proxy.  Every GPU step has its own time limit.
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 170 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1
for st in 140 20; do
  o=gpurun_out/prof_${tag}_s$st; mkdir -p $o
  timeout -k 10 300 python bench.py --steps $st > $o/bench.json 2> $o/bench.err
  B="python bench.py --steps $st --warmup 5 --no-cpu-baseline"
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- $B > $o/trace.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o -o fetch --output-format csv -- $B > $o/fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o -o write --output-format csv -- $B > $o/write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $o -o sq --output-format csv -- $B > $o/sq.log 2>&1
done
o=gpurun_out/prof_ns_$tag; mkdir -p $o
timeout -k 10 200 python bench.py --workload ns --no-cpu-baseline > $o/bench.json 2>$o/bench.err
B="python bench.py --workload ns --no-cpu-baseline --steps 4 --warmup 2"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- $B > $o/trace.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $o -o fetch --output-format csv -- $B > $o/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $o -o write --output-format csv -- $B > $o/write.log 2>&1
timeout -k 10 300 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 2 --sweeps 56 --chain=-1,0 \
    > gpurun_out/scale_proxy_$tag.txt 2>&1
timeout -k 10 200 python bench.py --local-ranks 8 --size 8192 --steps 20 --warmup 3 --check \
    > gpurun_out/bench_local8_$tag.json 2> gpurun_out/bench_local8_$tag.err
