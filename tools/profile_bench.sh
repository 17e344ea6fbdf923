# Bench + rocprofv3 evidence for the default configuration (run on the GPU box):
#   bash tools/profile_bench.sh <tag>
# -> gpurun_out/prof_<tag>/{bench.json, trace_kernel_stats.csv, fetch/write/sq counter CSVs}
set -e
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 300 python bench.py "$@" > $out/bench.json 2> $out/bench.err
B="python bench.py --steps 32 --warmup 8 --no-cpu-baseline $*"
# the kernel trace runs the bench's own default steps, so its average launch
# duration is comparable with roofline.kernel_ms of bench.json
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $out -o trace --output-format csv -- python bench.py --no-cpu-baseline "$@" > $out/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out -o fetch --output-format csv -- $B > $out/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out -o write --output-format csv -- $B > $out/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $out -o sq --output-format csv -- $B > $out/sq.log 2>&1
