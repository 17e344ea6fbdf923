# SQ issue/stall counters of the sweep kernel (one rocprofv3 --pmc pass each).
#   bash tools/pmc_sq.sh <tag> [bench args...]
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_$tag -o sq --output-format csv -- python bench.py --steps 8 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmc_$tag/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$tag -o fetch --output-format csv -- python bench.py --steps 8 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmc_$tag/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$tag -o write --output-format csv -- python bench.py --steps 8 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmc_$tag/write.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_$tag -o trace --output-format csv -- python bench.py --steps 8 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmc_$tag/trace.log 2>&1
