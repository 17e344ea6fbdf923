# the resident 3D solve: parity tests, then the 128^3 bench with and without it
# and a kernel trace (bash tools/gpu_res3d.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ns3d_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "solve or short_run or medium or tuning or resident" > gpurun_out/res3d_tests_$tag.log 2>&1
timeout -k 10 200 python bench.py --workload ns3d --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/res3d_bench_$tag.json 2> gpurun_out/res3d_bench_$tag.err
timeout -k 10 200 python tools/tune3d.py --size 128 --iters 200 --configs 1,8,0,1,0,0 1,8,0,1,0,1 1,8,0,1,0,0 1,8,0,1,0,1 > gpurun_out/res3d_tune_$tag.txt 2>&1
o=gpurun_out/res3d_prof_$tag; mkdir -p $o
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- python bench.py --workload ns3d --no-cpu-baseline --steps 4 --warmup 1 > $o/trace.log 2>&1
