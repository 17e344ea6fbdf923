# the 3D tests with the resident solve as the default, then the 3D benches and a
# kernel trace at 128^3 (bash tools/gpu_res3d_final.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ns3d_gpu.py tests/test_ns3d_decomposed_gpu.py tests/test_ns3d_host_gpu.py \
    -x -q --timeout 150 --timeout-method thread > gpurun_out/res3d_alltests_$tag.log 2>&1
timeout -k 10 200 python bench.py --workload ns3d > gpurun_out/res3d_bench128_$tag.json 2> gpurun_out/res3d_bench128_$tag.err
timeout -k 10 200 python tools/tune3d.py --size 128 --iters 400 --configs 1,8,0,1,0,0 1,8,0,1,0,1 1,8,0,1,0,0 1,8,0,1,0,1 > gpurun_out/res3d_ab_$tag.txt 2>&1
o=gpurun_out/res3d_prof_$tag; mkdir -p $o
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- python bench.py --workload ns3d --no-cpu-baseline --steps 6 --warmup 1 > $o/trace.log 2>&1
