# 3D resident solve (LDS receive lists): the 3D suite, then A/B timing against
# the previous build (lib_ab/libmisor_res1.so) and the streaming sweep (bash tools/gpu_r3d.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
T3="tests/test_ns3d_gpu.py tests/test_ns3d_decomposed_gpu.py tests/test_ns3d_host_gpu.py"
timeout -k 10 400 python -u -m pytest $T3 -x -q --timeout 150 --timeout-method thread > gpurun_out/r3d_tests_$tag.log 2>&1
o=gpurun_out/r3d_ab_$tag.txt; : > $o
for r in 1 2; do
  timeout -k 10 100 python tools/tune3d.py --size 128 --iters 400 --configs 1,8,0,1,0,1 >> $o 2>&1
  timeout -k 10 100 python tools/tune3d.py --size 128 --iters 400 --configs 1,8,0,1,0,0 >> $o 2>&1
done
timeout -k 10 200 python bench.py --workload ns3d > gpurun_out/r3d_bench128_$tag.json 2> gpurun_out/r3d_bench128_$tag.err
