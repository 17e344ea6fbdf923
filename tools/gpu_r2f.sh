# 3D preload/fold overlap + adapt compact tiles
set -e
export TMPDIR=/tmp
o=gpurun_out/r2f; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_ns3d_gpu.py tests/test_ns_gpu.py tests/test_ns3d_decomposed_gpu.py -x -v -m gpu --timeout 170 --timeout-method thread > $o/tests.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o -o ns3d_trace --output-format csv -- python bench.py --workload ns3d --size 128 --steps 20 --warmup 3 --no-cpu-baseline > $o/ns3d_trace.log 2>&1
timeout -k 10 300 python tools/tune3d.py --size 128 384 --iters 400 --configs 1,8,0 0,8,0 > $o/tune3d.txt 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o -o ns_trace --output-format csv -- python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline > $o/ns_trace.log 2>&1
