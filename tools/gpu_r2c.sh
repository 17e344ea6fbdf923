# aligned fused FG+RHS: NS tests, A/B, NS trace; 3D 128^3 trace
set -e
export TMPDIR=/tmp
o=gpurun_out/r2c; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_ns_gpu.py -x -v -m gpu --timeout 170 --timeout-method thread > $o/tests.log 2>&1
for f in 0 1 0 1; do MISOR_NS_FUSE=$f timeout -k 10 300 python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline >> $o/ns_ab_fuse$f.json 2>>$o/ns_ab.err; done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o -o ns_trace --output-format csv -- python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline > $o/ns_trace.log 2>&1
timeout -k 10 300 python bench.py --workload ns3d --size 128 --steps 20 --warmup 3 --no-cpu-baseline > $o/ns3d128.json 2>$o/ns3d128.err
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o -o ns3d_trace --output-format csv -- python bench.py --workload ns3d --size 128 --steps 20 --warmup 3 --no-cpu-baseline > $o/ns3d_trace.log 2>&1
