# adapt unroll + reserve/T8 decomposed tests + decomposition shape proxy
set -e
export TMPDIR=/tmp
o=gpurun_out/r2d; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_ns_gpu.py tests/test_decomposed_gpu.py -x -v -m gpu --timeout 170 --timeout-method thread > $o/tests.log 2>&1
for f in 1 1; do timeout -k 10 300 python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline >> $o/ns.json 2>>$o/ns.err; done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o -o ns_trace --output-format csv -- python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline > $o/ns_trace.log 2>&1
timeout -k 10 600 python tools/scale_proxy.py --shapes 8192x16384:8,16384x8192:8,32768x4096:8,16384x16384:4,32768x8192:4,16384x32768:2,32768x16384:2 --tsteps 7,8 --rows 0 --rounds 3 --sweeps 56 > $o/proxy_shapes.txt 2>&1
