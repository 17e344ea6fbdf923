# NS fusion + pipelined-reserve session
set -e
export TMPDIR=/tmp
o=gpurun_out/r2b; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_ns_gpu.py tests/test_decomposed_gpu.py tests/test_host_programs_gpu.py -x -v -m gpu --timeout 170 --timeout-method thread > $o/tests.log 2>&1
for f in 0 1 0 1; do MISOR_NS_FUSE=$f timeout -k 10 300 python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline >> $o/ns_ab_fuse$f.json 2>>$o/ns_ab.err; done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $o -o ns_trace --output-format csv -- python bench.py --workload ns --size 16384 --itermax 100 --steps 10 --warmup 2 --no-cpu-baseline > $o/ns_trace.log 2>&1
timeout -k 10 300 python tools/scale_proxy.py --comm --ranks 8 --tsteps 7 --rows 0 --rounds 3 --sweeps 56 --reserve 0,8,16,32 > $o/proxy_comm_n8.txt 2>&1
timeout -k 10 300 python tools/scale_proxy.py --comm --ranks 1 --tsteps 8 --rows 0 --rounds 2 --sweeps 48 --reserve 0,16 > $o/proxy_comm_n1.txt 2>&1
