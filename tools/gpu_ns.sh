# NS step kernels: tests, bench, per-kernel traffic (bash tools/gpu_ns.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_ns_gpu.py tests/test_host_programs_gpu.py > gpurun_out/ns_tests_$tag.log 2>&1
o=gpurun_out/prof_ns_$tag; mkdir -p $o
timeout -k 10 200 python bench.py --workload ns --no-cpu-baseline > $o/bench.json 2>$o/bench.err
B="python bench.py --workload ns --no-cpu-baseline --steps 4 --warmup 2"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- $B > $o/trace.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $o -o fetch --output-format csv -- $B > $o/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $o -o write --output-format csv -- $B > $o/write.log 2>&1
