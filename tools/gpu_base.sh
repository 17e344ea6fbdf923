set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r03base.log 2>&1
bash tools/profile_bench.sh r03base
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_r03base.json 2>gpurun_out/bench20_r03base.err
o=gpurun_out/prof_ns_r03base; mkdir -p $o
timeout -k 10 200 python bench.py --workload ns --no-cpu-baseline > $o/bench.json 2>$o/bench.err
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- python bench.py --workload ns --no-cpu-baseline --steps 4 --warmup 2 > $o/trace.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $o -o fetch --output-format csv -- python bench.py --workload ns --no-cpu-baseline --steps 4 --warmup 2 > $o/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $o -o write --output-format csv -- python bench.py --workload ns --no-cpu-baseline --steps 4 --warmup 2 > $o/write.log 2>&1
timeout -k 10 300 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 2 --sweeps 56 > gpurun_out/scale_proxy_r03base.txt 2>&1
