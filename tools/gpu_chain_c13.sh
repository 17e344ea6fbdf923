export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_chain_gpu.py tests/test_bench_local_gpu.py tests/test_decomposed_gpu.py > gpurun_out/chain_tests_$tag.log 2>&1 || exit 1
o=gpurun_out/chain_proxy_$tag.txt; : > $o
timeout -k 10 300 python tools/scale_proxy.py --tsteps 8 --rows 72,108,144 --rounds 3 --sweeps 56 >> $o 2>&1 || exit 1
timeout -k 10 200 python tools/scale_proxy.py --tsteps 8 --rows 0 --rounds 3 --sweeps 56 --chain 0 >> $o 2>&1 || exit 1
o=gpurun_out/chain_trace_$tag.txt; : > $o
for sh in 8192x16384 32768x32768; do
  timeout -k 10 120 python tools/chain_trace.py --shape $sh --per-solve 7 >> $o 2>&1 || exit 1
done
