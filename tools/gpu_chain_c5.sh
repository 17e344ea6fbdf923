export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_chain_gpu.py > gpurun_out/chain_tests_$tag.log 2>&1 || exit 1
o=gpurun_out/chain_trace_$tag.txt; : > $o
for sh in 8192x16384 32768x32768; do
  timeout -k 10 120 python tools/chain_trace.py --shape $sh >> $o 2>&1 || exit 1
done
o=gpurun_out/chain_proxy_$tag.txt; : > $o
for E in 1.0 1.3 1.6; do
  echo "edge cost $E" >> $o
  MISOR_CHAIN_EDGE_COST=$E timeout -k 10 200 python tools/scale_proxy.py --shapes 32768x32768:1,8192x16384:8 --tsteps 8 --rows 72 --rounds 2 --sweeps 56 >> $o 2>&1 || exit 1
done
