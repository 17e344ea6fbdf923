export TMPDIR=/tmp
o=gpurun_out/chain_c4.txt; : > $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_chain_gpu.py > gpurun_out/chain_tests_c4.log 2>&1
for E in 1.0 1.5 2.0 3.0; do
  echo "edge cost $E" >> $o
  MISOR_CHAIN_EDGE_COST=$E timeout -k 10 200 python tools/scale_proxy.py --shapes 32768x32768:1,8192x16384:8 --tsteps 8 --rows 72,144 --rounds 2 --sweeps 56 >> $o 2>&1
done
