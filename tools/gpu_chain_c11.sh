export TMPDIR=/tmp
tag=$1
o=gpurun_out/chain_proxy_$tag.txt; : > $o
for E in 1.6 2.0 2.5; do
  echo "edge cost $E" >> $o
  MISOR_CHAIN_EDGE_COST=$E timeout -k 10 200 python tools/scale_proxy.py --tsteps 8 --rows 0 --rounds 3 --sweeps 56 >> $o 2>&1 || exit 1
done
echo "unchained" >> $o
timeout -k 10 200 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 3 --sweeps 56 --chain 0 >> $o 2>&1 || exit 1
o=gpurun_out/chain_trace_$tag.txt; : > $o
for sh in 8192x16384 32768x32768; do
  timeout -k 10 120 python tools/chain_trace.py --shape $sh --per-solve 7 >> $o 2>&1 || exit 1
done
