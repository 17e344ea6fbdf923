export TMPDIR=/tmp
o=gpurun_out/chain_trace_$1.txt; : > $o
for sh in 8192x16384 32768x32768; do
  MISOR_CHAIN_EDGE_COST=1.5 timeout -k 10 120 python tools/chain_trace.py --shape $sh --per-solve 7 >> $o 2>&1 || exit 1
done
