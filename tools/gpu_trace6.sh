# chained 32768^2 pass timelines at three edge-column costs (bash tools/gpu_trace6.sh <tag>)
export TMPDIR=/tmp
o=gpurun_out/chain_trace_$1.txt; : > $o
for e in 2.0 3.0; do
  echo "edge cost $e" >> $o
  MISOR_CHAIN_EDGE_COST=$e timeout -k 10 120 python tools/chain_trace.py --shape 32768x32768 --per-solve 7 >> $o 2>&1 || exit 1
done
