export TMPDIR=/tmp
o=gpurun_out/chain_trace_$1.txt; : > $o
for x in 0 1 2 3; do
  echo "xmode $x" >> $o
  MISOR_CHAIN_XMODE=$x timeout -k 10 120 python tools/chain_trace.py --shape 32768x32768 --per-solve 7 >> $o 2>&1 || exit 1
done
