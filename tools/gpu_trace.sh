export TMPDIR=/tmp
o=gpurun_out/chain_trace_$1.txt; : > $o
for sh in 8192x16384 32768x32768; do for r in 72 144; do
  timeout -k 10 120 python tools/chain_trace.py --shape $sh --rows $r >> $o 2>&1 || exit 1
done; done
