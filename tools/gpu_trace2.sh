export TMPDIR=/tmp
o=gpurun_out/chain_trace_$1.txt; : > $o
for ps in 1 7; do
  timeout -k 10 120 python tools/chain_trace.py --shape 32768x32768 --per-solve $ps >> $o 2>&1 || exit 1
done
timeout -k 10 120 python tools/chain_trace.py --shape 8192x16384 --per-solve 7 >> $o 2>&1 || exit 1
