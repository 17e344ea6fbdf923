export TMPDIR=/tmp
tag=$1
o=gpurun_out/chain_proxy_$tag.txt; : > $o
timeout -k 10 300 python tools/scale_proxy.py --tsteps 8 --rows 72,108,144,216 --rounds 3 --sweeps 56 >> $o 2>&1 || exit 1
o=gpurun_out/chain_trace_$tag.txt; : > $o
for r in 144 216; do
  timeout -k 10 120 python tools/chain_trace.py --shape 32768x32768 --per-solve 7 --rows $r >> $o 2>&1 || exit 1
done
