export TMPDIR=/tmp
o=gpurun_out/chain_trace_$1.txt; : > $o
timeout -k 10 120 python tools/chain_trace.py --shape 32768x32768 --T 7 --per-solve 7 >> $o 2>&1 || exit 1
HSA_SCRATCH_SINGLE_LIMIT=1 timeout -k 10 120 python tools/chain_trace.py --shape 32768x32768 --per-solve 7 >> $o 2>&1 || exit 1
