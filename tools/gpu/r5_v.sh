#!/bin/bash
# NS config 5 PMC (HBM bytes of fg_rhs / adapt_absmax with nontemporal stores):
# separate FETCH_SIZE and WRITE_SIZE passes, kernel trace only otherwise
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5v
mkdir -p $out
B="python bench.py --workload ns --steps 4 --warmup 1"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $out -o fetch --output-format csv -- $B > $out/fetch.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $out -o write --output-format csv -- $B > $out/write.log 2>&1 || exit 1
echo done
