#!/bin/bash
# Time-to-solution of the 2D NS drivers on assignment-6's .par files (read as 2D).
# GPU: the reference-compatible host program bin/exe-ns (libmisor).
# Usage: tools/ns_time.sh <par> [te]
set -e
par=$1; te=${2:-}
tmp=$(mktemp -d)
cp "$par" "$tmp/run.par"
if [ -n "$te" ]; then sed -i "s/^te .*/te       $te/" "$tmp/run.par"; fi
bin=$(cd "$(dirname "$0")/.." && pwd)/practical-parallel-algorithms-with-mpi_amd/bin/exe-ns
cd "$tmp"
start=$(date +%s.%N)
MISOR_ITERLOG=iters.log "$bin" run.par > out.log
end=$(date +%s.%N)
steps=$(wc -l < iters.log)
sweeps=$(awk '{s+=$4} END {print s}' iters.log)
grep "Solution took" out.log
python3 -c "print(\"wall %.2f s, steps $steps, sweeps $sweeps\" % ($end - $start))"
rm -rf "$tmp"
