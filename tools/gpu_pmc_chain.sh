# PMC traffic of chained vs unchained passes (bash tools/gpu_pmc_chain.sh <tag>)
export TMPDIR=/tmp
tag=$1
for sh in 32768x32768:1 8192x16384:8; do
  for ch in 1 0; do
    d=gpurun_out/pmc_${tag}_${sh%%:*}_c$ch
    mkdir -p $d
    P="python tools/scale_proxy.py --shapes $sh --tsteps 8 --rows 0 --rounds 1 --sweeps 16 --chain $ch"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $d -o fetch --output-format csv -- $P > $d/fetch.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $d -o write --output-format csv -- $P > $d/write.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $d -o trace --output-format csv -- $P > $d/trace.log 2>&1 || exit 1
  done
done
