set -e
for r in 1 2; do
 for L in ab/old/libmisor.so practical-parallel-algorithms-with-mpi_amd/lib/libmisor.so; do
  echo "== $L"; timeout -k 10 120 python tools/scale_proxy.py --lib $L --shapes 32768x32768,8192x16384 --rows 0 --sweeps 84 --rounds 3 --tsteps 7
 done
done
