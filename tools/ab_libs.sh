# Interleaved A/B of two libmisor builds on the rank blocks of the 1- and 8-GPU splits:
#   bash tools/ab_libs.sh A/libmisor.so B/libmisor.so [extra scale_proxy args]
set -e
A=$1; B=$2; shift 2
for r in 1 2; do
 for L in $A $B; do
  echo "== $L"; timeout -k 10 120 python tools/scale_proxy.py --lib $L --shapes 32768x32768,8192x16384 --rows 0 --sweeps 84 --rounds 3 --tsteps 7 "$@"
 done
done
