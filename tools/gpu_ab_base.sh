# A/B on one box (bash tools/gpu_ab_base.sh <tag>), alternated:
#  - the unchained 32768^2 pass, this build against the round-start build
#    (lib_ab/libmisor_base.so, git a50daf0);
#  - the cost of an order-independent residual: this build against the same
#    sources built with -DMISOR_RES_BINNED (lib_ab/libmisor_rx.so, sor_tb.h
#    TallyAcc), at 32768^2 and on one 8-GPU rank's block;
# then the strong-scaling proxy and the 8-local-rank bench.
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
o=gpurun_out/ab_base_$tag.txt
: > $o
P="python tools/scale_proxy.py --tsteps 8 --rows 0 --rounds 2 --sweeps 56"
for r in 1 2 3; do
  for L in "" lib_ab/libmisor_base.so lib_ab/libmisor_rx.so; do
    echo "# lib ${L:-current}" >> $o
    timeout -k 10 120 $P --shapes 32768x32768 ${L:+--lib $L} >> $o 2>&1
  done
  for L in "" lib_ab/libmisor_rx.so; do
    echo "# lib ${L:-current}" >> $o
    timeout -k 10 120 $P --shapes 8192x16384:8 ${L:+--lib $L} >> $o 2>&1
  done
done
timeout -k 10 300 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 2 --sweeps 56 --chain=-1,0 \
    > gpurun_out/scale_proxy_$tag.txt 2>&1
timeout -k 10 200 python bench.py --local-ranks 8 --size 8192 --steps 20 --warmup 3 --check \
    > gpurun_out/bench_local8_$tag.json 2> gpurun_out/bench_local8_$tag.err
