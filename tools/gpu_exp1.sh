# round-4 experiments: exchange variant builds / widths vs the default kernel; the default
# bench with its CPU baselines; chained-pass knobs on one 8-GPU rank's block
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
L=practical-parallel-algorithms-with-mpi_amd
timeout -k 10 600 python tools/ab_libs.py --size 32768 --passes 4 --rounds 2 \
  main::0:8 main::6:10 main::6:8 main::8:10 main::7:10 x0:$L/lib_x0/libmisor.so:6:10 xn:$L/lib_xn/libmisor.so:6:10 \
  > $o/e1_ablibs.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 7 > $o/e1_base_b20.json 2> $o/e1_base_b20.err || exit 1
timeout -k 10 400 python tools/ab_env.py --var MISOR_CHAIN_EDGE_COST --values 1.5,1.77,2.0 --ni 8192 --nj 16384 --size 32768 --tsteps 8 --passes 12 --rounds 2 > $o/e1_edgecost.txt 2>&1 || exit 1
echo done
