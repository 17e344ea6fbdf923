# round-4 experiments: exchange variant (prefetch build) vs default; chained-pass knobs on
# one 8-GPU rank's block
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
for T in 10 8; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline --tb-variant 6 --tsteps $T > $o/e1_xch_b20_t$T.json 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline > $o/e1_base_b20.json 2>&1 || exit 1
timeout -k 10 400 python tools/ab_env.py --var MISOR_CHAIN_EDGE_COST --values 1.5,1.77,2.0 --ni 8192 --nj 16384 --size 32768 --tsteps 8 --passes 12 --rounds 2 > $o/e1_edgecost.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab_env.py --var MISOR_TB_CHAIN_RINGS --values 3,4 --ni 8192 --nj 16384 --size 32768 --tsteps 8 --passes 12 --rounds 2 > $o/e1_rings.txt 2>&1 || exit 1
echo done
