# exchange-variant benches (20 / 140 steps, T = 10 / 8, W = 4 / 8) + one kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for T in 10 8; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline --tb-variant 6 --tsteps $T > gpurun_out/xch_b20_t$T.json 2> gpurun_out/xch_b20_t$T.err || exit 1
  timeout -k 10 300 python bench.py --steps 140 --warmup 7 --no-cpu-baseline --tb-variant 6 --tsteps $T > gpurun_out/xch_b140_t$T.json 2> gpurun_out/xch_b140_t$T.err || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline --tb-variant 7 --tsteps 10 > gpurun_out/xch8_b20_t10.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline > gpurun_out/base_b20.json 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_xch -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 7 --no-cpu-baseline --tb-variant 6 --tsteps 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_xch.log 2>&1
echo done
