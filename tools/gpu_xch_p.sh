set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_bench.sh xch8 --steps 16 --warmup 8 --tb-variant 6 --tsteps 8 || exit 1
bash tools/profile_bench.sh old8 --steps 16 --warmup 8 --tsteps 8 || exit 1
python tools/pmc_summary.py gpurun_out/prof_xch8 gpurun_out/pmc_xch8.json --iters 8 > /dev/null 2>&1
python tools/pmc_summary.py gpurun_out/prof_old8 gpurun_out/pmc_old8.json --iters 8 > /dev/null 2>&1
echo done
