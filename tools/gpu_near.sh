# near-threshold (N1) tests + the round-4 experiments (tools/gpu_exp1.sh), one box
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread --durations=10 tests/test_near_threshold_gpu.py tests/test_sor_gpu.py tests/test_decomposed_gpu.py -k "near or kat or poisson_par or fixed_sweeps" > gpurun_out/near_tests.log 2>&1
echo "rc=$?"; tail -15 gpurun_out/near_tests.log
bash tools/gpu_exp1.sh
