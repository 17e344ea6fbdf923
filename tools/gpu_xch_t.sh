# exchange-variant parity tests only (no -x: the full failure pattern)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_xch_gpu.py > gpurun_out/xch_tests.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/xch_tests.log
