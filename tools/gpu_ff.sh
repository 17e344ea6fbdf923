set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_fullfield_gpu.py > gpurun_out/ff.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline > gpurun_out/bench20.json 2> gpurun_out/bench20.err
