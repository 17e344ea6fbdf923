# smoke + the whole -m gpu suite (bash tools/gpu_suite.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --durations=25 --timeout 250 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
