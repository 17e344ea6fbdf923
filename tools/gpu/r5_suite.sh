#!/bin/bash
# smoke + the whole -m gpu suite + the driver's bench setting (bash tools/gpu/r5_suite.sh <tag>)
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --durations=30 --maxfail=15 --timeout 250 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$tag.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$tag.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
cat gpurun_out/bench_$tag.json
