# chained-pass session: proxy, bench, then the decomposed tests timed (bash tools/gpu_chain.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 2 --sweeps 56 \
    > gpurun_out/scale_proxy_$tag.txt 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.json 2>gpurun_out/bench_$tag.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20_$tag.json 2>gpurun_out/bench20_$tag.err
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu --durations=30 \
    tests/test_decomposed_gpu.py > gpurun_out/dec_$tag.log 2>&1
