# One GPU-box session: smoke, full -m gpu suite, profiled default bench, scaling proxies.
#   bash tools/gpu_round.sh <tag>
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 170 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1
bash tools/profile_bench.sh $tag
timeout -k 10 300 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 2 --sweeps 56 \
    > gpurun_out/scale_proxy_$tag.txt 2>&1
# the driver's launcher path with one rank
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 1 --steps 24 --warmup 8 --no-cpu-baseline \
    > gpurun_out/bench_torchrun_$tag.json 2> gpurun_out/bench_torchrun_$tag.err
timeout -k 10 300 python bench.py --scaling weak --steps 24 --warmup 8 --no-cpu-baseline \
    > gpurun_out/bench_weak_$tag.json 2> gpurun_out/bench_weak_$tag.err
