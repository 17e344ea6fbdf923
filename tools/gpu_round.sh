# One GPU-box session: full -m gpu suite, profiled default bench, comm-pipeline proxy.
#   bash tools/gpu_round.sh <tag>
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 170 --timeout-method thread \
    > gpurun_out/gpu_tests_$tag.log 2>&1
bash tools/profile_bench.sh $tag
timeout -k 10 300 python tools/scale_proxy.py --comm --tsteps 7,8 --rows 0 --rounds 2 --sweeps 48 \
    > gpurun_out/scale_proxy_comm_$tag.txt 2>&1
timeout -k 10 300 python tools/scale_proxy.py --tsteps 7,8 --rows 0 --rounds 2 --sweeps 48 \
    > gpurun_out/scale_proxy_$tag.txt 2>&1
