# three-level block rows + 3D deep prefetch: parity tests, proxy A/B, 3D tuning, bench
set -e
export TMPDIR=/tmp
o=gpurun_out/r2g; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests/test_sor_gpu.py tests/test_decomposed_gpu.py tests/test_bench_configs_gpu.py tests/test_ns3d_gpu.py -x -v -m gpu --timeout 170 --timeout-method thread > $o/tests.log 2>&1
timeout -k 10 300 python tools/tune3d.py --size 128 384 --iters 300 --configs 1,8,0 1,8,0,0,0 1,8,0,1,1 1,4,8 1,8,4 1,8,16 > $o/tune3d.txt 2>&1
for lv in 2 3 2 3; do MISOR_TB_LEVELS=$lv timeout -k 10 300 python tools/scale_proxy.py --tsteps 8,7 --rows 0 --rounds 2 --sweeps 56 >> $o/proxy_levels$lv.txt 2>&1; done
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err
