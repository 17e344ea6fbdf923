set -e
export TMPDIR=/tmp
o=gpurun_out/even; mkdir -p $o
for e in 1 0 1 0; do
  MISOR_EVEN_PASSES=$e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> $o/steps20_even$e.json 2>>$o/err.log
  MISOR_EVEN_PASSES=$e timeout -k 10 200 python bench.py --steps 140 --warmup 7 --no-cpu-baseline >> $o/steps140_even$e.json 2>>$o/err.log
done
timeout -k 10 600 python -u -m pytest tests/test_sor_gpu.py tests/test_bench_configs_gpu.py tests/test_decomposed_gpu.py -x -q -m gpu --timeout 170 --timeout-method thread -k "not 8_ranks" > $o/tests.log 2>&1
