# TB variants (9 skew, 10/11 LDS row queue, 13 skewed split ring) -- parity
# tests, the whole-field driver sequence, then the driver's 20-step bench
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tb_variants_gpu.py \
  > $o/tbv_tests.log 2>&1 || { echo "variant tests failed"; tail -30 $o/tbv_tests.log; exit 1; }
tail -2 $o/tbv_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 350 --timeout-method thread tests/test_fullfield_gpu.py \
  > $o/ff_tests.log 2>&1 || { echo "fullfield failed"; tail -30 $o/ff_tests.log; exit 1; }
tail -2 $o/ff_tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline > $o/wu_b20_$r.json 2> $o/wu_b20_$r.err || exit 1
  MISOR_SHORT_PLAN=0 timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline > $o/wu_b20_off_$r.json 2> $o/wu_b20_off_$r.err || exit 1
done
for f in $o/wu_b20_1.json $o/wu_b20_off_1.json $o/wu_b20_2.json $o/wu_b20_off_2.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"; done
echo done
