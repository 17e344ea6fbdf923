# round-4: TB variants (9 skew, 10/11 LDS row queue, 12 split rhs ring) --
# parity tests, then A/B against the default kernel at 32768^2 and the
# driver's 20-step bench at T = 10 on the split ring
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tb_variants_gpu.py \
  > $o/tbv_tests.log 2>&1 || { echo "variant tests failed"; tail -30 $o/tbv_tests.log; exit 1; }
tail -3 $o/tbv_tests.log
timeout -k 10 500 python tools/ab_libs.py --size 32768 --passes 4 --rounds 2 \
  main::0:8 main::12:8 main::13:8 main::12:10 main::13:10 main::13:12 main::0:7 > $o/hr_ab.txt 2>&1 || exit 1
cat $o/hr_ab.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline > $o/hr_b20_base.json 2> $o/hr_b20_base.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 7 --no-cpu-baseline --tb-variant 13 --tsteps 10 > $o/hr_b20_t10.json 2> $o/hr_b20_t10.err || exit 1
cat $o/hr_b20_base.json $o/hr_b20_t10.json
echo done
