# round-4: the short pass plan on 2-rank blocks -- whole-field parity (LOCAL
# transport, 2 ranks) and the bench's --local-ranks leg
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 350 --timeout-method thread tests/test_fullfield_gpu.py -k "ranks" > $o/ff_ranks.log 2>&1 || { echo "ff failed"; tail -30 $o/ff_ranks.log; exit 1; }
tail -4 $o/ff_ranks.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_decomposed_gpu.py tests/test_bench_local_gpu.py > $o/dec_tests.log 2>&1 || { echo "dec failed"; tail -30 $o/dec_tests.log; exit 1; }
tail -2 $o/dec_tests.log
echo done
