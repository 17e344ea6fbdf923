# round-4: the resident 3D solve -- parity tests (1024 threads, residual sums
# folded into the grid barrier; and the register-column form), then timing of
# the forms: 240 (1024 threads), 4336 (+ register columns), 368 (512), 4464
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
for m in 240 4336 4464; do
  MISOR3_RESIDENT_MODE=$m timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_ns3d_gpu.py -k "resident or solve" > $o/res3d_tests_$m.log 2>&1 || { echo "tests failed mode $m"; tail -20 $o/res3d_tests_$m.log; exit 1; }
  tail -1 $o/res3d_tests_$m.log
done
rm -f $o/res3d_modes_r4e.txt
for r in 1 2 3; do
  for m in 240 4336 368 4464; do
    echo "mode $m" >> $o/res3d_modes_r4e.txt
    MISOR3_RESIDENT_MODE=$m timeout -k 10 120 python tools/tune3d.py --size 128 --iters 400 --reps 3 --configs 1,8,0,1,0,1 >> $o/res3d_modes_r4e.txt 2>&1 || exit 1
  done
done
cat $o/res3d_modes_r4e.txt
echo done
