# round-4: the resident 3D solve -- parity tests of the default (1024 threads,
# register-resident thread columns, deep red cells during the barrier) and of
# the LDS-only form, then timing against the round-3 form (112)
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
for m in 240 4336; do
  MISOR3_RESIDENT_MODE=$m timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_ns3d_gpu.py -k "resident or solve" > $o/res3d_tests_$m.log 2>&1 || { echo "tests failed mode $m"; tail -20 $o/res3d_tests_$m.log; exit 1; }
  tail -1 $o/res3d_tests_$m.log
done
rm -f $o/res3d_modes_r4c.txt
for r in 1 2; do
for m in 240 4336 112; do
  echo "mode $m" >> $o/res3d_modes_r4c.txt
  MISOR3_RESIDENT_MODE=$m timeout -k 10 120 python tools/tune3d.py --size 128 --iters 400 --reps 3 --configs 1,8,0,1,0,1 >> $o/res3d_modes_r4c.txt 2>&1 || exit 1
done
done
cat $o/res3d_modes_r4c.txt
echo done
