# round-4: the resident 3D solve -- parity tests of the default (register
# columns, far x-neighbour by DPP) and timing against the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
for m in 240 4336; do
  MISOR3_RESIDENT_MODE=$m timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_ns3d_gpu.py -k "resident or solve" > $o/res3d_tests_$m.log 2>&1 || { echo "tests failed mode $m"; tail -20 $o/res3d_tests_$m.log; exit 1; }
  tail -1 $o/res3d_tests_$m.log
done
rm -f $o/res3d_modes_r4f.txt
P=practical-parallel-algorithms-with-mpi_amd/lib_prev/libmisor.so
for r in 1 2 3; do
  echo "cur" >> $o/res3d_modes_r4f.txt
  timeout -k 10 120 python tools/tune3d.py --size 128 --iters 400 --reps 3 --configs 1,8,0,1,0,1 >> $o/res3d_modes_r4f.txt 2>&1 || exit 1
  echo "prev" >> $o/res3d_modes_r4f.txt
  timeout -k 10 120 python tools/tune3d.py --lib $P --size 128 --iters 400 --reps 3 --configs 1,8,0,1,0,1 >> $o/res3d_modes_r4f.txt 2>&1 || exit 1
done
cat $o/res3d_modes_r4f.txt
echo done
