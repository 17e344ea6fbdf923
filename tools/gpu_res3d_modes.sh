# resident 3D solve: cost of its parts (MISOR3_RESIDENT_MODE experiments; modes 2-7
# compute wrong values -- timing only) (bash tools/gpu_res3d_modes.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
o=gpurun_out/res3d_modes_$tag.txt; : > $o
timeout -k 10 300 python -u -m pytest tests/test_ns3d_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "resident or short_run or medium" > gpurun_out/res3d_tests_$tag.log 2>&1
for m in 0 1 3 5 7; do
  echo "mode $m" >> $o
  MISOR3_RESIDENT_MODE=$m timeout -k 10 100 python tools/tune3d.py --size 128 --iters 200 --configs 1,8,0,1,0,1 >> $o 2>&1
done
