# resident 3D solve: cost of its parts (MISOR3_RESIDENT_MODE experiments; modes 2-7
# compute wrong values -- timing only) (bash tools/gpu_res3d_modes.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
o=gpurun_out/res3d_modes_$tag.txt; : > $o
for m in ${TMODES:-16}; do
  MISOR3_RESIDENT_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_ns3d_gpu.py -q --timeout 120 --timeout-method thread \
    -k "resident or short_run or medium" > gpurun_out/res3d_tests_${tag}_m$m.log 2>&1 || rc=$?
  rc=${rc:-0}; if [ $rc -gt 1 ]; then echo "mode $m: pytest rc $rc" >> $o; exit $rc; fi; rc=0
done
for m in ${MODES:-16 26 30}; do
  echo "mode $m" >> $o
  MISOR3_RESIDENT_MODE=$m timeout -k 10 100 python tools/tune3d.py --size 128 --iters 200 --configs 1,8,0,1,0,1 >> $o 2>&1
done
