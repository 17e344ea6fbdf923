# 3D resident solve: the whole 3D suite under the two barrier layouts, their
# timings, the 128^3 bench and a kernel trace (bash tools/gpu_r3c.sh <tag>)
set -e
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
T3="tests/test_ns3d_gpu.py tests/test_ns3d_decomposed_gpu.py tests/test_ns3d_host_gpu.py"
for m in 48 112; do
  MISOR3_RESIDENT_MODE=$m timeout -k 10 400 python -u -m pytest $T3 -q --timeout 150 --timeout-method thread \
      > gpurun_out/r3c_tests_${tag}_m$m.log 2>&1 || rc=$?
  rc=${rc:-0}; if [ $rc -gt 1 ]; then exit $rc; fi; rc=0
done
o=gpurun_out/r3c_modes_$tag.txt; : > $o
for m in 48 112 48 112; do
  echo "mode $m" >> $o
  MISOR3_RESIDENT_MODE=$m timeout -k 10 100 python tools/tune3d.py --size 128 --iters 400 --configs 1,8,0,1,0,1 >> $o 2>&1
done
timeout -k 10 100 python tools/tune3d.py --size 128 --iters 400 --configs 1,8,0,1,0,0 >> $o 2>&1
timeout -k 10 200 python bench.py --workload ns3d > gpurun_out/r3c_bench128_$tag.json 2> gpurun_out/r3c_bench128_$tag.err
p=gpurun_out/r3c_prof_$tag; mkdir -p $p
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $p -o trace --output-format csv -- python bench.py --workload ns3d --no-cpu-baseline --steps 6 --warmup 1 > $p/trace.log 2>&1
