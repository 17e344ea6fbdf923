#!/bin/bash
# build_variant.sh NAME "FLAGS" "T values": an experiment copy of libmisor.so,
# practical-parallel-algorithms-with-mpi_amd/lib_NAME/libmisor.so, with the TB units of the
# given T recompiled with FLAGS (the rest reused from build/); tools/ab_libs.py times them
set -e
cd /root/repo/practical-parallel-algorithms-with-mpi_amd
name=$1; flags=$2; ts=$3
mkdir -p build_$name lib_$name
cp build/*.o build_$name/
for t in $ts; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result \
    -I../include -Icsrc -DMISOR_TB_T=$t $flags -c csrc/sor_tb_inst.hip -o build_$name/sor_tb_t$t.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_$name/libmisor.so build_$name/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built lib_$name/libmisor.so
