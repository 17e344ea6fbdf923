#!/bin/bash
# resource usage (VGPRs, scratch) of the exchange kernel for the T values given
cd /root/repo/practical-parallel-algorithms-with-mpi_amd
for T in "$@"; do
  echo "T=$T"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc \
    -DMISOR_TB_T=$T ${EXTRA} -c /tmp/tbx_only.hip -o /tmp/tx_$T.o -Rpass-analysis=kernel-resource-usage 2>&1 \
    | grep -E "error|VGPRs:|ScratchSize|LDS Size" | sed 's/.*remark: *//'
done
