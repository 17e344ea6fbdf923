# compute-only proxy of one 8-GPU rank's block (tools/scale_proxy.py) and of
# N = 1: this build against the round-3 build (lib_r3), alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
L=practical-parallel-algorithms-with-mpi_amd/lib_r3/libmisor.so
rm -f $o/proxy_r4ab.txt
for r in 1 2; do
  echo "# current" >> $o/proxy_r4ab.txt
  timeout -k 10 300 python tools/scale_proxy.py --ranks 1,8 --tsteps 8 --rows 0 --chain=-1 --sweeps 24 --rounds 2 >> $o/proxy_r4ab.txt 2>&1 || exit 1
  echo "# round 3" >> $o/proxy_r4ab.txt
  timeout -k 10 300 python tools/scale_proxy.py --lib $L --ranks 1,8 --tsteps 8 --rows 0 --chain=-1 --sweeps 24 --rounds 2 >> $o/proxy_r4ab.txt 2>&1 || exit 1
done
cat $o/proxy_r4ab.txt
echo done
