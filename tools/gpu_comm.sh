# the decomposed, pipelined pass loop on one 8-GPU rank's block (scale_proxy
# --comm: a one-rank RCCL communicator -- comm stream, all-reduce, split
# launches, no neighbours) against the plain single-rank pass loop
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 300 python tools/scale_proxy.py --ranks 8 --tsteps 8 --rows 0 --chain=-1 --sweeps 24 --rounds 2 > $o/proxy_nocomm.txt 2>&1 || exit 1
timeout -k 10 300 python tools/scale_proxy.py --ranks 8 --tsteps 8 --rows 0 --chain=-1 --sweeps 24 --rounds 2 --comm > $o/proxy_comm.txt 2>&1 || exit 1
cat $o/proxy_nocomm.txt $o/proxy_comm.txt
echo done
