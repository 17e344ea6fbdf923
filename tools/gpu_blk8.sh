# one 8-GPU rank's block (8192 x 16384): the default chained passes (T = 7, as
# the 20-iteration split 7 + 7 + 6 runs) against split-ring passes of 10
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 400 python tools/ab_libs.py --ni 8192 --nj 16384 --size 32768 --passes 12 --rounds 3 \
  main::0:7 main::0:8 main::13:10 main::12:10 > $o/blk8.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab_libs.py --ni 16384 --nj 16384 --size 32768 --passes 12 --rounds 2 \
  main::0:7 main::13:10 > $o/blk4.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab_libs.py --ni 16384 --nj 32768 --size 32768 --passes 8 --rounds 2 \
  main::0:7 main::13:10 > $o/blk2.txt 2>&1 || exit 1
cat $o/blk8.txt $o/blk4.txt $o/blk2.txt
echo done
