# per-launch time of the default TB kernel against T at 32768^2 (ms per
# iteration x T): the intercept is the launch's T-independent (streaming) part
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 500 python tools/ab_libs.py --size 32768 --passes 4 --rounds 2 \
  main::0:1 main::0:2 main::0:3 main::0:4 main::0:5 main::0:6 main::0:7 main::0:8 main::9:8 > $o/tcurve.txt 2>&1 || exit 1
cat $o/tcurve.txt
echo done
