# block height at T = 10 (split ring) and T = 8 (default): fewer warm-up rows
# per block against the pass's load balance
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 400 python tools/ab_env.py --var MISOR_TB_TARGET_ROWS --values 576,864,1152,1728 --size 32768 --tsteps 10 --variant 12 --passes 4 --rounds 2 > $o/rows_hr10.txt 2>&1 || exit 1
cat $o/rows_hr10.txt
timeout -k 10 400 python tools/ab_env.py --var MISOR_TB_TARGET_ROWS --values 576,1152 --size 32768 --tsteps 8 --variant 0 --passes 4 --rounds 2 > $o/rows_t8.txt 2>&1 || exit 1
cat $o/rows_t8.txt
echo done
