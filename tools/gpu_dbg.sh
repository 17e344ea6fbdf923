set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/debug_xch.py > gpurun_out/dbg_xch.txt 2>&1; echo rc=$?
cat gpurun_out/dbg_xch.txt | tail -20
