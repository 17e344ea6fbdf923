# the secondary bench lines: NS config 5 (dcavity 16384^2 per GPU) and the 3D
# 128^3 solve, for the record
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 400 python bench.py --workload ns --no-cpu-baseline > $o/line_ns.json 2> $o/line_ns.err || exit 1
timeout -k 10 300 python bench.py --workload ns3d --no-cpu-baseline > $o/line_ns3d.json 2> $o/line_ns3d.err || exit 1
cat $o/line_ns.json $o/line_ns3d.json
echo done
