# round-4 evidence for the driver's configuration (32768^2, --steps 20): the
# short pass plan's parity (whole field), the bench line with CPU baselines,
# rocprofv3 kernel trace and PMC passes of the same command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/prof_r4
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_fullfield_gpu.py \
  -k bench_sequence > $o/fullfield.log 2>&1 || { echo "fullfield failed"; tail -20 $o/fullfield.log; exit 1; }
tail -2 $o/fullfield.log
timeout -k 10 400 python bench.py --steps 20 --warmup 7 > $o/bench.json 2> $o/bench.err || exit 1
cat $o/bench.json
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $o -o trace --output-format csv -- python bench.py --steps 20 --warmup 7 --no-cpu-baseline > $o/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $o -o fetch --output-format csv -- $B > $o/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $o -o write --output-format csv -- $B > $o/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $o -o sq --output-format csv -- $B > $o/sq.log 2>&1 || exit 1
python tools/pmc_summary.py $o $o/pmc_tbh10.json --size 32768 --iters 10 > $o/pmc.log 2>&1 || true
find $o -name "*kernel_stats.csv" | head -3
echo done
