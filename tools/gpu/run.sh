#!/bin/bash
# GPU-box evidence runs, one parameterised script (replaces round 5's one-off
# tools/gpu/r5_*.sh).  Run through gpurun:
#   gpurun -- 'bash tools/gpu/run.sh TAG STEP [STEP ...]'
# STEPs, in the order given (each under its own time limit; the first failure
# ends the call, nothing further touches the GPU):
#   smoke   __graft_entry__.smoke()
#   suite   python -m pytest tests -m gpu (the driver's GPU suite)
#   tests=EXPR   the GPU tests selected by -k EXPR
#   bench   bench.py --steps 20 --warmup 5 (the driver's N = 1 line, CPU baselines included)
#   quick   bench.py --steps 20 --warmup 5 --no-cpu-baseline
#   trace   rocprofv3 --kernel-trace --stats of the quick bench
#   pmc     rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ) of the quick bench
#   ns      bench.py --workload ns (config 5, 16384^2), and its kernel trace + PMC
#   ns3d    bench.py --workload ns3d (128^3)
#   proxy   one-GPU proxies of the decomposed ranks (needs lib_proxy, the MISOR_PROXY build)
#   micro   tools/micro/fp64_lat.bin (FP64 issue / latency microbenchmark)
# Outputs: gpurun_out/TAG/...
set -o pipefail
export TMPDIR=/tmp
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
B="python bench.py --steps 20 --warmup 5"
NS="python bench.py --workload ns --steps 20 --warmup 3"
die() { echo "FAILED: $*"; tail -30 "$out/$2" 2>/dev/null; exit 1; }
pmc_passes() {  # name, command...
    local name=$1
    shift
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$out/${name}_pmc" -o fetch --output-format csv -- "$@" \
        > "$out/${name}_fetch.log" 2>&1 || return 1
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$out/${name}_pmc" -o write --output-format csv -- "$@" \
        > "$out/${name}_write.log" 2>&1 || return 1
    timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
        -d "$out/${name}_pmc" -o sq --output-format csv -- "$@" > "$out/${name}_sq.log" 2>&1 || return 1
}
for step in "$@"; do
    echo "== $step $(date +%T)"
    case $step in
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
            > "$out/smoke.log" 2>&1 || die smoke smoke.log
        tail -1 "$out/smoke.log" ;;
    suite)
        timeout -k 10 1100 python -u -m pytest tests -v -m gpu --durations=30 --timeout 250 \
            --timeout-method thread > "$out/gpu_tests.log" 2>&1 || die suite gpu_tests.log
        tail -1 "$out/gpu_tests.log" ;;
    tests=*)
        timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 250 --timeout-method thread \
            -k "${step#tests=}" > "$out/gpu_tests_k.log" 2>&1 || die "$step" gpu_tests_k.log
        tail -1 "$out/gpu_tests_k.log" ;;
    bench)
        timeout -k 10 400 $B > "$out/bench.json" 2> "$out/bench.err" || die bench bench.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['bound'])" "$out/bench.json" ;;
    quick)
        timeout -k 10 200 $B --no-cpu-baseline > "$out/quick.json" 2> "$out/quick.err" || die quick quick.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('quick', d['ms_per_step'], d['roofline']['kernel_ms'])" "$out/quick.json" ;;
    trace)
        timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv \
            -- $B --no-cpu-baseline > "$out/trace.log" 2>&1 || die trace trace.log ;;
    pmc)
        pmc_passes bench $B --no-cpu-baseline || die pmc bench_sq.log ;;
    ns)
        timeout -k 10 300 $NS > "$out/ns.json" 2> "$out/ns.err" || die ns ns.err
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('NS', d['ms_per_step'], d['solve_kernel_ms_per_step'], d['other_ms_per_step'])" "$out/ns.json"
        timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$out/ns_trace" -o trace --output-format csv \
            -- $NS --no-cpu-baseline > "$out/ns_trace.log" 2>&1 || die ns-trace ns_trace.log
        pmc_passes ns $NS --no-cpu-baseline || die ns-pmc ns_sq.log ;;
    ns3d)
        timeout -k 10 300 python bench.py --workload ns3d --steps 5 --warmup 2 > "$out/ns3d.json" \
            2> "$out/ns3d.err" || die ns3d ns3d.err ;;
    proxy)
        P="python tools/scale_proxy.py --sweeps 20 --rows 0 --tsteps 10 --variants 13 --rounds 5"
        : > "$out/proxy.txt"
        for sh in "8192x16384:8 --sides LB" "8192x16384:8 --sides B" "16384x8192:8 --sides LB" \
                  "32768x4096:8 --sides LRB" "16384x16384:4 --sides LB" "16384x32768:2 --sides LBT"; do
            timeout -k 10 200 $P --shapes $sh > "$out/proxy_tmp.txt" 2>&1 || die proxy proxy_tmp.txt
            grep -v "^RCCL\|^HIP\|^ROCm\|^Host\|^Lib\|^N " "$out/proxy_tmp.txt" | sed "s/^/$sh: /" \
                | tee -a "$out/proxy.txt"
        done ;;
    micro)
        timeout -k 10 200 tools/micro/fp64_lat.bin > "$out/fp64_lat.txt" 2>&1 || die micro fp64_lat.txt ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== done $(date +%T)"
