#!/bin/bash
# lex tests (DPP form), the NS and 3D lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lex_gpu.py tests/test_host_programs_gpu.py -x -q --durations=6 --timeout 250 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1 || { tail -30 gpurun_out/r5k_tests.log; exit 1; }
tail -9 gpurun_out/r5k_tests.log
timeout -k 10 300 python bench.py --workload ns --steps 20 --warmup 3 > gpurun_out/r5k_ns.json 2> gpurun_out/r5k_ns.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5k_ns.json')); print('NS', d['ms_per_step'], d['solve_kernel_ms_per_step'], d['other_ms_per_step'])"
timeout -k 10 300 python bench.py --workload ns3d --steps 5 --warmup 2 > gpurun_out/r5k_ns3d.json 2> gpurun_out/r5k_ns3d.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5k_ns3d.json')); print('NS3D', d['ms_per_step'], d['roofline'].get('solve_ms_per_iteration'))"
