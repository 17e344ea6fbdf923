#!/bin/bash
# 3D: parity of the spread partial sum, A/B against the previous build; lex sanity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ns3d_gpu.py tests/test_ns3d_decomposed_gpu.py tests/test_ns3d_host_gpu.py tests/test_lex_gpu.py -x -q --durations=4 --timeout 250 --timeout-method thread > gpurun_out/r5l_tests.log 2>&1 || { tail -30 gpurun_out/r5l_tests.log; exit 1; }
tail -6 gpurun_out/r5l_tests.log
timeout -k 10 400 python tools/ab3d.py --libs main:,old:practical-parallel-algorithms-with-mpi_amd/lib_x/libmisor.so --rounds 4 > gpurun_out/r5l_ab3d.txt 2>&1 || { tail gpurun_out/r5l_ab3d.txt; exit 1; }
cat gpurun_out/r5l_ab3d.txt
timeout -k 10 300 python bench.py --workload ns3d --steps 5 --warmup 2 > gpurun_out/r5l_ns3d.json 2> gpurun_out/r5l_ns3d.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r5l_ns3d.json')); print('NS3D', d['ms_per_step'], d['roofline'].get('solve_ms_per_iteration'))"
