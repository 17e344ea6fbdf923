# NS end-to-end numbers on the final build: config 5 bench, and the drop-in
# host program on assignment-6 dcavity.par read as 2D (128^2, te = 10: 4628 steps)
set -e
export TMPDIR=/tmp
o=gpurun_out/nsfinal; mkdir -p $o/dc
timeout -k 10 300 python bench.py --workload ns --no-cpu-baseline > $o/ns16384.json 2> $o/ns16384.err
cp tests/golden/a6_dcavity.par $o/dc/dcavity.par
(cd $o/dc && timeout -k 10 300 ../../../practical-parallel-algorithms-with-mpi_amd/bin/exe-ns dcavity.par > run.log 2>&1)
