# The reference's sequential NS (assignment-5/sequential/dcavity.par, te=10,
# 80,000 steps, lexicographic solve) end to end on the GPU host program, then
# its pressure.dat / velocity.dat against the committed reference outputs.
#   bash tools/ns_seq_lex_full.sh   (on the GPU box)
set -e
out=gpurun_out/ns_seq_lex
mkdir -p $out
cp tests/golden/seq_dcavity.par $out/dcavity.par
( cd $out && MISOR_SOLVER=lex timeout -k 10 900 ../../practical-parallel-algorithms-with-mpi_amd/bin/exe-ns dcavity.par > run.log 2>&1 )
python3 - <<'PY' | tee $out/compare.txt
import numpy as np
d = "gpurun_out/ns_seq_lex/"
for f in ("pressure.dat", "velocity.dat"):
    a = np.loadtxt(d + f); b = np.loadtxt("tests/golden/seq_" + f)
    same = open(d + f).read() == open("tests/golden/seq_" + f).read()
    print(f, "rows", a.shape, b.shape, "max|diff|", float(np.abs(a - b).max()),
          "byte-identical" if same else "not byte-identical")
PY
