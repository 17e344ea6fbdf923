# The reference's sequential NS (assignment-5/sequential/dcavity.par, te=10,
# 80,000 steps, lexicographic solve) end to end on the GPU host program, then
#  - per-step pressure iterations against the oracle's (the reference's
#    arithmetic incl. its sequential residual sum; tests/golden/*_full_iters.npz)
#  - pressure.dat / velocity.dat against the reference's own output built with
#    gcc -O2 -ffp-contract=off (seq_refgcc_*) and the committed one (seq_*, made
#    by the reference's clang build)
#   bash tools/ns_seq_lex_full.sh   (on the GPU box)
set -e
out=gpurun_out/ns_seq_lex
mkdir -p $out
cp tests/golden/seq_dcavity.par $out/dcavity.par
( cd $out && MISOR_SOLVER=lex MISOR_ITERLOG=iters.log timeout -k 10 900 ../../practical-parallel-algorithms-with-mpi_amd/bin/exe-ns dcavity.par > run.log 2>&1 )
python3 - <<'PY' | tee $out/compare.txt
import numpy as np
d = "gpurun_out/ns_seq_lex/"
it = np.loadtxt(d + "iters.log")[:, 3].astype(int)
ref = np.load("tests/golden/ns_seq_dcavity_lex_full_iters.npz")["iters"].astype(int)
diff = np.flatnonzero(it != ref)
print("steps", len(it), len(ref), "total iterations", int(it.sum()), int(ref.sum()),
      "steps with a different iteration count:", len(diff), "first:", diff[:5].tolist())
for f in ("pressure.dat", "velocity.dat"):
    a = np.loadtxt(d + f)
    for tag in ("refgcc_", ""):
        b = np.loadtxt("tests/golden/seq_" + tag + f)
        same = open(d + f).read() == open("tests/golden/seq_" + tag + f).read()
        print(f, "vs", "reference gcc build" if tag else "committed (clang build)",
              "max|diff|", float(np.abs(a - b).max()),
              "byte-identical" if same else "not byte-identical")
PY
