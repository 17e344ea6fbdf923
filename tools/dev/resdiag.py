"""Decomposed res against the restatement, per iteration count (diagnostic, GPU box)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "practical-parallel-algorithms-with-mpi_amd")
import orc
import test_res_lite_gpu as t

NI, NJ = t.NI, t.NJ
dx, dy = 1.0 / NI, 1.0 / NJ
rng = np.random.default_rng(7)
p0 = rng.standard_normal((NJ + 2, NI + 2))
rhs = rng.standard_normal((NJ + 2, NI + 2))
q, res = p0.copy(), {}
for k in range(1, 31):
    res[k] = orc.solve_rb(q, rhs, dx, dy, 1.9, 1e-300, 1)[1]
for world, T, var in ((4, 10, 13), (4, 8, 0), (4, 5, 13), (2, 10, 13), (8, 10, 13)):
    line = []
    for k in (1, 2, 5, 8, 9, 10, 11, 15, 20, 25, 30):
        got, it, r, m = t.ranks(world, p0, rhs, dx, dy, 1e-300, k, 0, T=T, variant=var)
        line.append("%d:%.1e" % (k, (r - res[k]) / res[k]))
    print(world, T, var, " ".join(line), flush=True)
