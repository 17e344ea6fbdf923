"""Decomposed res on the converging field (diagnostic, GPU box)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "practical-parallel-algorithms-with-mpi_amd")
import orc
import test_res_lite_gpu as t

NI, NJ = t.NI, t.NJ
dx, dy = 1.0 / NI, 1.0 / NJ
rng = np.random.default_rng(7)
p0 = rng.standard_normal((NJ + 2, NI + 2)) * 2.0 ** -30
rhs = np.zeros_like(p0)
q, res = p0.copy(), {}
for k in range(1, 50):
    res[k] = orc.solve_rb(q, rhs, dx, dy, 1.9, 1e-300, 1)[1]
lo = min(res[k] for k in range(1, 45))
eps = ((res[45] + lo) / 2) ** 0.5
for world, T, var in ((4, 10, 13), (4, 8, 0), (2, 10, 13), (1, 10, 13)):
    line = []
    for k in (1, 10, 20, 40, 44, 45):
        got, it, r, m = t.ranks(world, p0, rhs, dx, dy, 1e-300, k, 0, T=T, variant=var)
        line.append("%d:%.1e" % (k, (r - res[k]) / res[k]))
    got, it, r, m = t.ranks(world, p0, rhs, dx, dy, eps, 100000, 0, T=T, variant=var)
    line.append("conv it %d: %.1e" % (it, (r - res[45]) / res[45]))
    got, it, r, m = t.ranks(world, p0, rhs, dx, dy, eps, 100000, 0, band=400, T=T, variant=var)
    line.append("conv noband it %d: %.1e" % (it, (r - res[45]) / res[45]))
    print(world, T, var, " ".join(line), flush=True)
