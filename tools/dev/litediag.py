"""Decomposed residual lower bounds near convergence (diagnostic, GPU box)."""
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
for k in range(1, 90):
    res[k] = orc.solve_rb(q, rhs, dx, dy, 1.9, 1e-300, 1)[1]
for ks in range(45, 90):
    lo = min(res[k] for k in range(1, ks))
    if res[ks] < lo * (1 - 1e-6) and ks % 10 not in (0, 1):
        break
eps = ((res[ks] + lo) / 2) ** 0.5
want = p0.copy()
it_r, res_r = orc.solve_rb(want, rhs, dx, dy, 1.9, eps, 100000)
print("ks", ks, "oracle", it_r, res_r, "res[ks-1..ks+1]", res[ks - 1], res[ks], res.get(ks + 1))
for world in (1, 2, 4):
    for lite in (0, 1):
        if world == 1:
            it, r, got, st = t.gpu(p0, rhs, dx, dy, eps, 100000, lite)
            m = st["lite_misses"]
        else:
            got, it, r, m = t.ranks(world, p0, rhs, dx, dy, eps, 100000, lite)
        bad = np.argwhere(got != want)
        print(world, lite, "it", it, "res %.10e rel %.2e" % (r, (r - res_r) / res_r), "misses", m,
              "p bad", len(bad), bad[:3].tolist(), flush=True)
