"""Which geometry makes the decomposed skewed split ring's leading stages miscount (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "practical-parallel-algorithms-with-mpi_amd")
import orc
import test_res_lite_gpu as t

for ni, nj, world in ((600, 700, 4), (600, 720, 4), (600, 712, 4), (300, 700, 2), (600, 350, 2),
                      (600, 1400, 8)):
    t.NI, t.NJ = ni, nj
    dx, dy = 1.0 / ni, 1.0 / nj
    rng = np.random.default_rng(7)
    p0 = rng.standard_normal((nj + 2, ni + 2)) * 2.0 ** -30
    rhs = np.zeros_like(p0)
    q, res = p0.copy(), {}
    for k in range(1, 52):
        res[k] = orc.solve_rb(q, rhs, dx, dy, 1.9, 1e-300, 1)[1]
    line = []
    for k in range(41, 51):
        lo = min(res[j] for j in range(1, k))
        if not res[k] < lo:
            line.append("%d:-" % k)
            continue
        eps = ((res[k] + lo) / 2) ** 0.5
        got, it, r, m = t.ranks(world, p0, rhs, dx, dy, eps, 100000, 0, band=400)
        line.append("%d:%s" % (k, "ok" if it == k else "it%d" % it))
    print(ni, nj, world, " ".join(line), flush=True)
