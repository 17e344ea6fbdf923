"""Decomposed res of converging solves stopping at each stage of a 10-iteration pass (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "practical-parallel-algorithms-with-mpi_amd")
import orc
import test_res_lite_gpu as t

dx, dy = 1.0 / t.NI, 1.0 / t.NJ
for seed, scale, zero_rhs in ((7, 2.0 ** -30, True), (3, 1.0, False)):
    rng = np.random.default_rng(seed)
    p0 = rng.standard_normal((t.NJ + 2, t.NI + 2)) * scale
    rhs = np.zeros_like(p0) if zero_rhs else rng.standard_normal((t.NJ + 2, t.NI + 2))
    q, res = p0.copy(), {}
    for k in range(1, 62):
        res[k] = orc.solve_rb(q, rhs, dx, dy, 1.9, 1e-300, 1)[1]
    for world in (4, 2):
        line = []
        for k in range(41, 61):
            # eps^2 just above res[k] and below every earlier residual: stops at k
            lo = min(res[j] for j in range(1, k))
            if not res[k] < lo:
                continue
            eps = ((res[k] + min(lo, res[k] * (1 + 1e-6))) / 2) ** 0.5
            got, it, r, m = t.ranks(world, p0, rhs, dx, dy, eps, 100000, 0, band=400)
            line.append("%d:%s%.0e" % (k, "" if it == k else "it%d!" % it, abs(r - res[k]) / res[k]))
        print(seed, world, " ".join(line), flush=True)
