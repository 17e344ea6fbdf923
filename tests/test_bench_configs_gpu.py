"""Parity at the sizes and launch geometry bench.py times (BASELINE configs 4
and 5), not only at the small grids of test_sor_gpu.py.

Config 4 (2D Poisson red-black SOR, 32768^2): the timed solve runs passes of
the default T iterations per launch over the automatic block geometry, with
a last pass of steps % T iterations (bench.py --steps 20: T + T + rest).
  * 8192^2 with the block height forced to the one the 32768^2 launch uses,
    k = one pass, two passes and the driver's 20 iterations, bit for bit
    against the restatement of solveRB (assignment-4/src/solver.c:179-238);
  * 32768^2 itself, every cell, and the 8-rank 4 x 2 split of it:
    test_fullfield_gpu.py.
Config 5 (dcavity NS, 16384^2 per GPU): two full time steps with the
pressure solve capped at 20 iterations against the composed red-black NS
oracle: identical iteration counts, p/u/v within 1e-12 relative.
"""
import functools
import os

import numpy as np
import pytest

import ns_gpu_driver as D
import orc
import pymisor as M

pytestmark = pytest.mark.gpu

OMEGA = 1.9


@functools.lru_cache(maxsize=None)
def bench_rows():
    """the block height the library picks for the 32768^2 bench launch
    (misor_api.hip pick_tb_nby)"""
    with M.Grid(32768, 32768, 1.0 / 32768, 1.0 / 32768, OMEGA, 1e-300, 1) as big:
        return big.get_tuning(M.TUNE_TB_ROWS)


@pytest.mark.parametrize("k", ["T", "2T", 20])
def test_benched_geometry_8192(k):
    n = 8192
    p, rhs = orc.poisson_init(n, n)
    with M.Grid(n, n, 1.0 / n, 1.0 / n, OMEGA, 1e-300, 1) as g:
        g.set_tuning(M.TUNE_TB_ROWS, bench_rows())
        T = g.get_tuning(M.TUNE_TSTEPS)
        kk = {"T": T, "2T": 2 * T}.get(k, k)
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb(itermax=kk)
        got = g.download(M.P)
        st = g.stats()
    # one pass: T; 16 / 20 iterations on this 2^26-cell grid: the chained split
    # ring's 10-iteration passes (misor_api.hip configure_tb short_all)
    if k == "T":
        assert st["iters_per_pass"] == T
    else:
        assert (st["iters_per_pass"], st["tb_variant"]) in ((T, 0), (10, 13)), st
    want = p.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / n, 1.0 / n, OMEGA, 1e-300, kk)
    assert it == it_ref == kk
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert abs(res - res_ref) <= 1e-10 * res_ref


def test_ns_dcavity_16384_two_steps(golden):
    """BASELINE config 5 per GPU: a6 dcavity.par read as 2D at 16384^2"""
    prm = orc.read_par(os.path.join(golden, "a6_dcavity.par"))
    prm.update(imax=16384, jmax=16384, itermax=20)
    ns = orc.NS(prm)
    # (the restatement's solveRB on 16 threads: p bit-identical to one thread,
    # test_oracle.py; 20 capped iterations per step, far from eps^2)
    steps_ref, iters_ref, _ = ns.run(solver=2, max_steps=2)
    g = D.ns_grid(prm)
    try:
        steps, iters, _ = D.run(g, prm, max_steps=2)
        assert steps == steps_ref == 2
        assert list(iters) == list(iters_ref)
        for name, fid in (("p", M.P), ("u", M.U), ("v", M.V)):
            got, want = g.download(fid), getattr(ns, name)
            scale = np.abs(want).max()
            assert np.abs(got - want).max() <= 1e-12 * scale, name
    finally:
        g.close()
