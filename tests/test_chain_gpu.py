"""Chained temporally blocked passes (sor_tb.h rb_tbc_kernel): vertical runs
of short blocks with work stealing, against the reference's solveRB
(assignment-4/src/solver.c:179-238, oracle orc.solve_rb).

Which workgroup runs which block -- and how the runs are split by steals --
changes from launch to launch, but every block is computed with the same
arithmetic and its residual partial goes to a fixed slot: p must be bit for
bit the reference's, and res identical from run to run.
"""
import numpy as np
import pytest

import orc
import pymisor as M

pytestmark = pytest.mark.gpu


def run(p, rhs, dx, dy, k, T, chain=1, rows=0, omega=1.7, eps=1e-300, pow2=None, ranks=None):
    ni, nj = p.shape[1] - 2, p.shape[0] - 2
    with M.Grid(ni, nj, dx, dy, omega, eps, k) as g:
        g.set_tuning(M.TUNE_SMALL_SOLVE, 0)
        g.set_tuning(M.TUNE_TB_CHAIN, chain)
        g.set_tuning(M.TUNE_TSTEPS, T)
        if rows:
            g.set_tuning(M.TUNE_TB_ROWS, rows)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        it, res = g.solve_rb()
        return it, res, g.download(M.P), g.get_tuning(M.TUNE_TB_ROWS)


@pytest.mark.parametrize("T", [2, 3, 5, 7, 8])
@pytest.mark.parametrize("ni,nj,rows", [(1000, 777, 0), (2049, 1300, 0), (300, 4000, 36),
                                        (130, 2500, 0), (4000, 260, 0), (777, 1500, 60)])
def test_chain_vs_oracle(ni, nj, rows, T):
    """one pass, two passes and a ragged rest; tall narrow grids (few
    columns: most workgroups start by stealing), wide short ones (one or two
    steady block rows), explicit block heights"""
    rng = np.random.default_rng(ni * 131 + nj + T)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    dx, dy = 1.3 / ni, 0.7 / nj
    for k in (T, 2 * T + 1):
        want = p.copy()
        it_ref, res_ref = orc.solve_rb(want, rhs, dx, dy, 1.7, 1e-300, k)
        it, res, got, h = run(p, rhs, dx, dy, k, T, rows=rows)
        assert it == it_ref == k
        assert np.array_equal(got, want), (k, np.argwhere(got != want)[:5])
        assert abs(res - res_ref) <= 1e-12 * abs(res_ref)
        if rows:
            assert h % (2 * T + 2) == 0  # a multiple of the ring (D = 2)


@pytest.mark.parametrize("T", [4, 8])
def test_chain_res_deterministic_and_equal_to_unchained(T):
    """several launches (different steals): identical res bits; the unchained
    persistent pass (MISOR_TUNE_TB_CHAIN = 0) gives the same p"""
    ni, nj = 3000, 2900
    rng = np.random.default_rng(T)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    h = 1.0 / 1024
    outs = [run(p, rhs, h, h, 3 * T, T) for _ in range(3)]
    for it, res, got, _ in outs[1:]:
        assert it == outs[0][0]
        assert res == outs[0][1]
        assert np.array_equal(got, outs[0][2])
    it, res, got, _ = run(p, rhs, h, h, 3 * T, T, chain=0)
    assert it == outs[0][0]
    assert np.array_equal(got, outs[0][2])
    assert abs(res - outs[0][1]) <= 1e-12 * abs(res)


@pytest.mark.parametrize("T", [2, 7, 8])
def test_chain_converges_mid_pass(T):
    """convergence inside a chained pass: eps is put between the residual of
    iteration ks (not a multiple of T) and the smallest one before it (the
    oracle's residual sequence), so solveRB stops at ks, inside a pass; the
    pass is recomputed with fewer iterations, and count and p are solveRB's"""
    ni, nj = 260, 1100
    rng = np.random.default_rng(T + 11)
    # scaled so every residual is < 1 (solveRB's loop starts from res = 1.0)
    p0 = rng.standard_normal((nj + 2, ni + 2)) * 2.0 ** -30
    rhs = np.zeros_like(p0)
    res = {}
    q = p0.copy()
    for k in range(1, 40):  # one iteration at a time: res[k] after k iterations
        res[k] = orc.solve_rb(q, rhs, 1.0 / ni, 1.0 / nj, 1.9, 1e-300, 1)[1]
    for ks in range(2 * T + 1, 40):
        lo = min(res[k] for k in range(1, ks))
        if res[ks] < lo * (1 - 1e-6) and ks % T:
            break
    else:
        pytest.skip("no strictly decreasing residual step in range")
    eps = ((res[ks] + lo) / 2) ** 0.5
    want = p0.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.9, eps, 100000)
    assert it_ref == ks
    it, r, got, _ = run(p0, rhs, 1.0 / ni, 1.0 / nj, 100000, T, omega=1.9, eps=eps, rows=36)
    assert it == it_ref
    assert np.array_equal(got, want)
    assert abs(r - res_ref) <= 1e-12 * res_ref


def test_chain_block_heights():
    """chained blocks of 1, 2 and 9 ring lengths (an explicit MISOR_TUNE_TB_ROWS)"""
    ni, nj = 1500, 1111
    rng = np.random.default_rng(9)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    want = p.copy()
    orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 17)
    for rings in (1, 2, 9):
        it, _, got, h = run(p, rhs, 1.0 / ni, 1.0 / nj, 17, 8, rows=rings * 18)
        assert h == rings * 18
        assert np.array_equal(got, want), rings
