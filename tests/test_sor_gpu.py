"""Parity of the HIP red-black SOR (libmisor, through its C ABI) with the
reference's solveRB (assignment-4/src/solver.c:179-238).

Bar: bit-exact p (the per-cell arithmetic follows the reference expression
order with no FMA contraction) and identical iteration counts.  Only the
residual's summation order differs, so res is compared with rel 1e-12.
"""
import json
import os

import numpy as np
import pytest

import orc
import pymisor as M

pytestmark = pytest.mark.gpu

OMEGA, EPS = 1.9, 1e-6


def set_mode(g, small):
    """small = 1: whole-solve LDS kernel where the grid fits; 0: the
    multi-block path with the default iterations per pass; "tN": the
    multi-block path with N iterations per pass (1: single-iteration sweep
    kernel, 2..8: temporally blocked kernel, 9..: its split-ring variant 13,
    the only one that runs more than 8); "hN": the split-ring variant 13 (its
    chained passes, sor_tbh.h rb_tbhc_kernel) at any N.  All must match the
    reference."""
    if isinstance(small, str):
        T = int(small[1:])
        g.set_tuning(M.TUNE_SMALL_SOLVE, 0)
        g.set_tuning(M.TUNE_TB_VARIANT, HRS if small[0] == "h" or T > 8 else 0)
        g.set_tuning(M.TUNE_TSTEPS, T)
    else:
        g.set_tuning(M.TUNE_SMALL_SOLVE, small)
    return g


def make_grid(ni, nj, xl=1.0, yl=1.0, omega=OMEGA, eps=EPS, itermax=1000000,
              variant=M.SOLVE_RB, small=1):
    g = M.Grid(ni, nj, xl / ni, yl / nj, omega, eps, itermax, variant=variant)
    return set_mode(g, small)


HRS = 13  # TB variant: the skewed split ring (sor_tbh.h)
TS = ["t%d" % t for t in range(1, 11)] + ["h2", "h5", "h8"]
PATHS = pytest.mark.parametrize("small", [1] + TS, ids=["lds"] + TS)


def test_poisson_init_bitwise():
    for (ni, nj, xl, yl) in ((100, 100, 1.0, 1.0), (37, 23, 1.0, 2.0), (700, 5, 3.0, 0.5)):
        with make_grid(ni, nj, xl, yl) as g:
            g.poisson_init(xl, yl, 2)
            p, rhs = orc.poisson_init(ni, nj, xl, yl, 2)
            assert np.array_equal(g.download(M.P), p)
            assert np.array_equal(g.download(M.RHS), rhs)
            g.poisson_init(xl, yl, 1)
            assert not g.download(M.RHS).any()


@PATHS
def test_sweep_fixtures(golden, small):
    z = np.load(os.path.join(golden, "rb_sweeps.npz"))
    for key in z.files:
        if not key.startswith("geom_"):
            continue
        ni, nj, xl, yl = z[key]
        ni, nj = int(ni), int(nj)
        for k in (1, 2, 7):
            with make_grid(ni, nj, xl, yl, eps=1e-300, small=small) as g:
                g.poisson_init(xl, yl, 2)
                it, res = g.solve_rb(itermax=k)
                assert it == k
                got = g.download(M.P)
                want = z["p_%dx%d_k%d" % (ni, nj, k)]
                assert np.array_equal(got, want), (ni, nj, k, np.abs(got - want).max())


@PATHS
def test_poisson_par_converges_like_reference(golden, small):
    z = np.load(os.path.join(golden, "rb_poisson100.npz"))
    with make_grid(100, 100, small=small) as g:
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb()
        assert it == int(z["iterations"]) == 2388
        assert np.array_equal(g.download(M.P), z["p"])
        assert res < EPS * EPS


@PATHS
def test_iteration_kats(golden, small):
    kat = json.load(open(os.path.join(golden, "rb_kat.json")))["iterations"]
    for key, want in kat.items():
        if "x" in key:
            ni, nj = map(int, key.split("x"))
        else:
            ni = nj = int(key)
        if ni * nj > 130 * 130:
            continue  # 200^2 takes 8.7k sweeps; covered by the CPU KAT test
        with make_grid(ni, nj, small=small) as g:
            g.poisson_init(1.0, 1.0, 2)
            it, _ = g.solve_rb()
            assert it == want, (key, it, want)


@PATHS
def test_rba_variant(small):
    ni, nj = 64, 48
    p, rhs = orc.poisson_init(ni, nj)
    it_ref, res_ref = orc.solve_rb(p, rhs, 1.0 / ni, 1.0 / nj, OMEGA, EPS, 100000, "rba")
    with make_grid(ni, nj, variant=M.SOLVE_RBA, small=small) as g:
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb()
        assert it == it_ref
        assert np.array_equal(g.download(M.P), p)
        assert abs(res - res_ref) <= 1e-12 * res_ref


@pytest.mark.parametrize("ni,nj,k", [(3, 2, 5), (2, 7, 4), (127, 129, 3), (128, 128, 3),
                                     (129, 33, 4), (255, 17, 2), (256, 300, 3),
                                     (511, 40, 3), (512, 65, 2), (513, 513, 3),
                                     (1000, 777, 2), (2049, 130, 2), (120, 9, 7),
                                     (121, 300, 5), (240, 241, 6), (112, 113, 9),
                                     (1001, 1537, 8)])
@PATHS
def test_random_fields_vs_oracle(ni, nj, k, small):
    rng = np.random.default_rng(ni * 7919 + nj)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    dx, dy = 1.3 / ni, 0.7 / nj
    want = p.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, dx, dy, 1.7, 1e-300, k)
    with M.Grid(ni, nj, dx, dy, 1.7, 1e-300, k) as g:
        set_mode(g, small)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        it, res = g.solve_rb()
        got = g.download(M.P)
    assert it == it_ref == k
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert abs(res - res_ref) <= 1e-12 * abs(res_ref)


@PATHS
def test_consecutive_solves_track_buffers(small):
    """odd + even + odd iteration counts: the ping-pong buffer bookkeeping"""
    ni, nj = 97, 61
    rng = np.random.default_rng(5)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    want = p.copy()
    with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.5, 1e-300, 10) as g:
        set_mode(g, small)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        for k in (3, 4, 1, 6):
            g.solve_rb(itermax=k)
            orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.5, 1e-300, k)
            assert np.array_equal(g.download(M.P), want), k


def test_zero_iterations():
    with make_grid(10, 10, itermax=0) as g:
        g.poisson_init(1.0, 1.0, 2)
        p0 = g.download(M.P)
        it, res = g.solve_rb()
        assert (it, res) == (0, 1.0)
        assert np.array_equal(g.download(M.P), p0)
    with make_grid(10, 10, eps=2.0) as g:  # eps^2 > res0 = 1: loop never entered
        assert g.solve_rb() == (0, 1.0)


@pytest.mark.parametrize("finish2", [1, 0])
@pytest.mark.parametrize("k", [2, 3])
def test_large_grid_few_sweeps(k, finish2):
    """8192^2 (67M cells, 0.54 GB per field): bit-exact after 2 and 3 sweeps
    (default path: temporally blocked; a capped solve's passes run only the
    iterations left, so these are single passes of T' = 2 and 3), with the
    single-rank loop test in two levels (MISOR_TUNE_FINISH2 = 1, default) and
    in one kernel (0): same p, same iteration count"""
    n = 8192
    p, rhs = orc.poisson_init(n, n)
    want = p.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / n, 1.0 / n, OMEGA, 1e-300, k)
    with make_grid(n, n, eps=1e-300, itermax=k) as g:
        g.set_tuning(M.TUNE_FINISH2, finish2)
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb()
        got = g.download(M.P)
    assert it == k
    assert np.array_equal(got, want)
    # res sums 6.7e7 squares: the oracle left to right, the device in a tree,
    # so only the rounding of the sum differs (p itself is bit-exact)
    assert abs(res - res_ref) <= 1e-10 * res_ref


@pytest.mark.parametrize("T", range(2, 11))
@pytest.mark.parametrize("variant", [0, 2, HRS])
def test_tb_converges_mid_pass(T, variant):
    """convergence inside a temporally blocked pass: the pass is recomputed
    with fewer iterations, so the count and p equal solveRB's for every T"""
    ni, nj = 300, 190
    p, rhs = orc.poisson_init(ni, nj)
    want = p.copy()
    eps = 3e-3
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, OMEGA, eps, 100000)
    if T > 8 and variant != HRS:  # the register-ring kernels run T <= 8
        with make_grid(ni, nj, small="t8") as g:
            g.set_tuning(M.TUNE_TB_VARIANT, variant)
            with pytest.raises(M.MisorError):
                g.set_tuning(M.TUNE_TSTEPS, T)
        return
    with make_grid(ni, nj, eps=eps, small="t%d" % T) as g:
        g.set_tuning(M.TUNE_TB_VARIANT, variant)  # strips per workgroup, rows in flight
        g.set_tuning(M.TUNE_TSTEPS, T)
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb()
        got = g.download(M.P)
        st = g.stats()
    assert st["iters_per_pass"] == T
    assert it == it_ref
    assert np.array_equal(got, want)
    assert abs(res - res_ref) <= 1e-12 * res_ref


@pytest.mark.parametrize("variant", [-1, 2], ids=["v0", "v2"])
@pytest.mark.parametrize("T", [2, 5, 8])
@pytest.mark.parametrize("ni,nj", [(1024, 1024), (1000, 1537), (2050, 300)])
def test_pow2_spacing_vs_oracle(ni, nj, T, variant):
    """dx == dy == 2^-10: the TB kernel computes r with one fma in place of
    two multiplies, an add and a subtract (sor_tb.h resid<true>); bit for bit
    the reference's expression, on random fields of a wide dynamic range; the
    default kernel and the 2-strip workgroup variant (the general form runs on
    every other spacing of the suite)"""
    rng = np.random.default_rng(ni + 7 * nj + T)
    p = rng.standard_normal((nj + 2, ni + 2)) * np.exp(rng.uniform(-20, 20, (nj + 2, ni + 2)))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 1e6
    h = 2.0 ** -10
    k = 2 * T + 1
    want = p.copy()
    orc.solve_rb(want, rhs, h, h, 1.7, 1e-300, k)
    with M.Grid(ni, nj, h, h, 1.7, 1e-300, k) as g:
        set_mode(g, "t%d" % T)
        if variant >= 0:
            g.set_tuning(M.TUNE_TB_VARIANT, variant)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        it, _ = g.solve_rb()
        got = g.download(M.P)
    assert it == k
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
