"""The exchange variant of the temporally blocked sweep (TB variants 6 and 7:
sor_tbx.h rb_tbx_kernel -- the strips of a workgroup hand each other their
edge columns through LDS, rhs ring in LDS) against the restatement of
solveRB (assignment-4/src/solver.c:179-238): p bit for bit, identical
iteration counts, res to 1e-12.

Geometry is chosen so that every path runs: interior blocks (static ring
chunks with the warm-up of whole chunks), the general march (physical sides,
ragged last block rows), physical right ghost columns at every position
relative to the strips -- including the first column of a strip, where the
ghost rule of the header applies -- and decomposed ranks.
"""
import threading

import numpy as np
import pytest

import orc
import pymisor as M

pytestmark = pytest.mark.gpu

XCH = 6      # 4 strips per workgroup
XCH8 = 7     # 8 strips per workgroup


def solve(p, rhs, dx, dy, k, T, variant=XCH, rows=0, omega=1.7, eps=1e-300, itermax=None):
    nj, ni = p.shape[0] - 2, p.shape[1] - 2
    with M.Grid(ni, nj, dx, dy, omega, eps, itermax or k) as g:
        g.set_tuning(M.TUNE_SMALL_SOLVE, 0)
        g.set_tuning(M.TUNE_TB_VARIANT, variant)
        g.set_tuning(M.TUNE_TSTEPS, T)
        if rows:
            g.set_tuning(M.TUNE_TB_ROWS, rows)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        it, res = g.solve_rb() if itermax else g.solve_rb(itermax=k)
        assert g.get_tuning(M.TUNE_TB_VARIANT) == variant
        st = g.stats()
        return it, res, g.download(M.P), st


def fields(ni, nj, seed):
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 10
    return p, rhs


@pytest.mark.parametrize("T,variant", [(t, XCH) for t in range(1, 11)] +
                         [(t, XCH8) for t in (2, 5, 8, 10)])
@pytest.mark.parametrize("ni,nj", [(1201, 700), (2000, 1033), (1826, 600), (300, 190)])
def test_xch_random_vs_oracle(ni, nj, T, variant):
    p, rhs = fields(ni, nj, ni + 7 * nj + T)
    dx, dy = 1.1 / ni, 0.9 / nj
    S = max(2, 2 * T - 2)
    for k in (T, 2 * T + 1):
        want = p.copy()
        it_ref, res_ref = orc.solve_rb(want, rhs, dx, dy, 1.7, 1e-300, k)
        # block rows of 4 ring lengths: interior blocks and several block rows
        it, res, got, st = solve(p, rhs, dx, dy, k, T, variant, rows=4 * S)
        assert st["iters_per_pass"] == T
        assert it == it_ref == k
        assert np.array_equal(got, want), (k, np.argwhere(got != want)[:5])
        assert abs(res - res_ref) <= 1e-12 * res_ref


@pytest.mark.parametrize("T", [4, 8, 10])
def test_xch_right_ghost_at_every_strip_position(T):
    """physical right side: column ni+1 as the first column of strip w of the
    last workgroup (w = 1 .. 3), and one column either side of it"""
    owg = 128 * 4 - 4 * T
    nj = 90
    for w in (1, 2, 3):
        cL = 1 + owg - 2 * T           # the second block column's first loaded column
        base = cL + 128 * w - 1        # ni + 1 = cL + 128 w
        for ni in (base - 1, base, base + 1):
            p, rhs = fields(ni, nj, ni * 3 + T)
            dx, dy = 1.0 / ni, 1.3 / nj
            k = 2 * T + 3
            want = p.copy()
            orc.solve_rb(want, rhs, dx, dy, 1.8, 1e-300, k)
            it, _, got, _ = solve(p, rhs, dx, dy, k, T, XCH, rows=2 * max(2, 2 * T - 2),
                                  omega=1.8)
            assert it == k
            assert np.array_equal(got, want), (ni, w, np.argwhere(got != want)[:5])


@pytest.fixture(scope="module")
def mid_pass_case():
    """a field whose solveRB residual sequence has strict drops: eps is put
    between the residual of iteration k* and the smallest one before it, so
    solveRB stops at k* (test_sor_gpu.py test_quad_converges_mid_pass_interior)"""
    ni, nj = 1000, 150
    rng = np.random.default_rng(5)
    # scaled so every residual is < 1 (solveRB's loop starts from res = 1.0)
    p0 = rng.standard_normal((nj + 2, ni + 2)) * 2.0 ** -30
    rhs = np.zeros_like(p0)
    res = {}
    for k in range(1, 80):
        q = p0.copy()
        res[k] = orc.solve_rb(q, rhs, 1.0 / ni, 1.0 / nj, 1.9, 1e-300, k)[1]
    return ni, nj, p0, rhs, res


@pytest.mark.parametrize("T", range(2, 11))
def test_xch_converges_mid_pass(T, mid_pass_case):
    """convergence inside a pass: the pass is recomputed with fewer
    iterations, so the count and p equal solveRB's"""
    ni, nj, p0, rhs, res = mid_pass_case
    for ks in range(25, 80):
        lo = min(res[k] for k in range(1, ks))
        if res[ks] < lo * (1 - 1e-6) and ks % T:
            break
    else:
        pytest.skip("no strictly decreasing residual step in range")
    eps = ((res[ks] + lo) / 2) ** 0.5
    want = p0.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.9, eps, 100000)
    assert it_ref == ks
    it, r, got, st = solve(p0, rhs, 1.0 / ni, 1.0 / nj, 0, T, XCH, omega=1.9, eps=eps,
                           itermax=100000)
    assert st["iters_per_pass"] == T
    assert it == it_ref
    assert np.array_equal(got, want)
    assert abs(r - res_ref) <= 1e-12 * res_ref


@pytest.mark.parametrize("T", [2, 7, 10])
@pytest.mark.parametrize("ni,nj", [(1024, 1024), (2050, 300)])
def test_xch_pow2_spacing(ni, nj, T, monkeypatch):
    """dx == dy == 2^-10: the power-of-two form of r (sor_tb.h resid<true>)
    on fields of a wide dynamic range, and the general form"""
    rng = np.random.default_rng(ni + 7 * nj + T)
    p = rng.standard_normal((nj + 2, ni + 2)) * np.exp(rng.uniform(-20, 20, (nj + 2, ni + 2)))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 1e6
    h = 2.0 ** -10
    k = 2 * T + 1
    want = p.copy()
    orc.solve_rb(want, rhs, h, h, 1.7, 1e-300, k)
    for no in ("0", "1"):
        monkeypatch.setenv("MISOR_NO_POW2", no)
        it, _, got, _ = solve(p, rhs, h, h, k, T, XCH)
        assert it == k
        assert np.array_equal(got, want), (no, np.argwhere(got != want)[:5])


def test_xch_default_geometry_large():
    """8192^2, the automatic block height, T = 10, the bench's problem 2
    fields: one pass and a 20-iteration solve (two passes)"""
    n = 8192
    p, rhs = orc.poisson_init(n, n)
    for k in (10, 20):
        want = p.copy()
        it_ref, res_ref = orc.solve_rb_mt(want, rhs, 1.0 / n, 1.0 / n, 1.9, 1e-300, k, 16)
        it, res, got, st = solve(p, rhs, 1.0 / n, 1.0 / n, k, 10, XCH, omega=1.9)
        assert st["iters_per_pass"] == 10
        assert it == k
        assert np.array_equal(got, want)
        assert abs(res - res_ref) <= 1e-12 * res_ref


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("T", [3, 10])
def test_xch_decomposed(world, T):
    """in-process ranks (LOCAL transport): neighbour sides are interior
    columns / rows of the exchange kernel, fed by the 2T-deep halo"""
    ni, nj, k = 2100, 900, 2 * T + 1
    p, rhs = fields(ni, nj, world * 100 + T)
    dx, dy = 1.1 / ni, 0.8 / nj
    want = p.copy()
    orc.solve_rb(want, rhs, dx, dy, 1.85, 1e-300, k)
    cid = ("LOCAL:xch%d_%d" % (world, T)).encode()
    outs, errs = [None] * world, []

    def body(r):
        try:
            with M.Grid(ni, nj, dx, dy, 1.85, 1e-300, k, device=0, nranks=world, rank=r,
                        comm_id=cid) as g:
                g.set_tuning(M.TUNE_TB_VARIANT, XCH)
                g.set_tuning(M.TUNE_TSTEPS, T)
                loc = g.loc
                g.upload(M.P, np.ascontiguousarray(
                    p[loc.joff:loc.joff + loc.nj + 2, loc.ioff:loc.ioff + loc.ni + 2]))
                g.upload(M.RHS, np.ascontiguousarray(
                    rhs[loc.joff:loc.joff + loc.nj + 2, loc.ioff:loc.ioff + loc.ni + 2]))
                it, _ = g.solve_rb()
                outs[r] = (loc, g.download(M.P), it)
        except BaseException as e:
            errs.append((r, repr(e)))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
        assert not t.is_alive(), "rank thread hung"
    assert not errs, errs
    got = np.full(p.shape, np.nan)
    for loc, blk, it in outs:
        assert it == k
        nb = list(loc.neighbours)
        i0, j0 = (0 if nb[0] < 0 else 1), (0 if nb[2] < 0 else 1)
        i1 = loc.ni + 1 if nb[1] < 0 else loc.ni
        j1 = loc.nj + 1 if nb[3] < 0 else loc.nj
        got[loc.joff + j0:loc.joff + j1 + 1, loc.ioff + i0:loc.ioff + i1 + 1] = \
            blk[j0:j1 + 1, i0:i1 + 1]
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
