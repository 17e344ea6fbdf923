"""Residual lower bounds of the 10-iteration split-ring pass (MISOR_TUNE_RES_LITE;
misor_solve.hip, sor_tbh.h hrs_step LITE, sor_kernels.hip finish_body).

On one rank a pass of 10 iterations counts r^2 of its first nine iterations on
one row in S of its steady chunks: a lower bound of each iteration's residual.
The loop test accepts such a sum only where it proves solveRB's loop goes on
(res >= eps^2, outside the near band, before itermax); otherwise the pass stops
before that iteration, is redone from its source up to there, and the rest of
the solve counts every cell.  So p, the iteration count and res must equal the
restatement of solveRB (assignment-4/src/solver.c:179-238) -- p bit for bit,
res to 1e-12 (the device sums in another order) -- and the same solve with the
bounds off bit for bit, res included: when the bounds decide every iteration,
when one misses near convergence, and when one misses at once (a near band
that takes in every residual).
"""
import threading

import numpy as np
import pytest

import orc
import pymisor as M

pytestmark = pytest.mark.gpu

# tall enough for chained steady blocks of the T = 10 split ring (the strips
# off the physical sides march kSteady chunks)
NI, NJ = 600, 700


def fields(seed, scale=1.0):
    rng = np.random.default_rng(seed)
    p = rng.standard_normal((NJ + 2, NI + 2)) * scale
    rhs = rng.standard_normal((NJ + 2, NI + 2)) * scale
    return p, rhs


def gpu(p, rhs, dx, dy, eps, itermax, lite, band=None):
    with M.Grid(NI, NJ, dx, dy, 1.9, eps, itermax) as g:
        g.set_tuning(M.TUNE_SMALL_SOLVE, 0)
        g.set_tuning(M.TUNE_TB_VARIANT, 13)
        g.set_tuning(M.TUNE_TSTEPS, 10)
        g.set_tuning(M.TUNE_RES_LITE, lite)
        assert g.get_tuning(M.TUNE_RES_LITE) == lite
        if band is not None:
            g.set_tuning(M.TUNE_NEAR_BAND, band)
        g.upload(M.P, p)
        g.upload(M.RHS, rhs)
        it, res = g.solve_rb()
        st = g.stats()
        return it, res, g.download(M.P), st


def oracle(p, rhs, dx, dy, eps, itermax):
    want = p.copy()
    it, res = orc.solve_rb(want, rhs, dx, dy, 1.9, eps, itermax)
    return it, res, want


@pytest.mark.parametrize("pow2", [False, True])
def test_bounds_decide_every_iteration(pow2):
    """eps far below every residual: the bounds prove every inner iteration,
    no miss; 4 passes of 10"""
    dx, dy = (1.0 / 512, 1.0 / 512) if pow2 else (1.0 / NI, 0.8 / NJ)
    p, rhs = fields(3)
    want_it, want_res, want = oracle(p, rhs, dx, dy, 1e-300, 40)
    runs = {}
    for lite in (1, 0):
        it, res, got, st = gpu(p, rhs, dx, dy, 1e-300, 40, lite)
        assert (it, st["iters_per_pass"], st["tb_variant"]) == (want_it, 10, 13)
        assert st["lite_misses"] == 0
        assert abs(res - want_res) <= 1e-12 * want_res
        assert np.array_equal(got, want)
        runs[lite] = res
    assert runs[1] == runs[0]


@pytest.fixture(scope="module")
def converging():
    """a field whose solveRB residual sequence has strict drops (one iteration
    at a time from the same p); eps^2 between the residual of iteration k*
    and the smallest one before it, so solveRB stops at k* -- inside a pass"""
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
            return p0, rhs, dx, dy, ((res[ks] + lo) / 2) ** 0.5, ks
    pytest.skip("no strictly decreasing residual step")


def test_bound_misses_near_convergence(converging):
    """the bound of an iteration just before k* does not clear eps^2: the pass
    is redone from its source and the solve ends at k* exactly"""
    p0, rhs, dx, dy, eps, ks = converging
    want_it, want_res, want = oracle(p0, rhs, dx, dy, eps, 100000)
    assert want_it == ks
    it, res, got, st = gpu(p0, rhs, dx, dy, eps, 100000, 1)
    assert it == ks and abs(res - want_res) <= 1e-12 * want_res
    assert np.array_equal(got, want)
    assert st["lite_misses"] == 1
    it0, res0, got0, st0 = gpu(p0, rhs, dx, dy, eps, 100000, 0)
    assert (it0, res0, st0["lite_misses"]) == (ks, res, 0)
    assert np.array_equal(got0, want)


def test_bound_misses_at_once(converging):
    """a near band of 10^30 takes in every residual: the first bound misses,
    the pass is redone counting every cell, and the exact tail
    (misor_solve.hip exact_tail) runs the solve to k*"""
    p0, rhs, dx, dy, eps, ks = converging
    want_it, want_res, want = oracle(p0, rhs, dx, dy, eps, 100000)
    it, res, got, st = gpu(p0, rhs, dx, dy, eps, 100000, 1, band=-30)
    assert it == want_it and abs(res - want_res) <= 1e-12 * want_res
    assert np.array_equal(got, want)
    assert st["lite_misses"] == 1


def ranks(world, p0, rhs, dx, dy, eps, itermax, lite, band=None, T=10, variant=13):
    """`world` in-process ranks (LOCAL transport, the pipelined decomposed loop
    with its 2T-deep exchanges); the owned blocks assembled into one field"""
    cid = ("LOCAL:lite%d_%d_%s_%g_%d_%d_%d" % (world, lite, band, eps, itermax, T,
                                               variant)).encode()
    outs, errs = [None] * world, []

    def body(r):
        try:
            with M.Grid(NI, NJ, dx, dy, 1.9, eps, itermax, device=0, nranks=world, rank=r,
                        comm_id=cid) as g:
                g.set_tuning(M.TUNE_TB_VARIANT, variant)
                g.set_tuning(M.TUNE_TSTEPS, T)
                g.set_tuning(M.TUNE_RES_LITE, lite)
                if band is not None:
                    g.set_tuning(M.TUNE_NEAR_BAND, band)
                loc = g.loc
                g.upload(M.P, np.ascontiguousarray(
                    p0[loc.joff:loc.joff + loc.nj + 2, loc.ioff:loc.ioff + loc.ni + 2]))
                g.upload(M.RHS, np.ascontiguousarray(
                    rhs[loc.joff:loc.joff + loc.nj + 2, loc.ioff:loc.ioff + loc.ni + 2]))
                it, res = g.solve_rb()
                outs[r] = (loc, g.download(M.P), it, res, g.stats()["lite_misses"])
        except BaseException as e:
            errs.append((r, repr(e)))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
        assert not t.is_alive(), "rank thread hung"
    assert not errs, errs
    got = np.full(p0.shape, np.nan)
    for loc, blk, it, res, _ in outs:
        nb = list(loc.neighbours)
        i0, j0 = (0 if nb[0] < 0 else 1), (0 if nb[2] < 0 else 1)
        i1 = loc.ni + 1 if nb[1] < 0 else loc.ni
        j1 = loc.nj + 1 if nb[3] < 0 else loc.nj
        got[loc.joff + j0:loc.joff + j1 + 1, loc.ioff + i0:loc.ioff + i1 + 1] = \
            blk[j0:j1 + 1, i0:i1 + 1]
    assert len({o[2] for o in outs}) == 1 and len({o[3] for o in outs}) == 1  # ranks agree
    assert len({o[4] for o in outs}) == 1
    return got, outs[0][2], outs[0][3], outs[0][4]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_decomposed_bounds(world, converging):
    """decomposed ranks: the all-reduced sum of the ranks' lower bounds decides
    (sor_kernels.hip rb_decide_kernel); far from eps every bound holds and the
    bits equal the bounds switched off; near convergence one misses and the
    solve still ends at k* with p bit for bit"""
    dx, dy = 1.0 / NI, 0.8 / NJ
    p, rhs = fields(5)
    want = p.copy()
    it_w, res_w = orc.solve_rb(want, rhs, dx, dy, 1.9, 1e-300, 30)
    runs = {}
    for lite in (1, 0):
        got, it, res, misses = ranks(world, p, rhs, dx, dy, 1e-300, 30, lite)
        assert (it, misses) == (it_w, 0)
        assert abs(res - res_w) <= 1e-12 * res_w
        assert np.array_equal(got, want)
        runs[lite] = res
    assert runs[1] == runs[0]
    p0, rhs0, dx0, dy0, eps, ks = converging
    want0 = p0.copy()
    it_r, res_r = orc.solve_rb(want0, rhs0, dx0, dy0, 1.9, eps, 100000)
    got, it, res, misses = ranks(world, p0, rhs0, dx0, dy0, eps, 100000, 1)
    assert (it, misses) == (ks, 1) and it_r == ks
    assert abs(res - res_r) <= 1e-12 * res_r
    assert np.array_equal(got, want0)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("band", [None, 400])
def test_decomposed_inner_stage_residual(converging, world, band):
    """a converging solve that stops at a leading stage (t < T/2, one row
    ahead in the skewed march) of a 10-iteration pass: res of that iteration
    to 1e-12 of the restatement's on every split, y-splits included (their
    top blocks read one halo row more: the 2T + 1-deep exchange)"""
    p0, rhs0, dx0, dy0, eps, ks = converging
    want0 = p0.copy()
    it_r, res_r = orc.solve_rb(want0, rhs0, dx0, dy0, 1.9, eps, 100000)
    got, it, res, misses = ranks(world, p0, rhs0, dx0, dy0, eps, 100000, 0, band=band)
    assert it == it_r == ks and np.array_equal(got, want0)
    assert abs(res - res_r) <= 1e-12 * res_r


def test_decomposed_leading_stage_near_eps():
    """eps^2 within 5e-7 of a leading stage's residual on 4 ranks: the solve
    stops exactly there (before the 2T + 1-deep exchange it ran one iteration
    on: the top rows of the leading stages' residual read a stale halo row)"""
    dx, dy = 1.0 / NI, 1.0 / NJ
    rng = np.random.default_rng(7)
    p0 = rng.standard_normal((NJ + 2, NI + 2)) * 2.0 ** -30
    rhs = np.zeros_like(p0)
    q, res = p0.copy(), {}
    for k in range(1, 47):
        res[k] = orc.solve_rb(q, rhs, dx, dy, 1.9, 1e-300, 1)[1]
    for k in (41, 43, 45):  # stages 0, 2, 4 of the fifth pass
        lo = min(res[j] for j in range(1, k))
        if not res[k] * (1 + 5e-7) < lo:
            continue
        eps = (res[k] * (1 + 5e-7)) ** 0.5
        got, it, r, _ = ranks(4, p0, rhs, dx, dy, eps, 100000, 0, band=400)
        assert it == k, (k, it)
        assert abs(r - res[k]) <= 1e-12 * res[k]


def test_bad_setting_refused():
    with M.Grid(300, 190, 1.0 / 300, 1.0 / 190, 1.7, 1e-300, 10) as g:
        with pytest.raises(M.MisorError):
            g.set_tuning(M.TUNE_RES_LITE, 2)
        assert g.get_tuning(M.TUNE_RES_LITE) == 1
