"""The 3D path (libmisor misor3_*: assignment-6/src/solver.c on the GPU)
against the 3D oracle (oracle/oracle3d.c, pinned bit for bit to the
reference's own 3D build by tests/test_oracle3d.py) and against the committed
reference fixtures (tests/golden/ns3d_*.npz, made by libref3d.so).

Every step function is compared bit for bit on random states; the solve is
bit-exact in p and its iteration count; the residual differs only in the
order its sum is taken (a fixed tree instead of the reference's sequential
sum), so it is checked to rtol 1e-12.
"""
import os
import zlib

import numpy as np
import pytest

import orc3
import pymisor as M

pytestmark = pytest.mark.gpu

STEP_FNS = {  # pymisor name -> oracle name
    "set_boundary_conditions": "set_bc",
    "set_special_boundary_condition": "set_special_bc",
    "compute_fg": "compute_fg",
    "compute_rhs": "compute_rhs",
    "adapt_uvw": "adapt_uvw",
    "normalize_pressure": "normalize_pressure",
}
GPU_FIELD = {"p": M.P3, "rhs": M.RHS3, "u": M.U3, "v": M.V3, "w": M.W3, "f": M.F3,
             "g": M.G3, "h": M.H3}
BCS = [(1, 1, 1, 1, 1, 1), (2, 3, 1, 2, 3, 1), (3, 3, 2, 2, 1, 3), (1, 2, 3, 1, 2, 3),
       (4, 4, 1, 1, 4, 2)]
BC_KEYS = ("bcLeft", "bcRight", "bcBottom", "bcTop", "bcFront", "bcBack")


def params(golden, name, **over):
    prm = orc3.read_par3(os.path.join(golden, name))
    prm.update(over)
    return prm


def random_state(shape, seed):
    rng = np.random.default_rng(seed)
    st = {n: rng.standard_normal(shape) for n in orc3.FIELDS}
    st["u"] *= 2.0
    return st


# 3D solve variants (sweep, rows, kchunk[, fold[, rhs_ahead]]): the fused
# k-march sweep with the default and odd geometries (chunk boundaries inside
# the grid), the loop test folded into the next sweep (default, single rank)
# or a finish kernel after every sweep, rhs loaded one or two plane steps
# ahead (default: by march length), and the two colour-pass form
# (sweep, rows, kchunk[, fold[, rhs_ahead[, resident]]]); resident 0 unless given
SOLVE_TUNES = [(1, 8, 0), (1, 4, 4), (1, 12, 5), (1, 8, 3 + 4), (1, 8, 0, 0), (1, 4, 4, 0),
               (1, 12, 5, 0), (1, 8, 0, 0, 2), (1, 4, 4, 1, 2), (1, 12, 5, 0, 2), (1, 8, 3 + 4, 0, 2), (1, 8, 16, 0, 1),
               (0, 8, 0), (1, 8, 0, 1, 0, 1)]


def set_tune(g, tune):
    g.set_tuning(M.TUNE3_SWEEP, tune[0])
    g.set_tuning(M.TUNE3_ROWS, tune[1])
    g.set_tuning(M.TUNE3_KCHUNK, tune[2])
    if len(tune) > 3:
        g.set_tuning(M.TUNE3_FOLD, tune[3])
    if len(tune) > 4:
        g.set_tuning(M.TUNE3_RHS_AHEAD, tune[4])
    g.set_tuning(M.TUNE3_RESIDENT, tune[5] if len(tune) > 5 else 0)
    if len(tune) > 5 and tune[5]:
        assert g.get_tuning(M.TUNE3_RESIDENT) == 1  # the grid fits: the resident solve runs


def pair(prm, st, dt, tune=None):
    """oracle and GPU grid holding the same state"""
    ns = orc3.NS3(prm)
    for n in orc3.FIELDS:
        getattr(ns, n)[...] = st[n]
    ns.s.dt = dt
    g = M.Grid3(prm)
    if tune is not None:
        set_tune(g, tune)
    for n in orc3.FIELDS:
        g.upload(GPU_FIELD[n], st[n])
    g.set_dt(dt)
    return ns, g


def assert_fields_equal(ns, g, what):
    for n in orc3.FIELDS:
        got = g.download(GPU_FIELD[n])
        ref = getattr(ns, n)
        if not np.array_equal(got, ref):
            bad = np.argwhere(got != ref)
            raise AssertionError("%s: field %s differs at %d cells, first (k,j,i)=%s: %r vs %r"
                                 % (what, n, len(bad), tuple(bad[0]), got[tuple(bad[0])],
                                    ref[tuple(bad[0])]))


@pytest.mark.parametrize("bcs", BCS)
@pytest.mark.parametrize("fn", sorted(STEP_FNS))
@pytest.mark.parametrize("name,dims", [("a6_dcavity.par", (13, 9, 7)),
                                       ("a6_canal.par", (70, 33, 6)),
                                       ("a6_dcavity.par", (129, 5, 3))])
def test_step_functions_bitwise(golden, name, dims, fn, bcs):
    over = dict(zip(BC_KEYS, bcs), imax=dims[0], jmax=dims[1], kmax=dims[2])
    prm = params(golden, name, **over)
    shape = (dims[2] + 2, dims[1] + 2, dims[0] + 2)
    st = random_state(shape, zlib.crc32(repr((name, fn, bcs, dims)).encode()))
    ns, g = pair(prm, st, 0.0137)
    with g:
        ns.call(STEP_FNS[fn])
        g.call(fn)
        if fn == "normalize_pressure":
            # the mean is summed in a fixed tree order, the reference sums
            # sequentially: p - avg agrees to the rounding of avg (the 3D main
            # never calls normalizePressure, assignment-6/src/main.c:45-60)
            got = g.download(M.P3)
            assert np.allclose(got, ns.p, rtol=0, atol=1e-14 * np.abs(ns.p).max())
            for n in orc3.FIELDS:
                if n != "p":
                    assert np.array_equal(g.download(GPU_FIELD[n]), getattr(ns, n)), n
            return
        assert_fields_equal(ns, g, fn)


@pytest.mark.parametrize("name,dims", [("a6_dcavity.par", (13, 9, 7)),
                                       ("a6_canal.par", (200, 50, 50))])
def test_compute_timestep_bitwise(golden, name, dims):
    prm = params(golden, name, imax=dims[0], jmax=dims[1], kmax=dims[2])
    shape = (dims[2] + 2, dims[1] + 2, dims[0] + 2)
    st = random_state(shape, 7)
    st["w"][3, 2, 1] = -9.5  # the maximum of |w| sits on a negative cell
    ns, g = pair(prm, st, 0.0)
    with g:
        ns.call("compute_timestep")
        dt = g.compute_timestep()
        assert dt == ns.s.dt
        mx = g.max_uvw()
        for q, n in enumerate(("u", "v", "w")):
            assert mx[q] == orc3.lib().orc3_max_element(ns.s, getattr(ns.s, n))


def test_compute_timestep_at_rest(golden):
    """all velocities 0: maxElement returns DBL_MIN (> 0) and dt = tau*min(dtBound, d/DBL_MIN)"""
    prm = params(golden, "a6_dcavity.par", imax=16, jmax=8, kmax=4)
    st = {n: np.zeros((6, 10, 18)) for n in orc3.FIELDS}
    ns, g = pair(prm, st, 0.0)
    with g:
        ns.call("compute_timestep")
        assert g.compute_timestep() == ns.s.dt


@pytest.mark.parametrize("tune", SOLVE_TUNES)
@pytest.mark.parametrize("dims,itermax", [((5, 4, 3), 37), ((12, 9, 7), 11),
                                          ((64, 16, 8), 25), ((131, 37, 19), 9),
                                          ((125, 13, 30), 4), ((249, 25, 17), 2),
                                          ((256, 128, 64), 3), ((128, 128, 128), 5)])
def test_solve_fixed_iterations_bitwise(golden, dims, itermax, tune):
    prm = params(golden, "a6_dcavity.par", imax=dims[0], jmax=dims[1], kmax=dims[2],
                 eps=1e-150, itermax=itermax)
    shape = (dims[2] + 2, dims[1] + 2, dims[0] + 2)
    st = random_state(shape, sum(dims))
    ns, g = pair(prm, st, 0.02, tune)
    with g:
        it_ref, res_ref = ns.solve()
        it, res = g.solve()
        assert it == it_ref == itermax
        assert_fields_equal(ns, g, "solve")  # p incl. every ghost, and nothing else touched
        assert res == pytest.approx(res_ref, rel=1e-12)


@pytest.mark.parametrize("tune", SOLVE_TUNES)
@pytest.mark.parametrize("dims,eps", [((24, 20, 16), 1e-3), ((40, 12, 10), 1e-4),
                                      ((33, 33, 33), 1e-4), ((64, 32, 32), 1e-4)])
def test_solve_converges_like_oracle(golden, dims, eps, tune):
    """convergence-driven stop: same iteration count and bit-identical p"""
    prm = params(golden, "a6_dcavity.par", imax=dims[0], jmax=dims[1], kmax=dims[2],
                 eps=eps, itermax=5000)
    shape = (dims[2] + 2, dims[1] + 2, dims[0] + 2)
    st = random_state(shape, 11)
    st["p"] *= 1e-3
    st["rhs"] *= 1e-3
    ns, g = pair(prm, st, 0.02, tune)
    with g:
        it_ref, res_ref = ns.solve()
        it, res = g.solve()
        assert 1 < it_ref < 5000
        assert it == it_ref
        assert np.array_equal(g.download(M.P3), ns.p)
        assert res == pytest.approx(res_ref, rel=1e-12)
        # a second solve continues from the converged p (as the next time step does)
        it2_ref, _ = ns.solve()
        it2, _ = g.solve()
        assert it2 == it2_ref
        assert np.array_equal(g.download(M.P3), ns.p)
        # a third after p was replaced from the host (edges and corners included)
        newp = np.random.default_rng(5).standard_normal(shape) * 1e-3
        ns.p[...] = newp
        g.upload(M.P3, newp)
        it3_ref, _ = ns.solve()
        assert g.solve()[0] == it3_ref
        assert np.array_equal(g.download(M.P3), ns.p)


def test_solve_itermax_zero_does_nothing(golden):
    prm = params(golden, "a6_dcavity.par", imax=8, jmax=8, kmax=8, itermax=0)
    st = random_state((10, 10, 10), 3)
    ns, g = pair(prm, st, 0.02)
    with g:
        assert g.solve()[0] == ns.solve()[0] == 0
        assert np.array_equal(g.download(M.P3), st["p"])


def run_gpu(prm, steps, tune=None):
    """assignment-6/src/main.c:45-60 through the C ABI (no normalizePressure)"""
    g = M.Grid3(prm)
    if tune is not None:
        set_tune(g, tune)
    g.fill(M.U3, prm["u_init"])
    g.fill(M.V3, prm["v_init"])
    g.fill(M.W3, prm["w_init"])
    g.fill(M.P3, prm["p_init"])
    g.set_dt(prm["dt"])
    t, iters = 0.0, []
    while t <= prm["te"] and len(iters) < steps:
        dt = g.compute_timestep() if prm["tau"] > 0.0 else prm["dt"]
        for fn in ("set_boundary_conditions", "set_special_boundary_condition", "compute_fg",
                   "compute_rhs"):
            g.call(fn)
        iters.append(g.solve()[0])
        g.call("adapt_uvw")
        t += dt
    return g, np.array(iters), t


@pytest.mark.parametrize("tune", [(1, 8, 0), (0, 8, 0), (1, 4, 4), (1, 8, 0, 0), (1, 8, 0, 0, 2),
                                  (1, 8, 0, 1, 0, 1)])
@pytest.mark.parametrize("fixture,par", [("ns3d_dcavity_short.npz", "a6_dcavity.par"),
                                         ("ns3d_canal_short.npz", "a6_canal.par")])
def test_short_run_matches_reference_fixture(golden, fixture, par, tune):
    ref = np.load(os.path.join(golden, fixture))
    dims = [int(x) for x in ref["dims"]]
    prm = params(golden, par, imax=dims[0], jmax=dims[1], kmax=dims[2])
    steps = int(ref["steps"])
    g, iters, t = run_gpu(prm, steps, tune)
    with g:
        assert np.array_equal(iters, ref["iters"])
        assert t == ref["t"]
        for n in ("p", "u", "v", "w"):
            assert np.array_equal(g.download(GPU_FIELD[n]), ref[n]), n


def test_medium_run_matches_oracle(golden):
    """a6 dcavity at 48^3 for 6 steps: the oracle's run, bit for bit"""
    prm = params(golden, "a6_dcavity.par", imax=48, jmax=48, kmax=48)
    ns = orc3.NS3(prm)
    n, iters_ref, t_ref = ns.run(max_steps=6)
    g, iters, t = run_gpu(prm, 6)
    with g:
        assert np.array_equal(iters, iters_ref)
        assert t == t_ref
        for n in ("p", "u", "v", "w"):
            assert np.array_equal(g.download(GPU_FIELD[n]), getattr(ns, n)), n


def test_resident_only_when_it_fits(golden):
    """288 x 128 x 64 needs 288 boxes of 32x16x16 (> 256 CUs): the streaming sweep runs"""
    prm = params(golden, "a6_dcavity.par", imax=288, jmax=128, kmax=64, itermax=2)
    with M.Grid3(prm) as g:
        g.set_tuning(M.TUNE3_RESIDENT, 1)
        assert g.get_tuning(M.TUNE3_RESIDENT) == 0
    prm = params(golden, "a6_dcavity.par", imax=128, jmax=128, kmax=128, itermax=2)
    with M.Grid3(prm) as g:
        g.set_tuning(M.TUNE3_RESIDENT, -1)
        assert g.get_tuning(M.TUNE3_RESIDENT) == 1


def test_tuning_keys(golden):
    prm = params(golden, "a6_dcavity.par", imax=8, jmax=8, kmax=8)
    with M.Grid3(prm) as g:
        assert g.get_tuning(M.TUNE3_SWEEP) == 1 and g.get_tuning(M.TUNE3_ROWS) == 8
        assert g.get_tuning(M.TUNE3_KCHUNK) >= 8
        assert g.get_tuning(M.TUNE3_FOLD) == 1 and g.get_tuning(M.TUNE3_RHS_AHEAD) == 0
        assert g.get_tuning(M.TUNE3_RESIDENT) == 1  # default: resident when the grid fits
        g.set_tuning(M.TUNE3_RESIDENT, 0)
        assert g.get_tuning(M.TUNE3_RESIDENT) == 0
        for key, bad in ((M.TUNE3_SWEEP, 2), (M.TUNE3_ROWS, 5), (M.TUNE3_KCHUNK, 2),
                         (M.TUNE3_RESIDENT, 2), (99, 0)):
            with pytest.raises(M.MisorError):
                g.set_tuning(key, bad)
