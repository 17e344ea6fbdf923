"""The 3D path decomposed into slabs of planes along k (misor3_decompose),
ranks as host threads of one process joined by libmisor's in-process
transport (comm_id "LOCAL:<name>") on the test box's single MI355X.  Everything
but the transport -- slab storage with 2-deep halos, the sweep's red on halo
planes, the physical-boundary flags, the all-reduced residual and loop test,
the gather -- is the code the RCCL path runs.

Bar: the gathered fields are bit-identical to the single-domain 3D oracle
(oracle/oracle3d.c, pinned to assignment-6's own build) with the same
iteration counts, for every slab count.
"""
import os
import threading

import numpy as np
import pytest

import orc3
import pymisor as M

pytestmark = pytest.mark.gpu

_gid = [0]
FIELD = {"p": M.P3, "rhs": M.RHS3, "u": M.U3, "v": M.V3, "w": M.W3, "f": M.F3, "g": M.G3,
         "h": M.H3}


def run_ranks(world, fn):
    _gid[0] += 1
    cid = ("LOCAL:n3d%d" % _gid[0]).encode()
    out = [None] * world
    err = []

    def body(r):
        try:
            out[r] = fn(r, cid)
        except BaseException as e:  # surfaced in the main thread
            err.append((r, repr(e)))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
        assert not t.is_alive(), "rank thread hung"
    assert not err, err
    return out


def params(golden, name, **over):
    prm = orc3.read_par3(os.path.join(golden, name))
    prm.update(over)
    return prm


def slab(a, koff, kloc):
    return np.ascontiguousarray(a[koff:koff + kloc + 2])


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("dims,itermax", [((13, 9, 16), 7), ((130, 37, 29), 4),
                                          ((64, 64, 64), 3)])
@pytest.mark.parametrize("rows,kc", [(8, 0), (4, 4)])
def test_solve_fixed_iterations_partition_independent(golden, world, dims, itermax, rows, kc):
    prm = params(golden, "a6_dcavity.par", imax=dims[0], jmax=dims[1], kmax=dims[2],
                 eps=1e-150, itermax=itermax)
    shape = (dims[2] + 2, dims[1] + 2, dims[0] + 2)
    rng = np.random.default_rng(sum(dims) + world)
    p0, rhs = rng.standard_normal(shape), rng.standard_normal(shape)
    ns = orc3.NS3(prm)
    ns.p[...] = p0
    ns.rhs[...] = rhs
    it_ref, res_ref = ns.solve()

    def rank(r, cid):
        with M.Grid3(prm, nranks=world, rank=r, comm_id=cid) as g:
            g.set_tuning(M.TUNE3_ROWS, rows)
            g.set_tuning(M.TUNE3_KCHUNK, kc)
            g.upload(M.P3, slab(p0, g.koff, g.kloc))
            g.upload(M.RHS3, slab(rhs, g.koff, g.kloc))
            it, res = g.solve()
            return it, res, g.gather(M.P3)

    out = run_ranks(world, rank)
    assert all(o[0] == it_ref == itermax for o in out)
    assert np.array_equal(out[0][2], ns.p)
    assert out[0][1] == pytest.approx(res_ref, rel=1e-12)


@pytest.mark.parametrize("world", [2, 4])
def test_solve_converges_partition_independent(golden, world):
    dims = (33, 33, 33)
    prm = params(golden, "a6_dcavity.par", imax=33, jmax=33, kmax=33, eps=1e-4, itermax=5000)
    shape = (35, 35, 35)
    rng = np.random.default_rng(11)
    p0, rhs = rng.standard_normal(shape) * 1e-3, rng.standard_normal(shape) * 1e-3
    ns = orc3.NS3(prm)
    ns.p[...] = p0
    ns.rhs[...] = rhs
    it_ref, _ = ns.solve()
    it2_ref, _ = ns.solve()

    def rank(r, cid):
        with M.Grid3(prm, nranks=world, rank=r, comm_id=cid) as g:
            g.upload(M.P3, slab(p0, g.koff, g.kloc))
            g.upload(M.RHS3, slab(rhs, g.koff, g.kloc))
            it, _ = g.solve()
            it2, _ = g.solve()
            return it, it2, g.gather(M.P3)

    out = run_ranks(world, rank)
    assert 1 < it_ref < 5000 and dims
    assert all(o[0] == it_ref and o[1] == it2_ref for o in out)
    assert np.array_equal(out[0][2], ns.p)


def run_steps(prm, world, steps):
    def rank(r, cid):
        with M.Grid3(prm, nranks=world, rank=r, comm_id=cid) as g:
            for f, v in ((M.U3, prm["u_init"]), (M.V3, prm["v_init"]), (M.W3, prm["w_init"]),
                         (M.P3, prm["p_init"])):
                g.fill(f, v)
            g.set_dt(prm["dt"])
            iters, t = [], 0.0
            for _ in range(steps):
                dt = g.compute_timestep() if prm["tau"] > 0.0 else prm["dt"]
                for fn in ("set_boundary_conditions", "set_special_boundary_condition",
                           "compute_fg", "compute_rhs"):
                    g.call(fn)
                iters.append(g.solve()[0])
                g.call("adapt_uvw")
                t += dt
            fields = {n: g.gather(FIELD[n]) for n in ("p", "u", "v", "w")}
            return iters, t, fields

    return run_ranks(world, rank)


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("name,dims", [("a6_dcavity.par", (24, 20, 16)),
                                       ("a6_canal.par", (40, 12, 12))])
def test_ns_steps_partition_independent(golden, world, name, dims):
    """assignment-6/src/main.c:45-60 decomposed: every field of every step as the
    single-domain oracle's run, bit for bit"""
    prm = params(golden, name, imax=dims[0], jmax=dims[1], kmax=dims[2])
    ns = orc3.NS3(prm)
    n, iters_ref, t_ref = ns.run(max_steps=8)
    out = run_steps(prm, world, 8)
    for iters, t, _ in out:
        assert iters == list(iters_ref) and t == t_ref
    for k in ("p", "u", "v", "w"):
        assert np.array_equal(out[0][2][k], getattr(ns, k)), k


def test_reference_fixture_on_four_slabs(golden):
    """the committed 16-step run of the reference itself, on 4 slabs"""
    ref = np.load(os.path.join(golden, "ns3d_dcavity_short.npz"))
    d = [int(x) for x in ref["dims"]]
    prm = params(golden, "a6_dcavity.par", imax=d[0], jmax=d[1], kmax=d[2])
    out = run_steps(prm, 4, int(ref["steps"]))
    assert out[0][0] == list(ref["iters"]) and out[0][1] == ref["t"]
    for k in ("p", "u", "v", "w"):
        assert np.array_equal(out[0][2][k], ref[k]), k


def test_normalize_and_timestep_decomposed(golden):
    prm = params(golden, "a6_canal.par", imax=20, jmax=10, kmax=12)
    shape = (14, 12, 22)
    rng = np.random.default_rng(3)
    st = {n: rng.standard_normal(shape) for n in orc3.FIELDS}
    st["w"][13, 4, 5] = 7.5  # the |w| maximum on the last physical ghost plane
    ns = orc3.NS3(prm)
    for n in orc3.FIELDS:
        getattr(ns, n)[...] = st[n]
    ns.call("compute_timestep")
    ns.call("normalize_pressure")

    def rank(r, cid):
        with M.Grid3(prm, nranks=3, rank=r, comm_id=cid) as g:
            for n in orc3.FIELDS:
                g.upload(FIELD[n], slab(st[n], g.koff, g.kloc))
            dt = g.compute_timestep()
            g.call("normalize_pressure")
            return dt, g.gather(M.P3)

    out = run_ranks(3, rank)
    assert all(o[0] == ns.s.dt for o in out)
    assert np.allclose(out[0][1], ns.p, rtol=0, atol=1e-14 * np.abs(ns.p).max())


def test_two_pass_refused_when_decomposed(golden):
    prm = params(golden, "a6_dcavity.par", imax=8, jmax=8, kmax=8)

    def rank(r, cid):
        with M.Grid3(prm, nranks=2, rank=r, comm_id=cid) as g:
            with pytest.raises(M.MisorError):
                g.set_tuning(M.TUNE3_SWEEP, 0)
        return True

    assert all(run_ranks(2, rank))
