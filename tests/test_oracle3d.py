"""The 3D oracle (oracle/oracle3d.c) against the reference's own 3D solver
(assignment-6/src/solver.c compiled in place: oracle/_ref/libref3d.so),
function by function on random states and over whole short runs: bit for bit.

TEST INFRASTRUCTURE: pins the checker of the GPU 3D path.  Skipped where the
reference build is absent (the GPU box); the GPU tests use the committed
fixtures made from it (tests/golden/make_golden.py).
"""
import itertools
import os

import numpy as np
import pytest

import orc3

pytestmark = pytest.mark.skipif(not orc3.have_ref3(), reason="reference 3D build absent")


def random_state(shape, seed):
    rng = np.random.default_rng(seed)
    return {n: rng.standard_normal(shape) for n in orc3.FIELDS}


def ns_with(prm, st, dt):
    ns = orc3.NS3(prm)
    for n in orc3.FIELDS:
        getattr(ns, n)[...] = st[n]
    ns.s.dt = dt
    return ns


def par_file(tmp_path, golden, name, **over):
    """a6 .par with overrides written to a temp file (the reference reads files)"""
    txt = open(os.path.join(golden, name)).read()
    import re
    for k, v in over.items():
        txt, n = re.subn(r"(?m)^%s\s.*$" % k, "%s %s" % (k, v), txt)
        if n == 0:
            txt += "\n%s %s\n" % (k, v)
    path = str(tmp_path / ("p_" + name))
    open(path, "w").write(txt)
    return path


BCS = [(1, 1, 1, 1, 1, 1), (2, 3, 1, 2, 3, 1), (3, 3, 2, 2, 1, 3), (1, 2, 3, 1, 2, 3),
       (4, 4, 1, 1, 4, 2)]


@pytest.mark.parametrize("bcs", BCS)
@pytest.mark.parametrize("fn", ["set_bc", "set_special_bc", "compute_fg", "compute_rhs",
                                "adapt_uvw", "normalize_pressure", "compute_timestep"])
@pytest.mark.parametrize("name", ["a6_dcavity.par", "a6_canal.par"])
def test_step_functions_bitwise(golden, tmp_path, name, fn, bcs):
    keys = ("bcLeft", "bcRight", "bcBottom", "bcTop", "bcFront", "bcBack")
    over = dict(zip(keys, bcs), imax=13, jmax=9, kmax=7)
    path = par_file(tmp_path, golden, name, **over)
    prm = orc3.read_par3(path)
    shape = (prm["kmax"] + 2, prm["jmax"] + 2, prm["imax"] + 2)
    st = random_state(shape, hash((name, fn, bcs)) & 0xFFFF)
    st["u"] *= 2.0
    ns = ns_with(prm, st, 0.0137)
    ref = {n: st[n].copy() for n in orc3.FIELDS}
    dt_ref, _ = orc3.ref3_call(path, (0, 0, 0), fn, 0.0137, ref)
    ns.call(fn)
    assert ns.s.dt == dt_ref
    for n in orc3.FIELDS:
        assert np.array_equal(getattr(ns, n), ref[n]), (fn, n)


@pytest.mark.parametrize("dims", [(5, 4, 3), (12, 9, 7), (16, 16, 16)])
def test_solve_bitwise(golden, tmp_path, dims):
    path = par_file(tmp_path, golden, "a6_dcavity.par", imax=dims[0], jmax=dims[1],
                    kmax=dims[2], eps=1e-9, itermax=37)
    prm = orc3.read_par3(path)
    shape = (dims[2] + 2, dims[1] + 2, dims[0] + 2)
    st = random_state(shape, sum(dims))
    ns = ns_with(prm, st, 0.02)
    ref = {n: st[n].copy() for n in orc3.FIELDS}
    _, it_ref = orc3.ref3_call(path, (0, 0, 0), "solve", 0.02, ref)
    it, _ = ns.solve()
    assert it == it_ref
    assert np.array_equal(ns.p, ref["p"])


@pytest.mark.parametrize("name,dims", [("a6_dcavity.par", (12, 10, 8)),
                                       ("a6_canal.par", (20, 6, 5))])
def test_short_runs_bitwise(golden, tmp_path, name, dims):
    path = par_file(tmp_path, golden, name, imax=dims[0], jmax=dims[1], kmax=dims[2])
    prm = orc3.read_par3(path)
    n, iters, p, u, v, w, t = orc3.ref3_run(path, max_steps=12)
    ns = orc3.NS3(prm)
    n2, iters2, t2 = ns.run(max_steps=12)
    assert n == n2 == 12 and t == t2
    assert np.array_equal(iters, iters2)
    for k, ref in (("p", p), ("u", u), ("v", v), ("w", w)):
        assert np.array_equal(getattr(ns, k), ref), k
