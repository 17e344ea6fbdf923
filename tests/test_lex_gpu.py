"""The reference's lexicographic Gauss-Seidel SOR `solve` on the GPU
(misor_solve_lex: anti-diagonal wavefront, lex_kernels.hip) -- the ordering
the reference's own programs call, so its committed outputs can be reproduced:

* assignment-4/src/solver.c:126-177 (xorder 0): poisson.par -> 2388 iterations
  and the committed assignment-4/p.dat, byte for byte;
* assignment-5/sequential/src/solver.c:140-191 (xorder 1): the sequential NS
  (its dcavity.par) step by step against the reference build's fields.

Bar: p bit-identical to the CPU oracle / reference (same expression order, no
FMA contraction); iteration counts identical (only the residual's summation
order differs).
"""
import os

import numpy as np
import pytest

import ns_gpu_driver as D
import orc
import pymisor as M

pytestmark = pytest.mark.gpu


def fmt_pdat(p):  # writeResult, assignment-4/src/solver.c:315-320
    return "\n".join("".join("%f " % x for x in row) for row in p) + "\n"


def test_lex_poisson_par_reproduces_committed_pdat(golden):
    z = np.load(os.path.join(golden, "rb_poisson100.npz"))
    with M.Grid(100, 100, 0.01, 0.01, 1.9, 1e-6, 1000000) as g:
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_lex(M.LEX_A4)
        p = g.download(M.P)
    assert it == int(z["iterations_lex"]) == 2388
    assert np.array_equal(p, z["p_lex"])
    assert fmt_pdat(p) == open(os.path.join(golden, "a4_p.dat")).read()


@pytest.mark.parametrize("ni,nj", [(5, 3), (2, 9), (37, 23), (64, 65), (10, 129), (100, 100),
                                   (139, 139), (3, 257), (20, 300), (150, 141), (301, 40)])
@pytest.mark.parametrize("xorder", [0, 1])
def test_lex_random_fields_vs_oracle(ni, nj, xorder):
    """p in LDS (workgroup sized to the longest diagonal: 64 .. 1024 threads);
    (150,141) and (301,40) do not fit in LDS: the HBM-resident form"""
    rng = np.random.default_rng(ni * 31 + nj + xorder)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    dx, dy = 1.3 / ni, 0.7 / nj
    for k in (1, 2, 5):
        want = p.copy()
        it_ref, res_ref = orc.solve_lex(want, rhs, dx, dy, 1.7, 1e-300, k, xorder=xorder)
        with M.Grid(ni, nj, dx, dy, 1.7, 1e-300, k) as g:
            g.upload(M.P, p)
            g.upload(M.RHS, rhs)
            it, res = g.solve_lex(xorder)
            got = g.download(M.P)
        assert it == it_ref == k
        assert np.array_equal(got, want), (k, np.argwhere(got != want)[:5])
        assert abs(res - res_ref) <= 1e-12 * abs(res_ref)


@pytest.mark.parametrize("n", [50, 64, 128])
def test_lex_iteration_counts(n):
    p, rhs = orc.poisson_init(n, n)
    want = p.copy()
    it_ref, _ = orc.solve_lex(want, rhs, 1.0 / n, 1.0 / n, 1.9, 1e-6, 1000000, xorder=0)
    with M.Grid(n, n, 1.0 / n, 1.0 / n, 1.9, 1e-6, 1000000) as g:
        g.poisson_init(1.0, 1.0, 2)
        it, _ = g.solve_lex(M.LEX_A4)
        assert it == it_ref
        assert np.array_equal(g.download(M.P), want)


def test_lex_ns_sequential_dcavity(golden):
    """the reference's own NS (assignment-5/sequential, lexicographic solve) on
    its dcavity.par for 400 steps: fields vs the reference build, per-step
    iterations vs the restatement's (iters_oracle of the fixture: the shipped
    solve() reports none; tests/golden/make_golden.py)"""
    z = np.load(os.path.join(golden, "ns_seq_dcavity_lex_short.npz"))
    prm = orc.read_par(os.path.join(golden, "seq_dcavity.par"))
    prm["te"] = float(z["te"])
    g = D.ns_grid(prm)
    steps, iters, t = D.run(g, prm, solver="lex")
    fields = {k: g.download(fid) for k, fid in (("p", M.P), ("u", M.U), ("v", M.V))}
    g.close()
    assert steps == int(z["steps"])
    assert np.array_equal(iters, z["iters_oracle"]), np.argwhere(iters != z["iters_oracle"])[:5]
    for k in ("p", "u", "v"):
        err = np.abs(fields[k] - z[k]).max() / np.abs(z[k]).max()
        assert err <= 1e-12, (k, err)


def test_lex_rejects_decomposed_grid():
    cid = b"LOCAL:lexreject"
    import threading
    errs = []

    def body(r):
        try:
            with M.Grid(20, 20, 0.05, 0.05, 1.9, 1e-6, 10, device=0, nranks=2, rank=r,
                        comm_id=cid) as g:
                try:
                    g.solve_lex(0)
                    errs.append("accepted")
                except M.MisorError:
                    pass
        except BaseException as e:
            errs.append(repr(e))

    th = [threading.Thread(target=body, args=(r,)) for r in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(60)
    assert not errs, errs
