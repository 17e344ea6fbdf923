"""Parity at the sizes and launch geometry bench.py times (BASELINE configs 4
and 5), not only at the small grids of test_sor_gpu.py.

Config 4 (2D Poisson red-black SOR, 32768^2): the timed solve runs passes of
the default T iterations per launch over the automatic block geometry, with
a last pass of steps % T iterations (bench.py --steps 20: T + T + rest).
  * 8192^2 with the block height forced to the one the 32768^2 launch uses,
    k = one pass, two passes and the driver's 20 iterations, bit for bit
    against the restatement of solveRB (assignment-4/src/solver.c:179-238);
  * 32768^2 itself: after k iterations a cell depends only on cells within
    2k of it (red reads +-1, black the new red +-1), so windows of the
    device's field are checked bit for bit against the oracle run on the
    same window with a 2k+2 margin trimmed -- the four physical corners
    (ghosts included: the window's outer sides are the real boundary) and
    one interior window.
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
    assert st["iters_per_pass"] == T
    want = p.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / n, 1.0 / n, OMEGA, 1e-300, kk)
    assert it == it_ref == kk
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert abs(res - res_ref) <= 1e-10 * res_ref


def window_oracle(p0, rhs, j0, i0, h, w, k, dx, dy):
    """solveRB over the (h, w) sub-array at (j0, i0) of the reference layout,
    treated as a whole grid (its outer rows/columns as ghosts)"""
    pw = np.ascontiguousarray(p0[j0:j0 + h, i0:i0 + w])
    rw = np.ascontiguousarray(rhs[j0:j0 + h, i0:i0 + w])
    it, _ = orc.solve_rb(pw, rw, dx, dy, OMEGA, 1e-300, k)
    assert it == k
    return pw


def test_full_size_32768_windows():
    n, k = 32768, 20
    m = 2 * k + 2            # dependency radius of k iterations, plus margin
    C = 812                  # corner window side (even: origins keep global parity)
    I = 768 + 2 * m          # interior window side
    N2 = n + 2               # rows / columns of the reference layout, ghosts included
    dx = dy = 1.0 / n
    # (j0, i0, h, w): the four physical corners and one interior window, all
    # with j0 + i0 even so the window's own (i+j) colouring is the global one
    wins = [(0, 0, C, C), (0, N2 - C, C, C), (N2 - C, 0, C, C), (N2 - C, N2 - C, C, C),
            (n // 2 - 600, n // 2 + 1000, I, I)]
    with M.Grid(n, n, dx, dy, OMEGA, 1e-300, k) as g:
        g.poisson_init(1.0, 1.0, 2)
        p0 = g.download(M.P)
        rhs = g.download(M.RHS)
        ref = [window_oracle(p0, rhs, j0, i0, h, w, k, dx, dy) for (j0, i0, h, w) in wins]
        del p0, rhs
        it, res = g.solve_rb()
        assert it == k
        got = g.download(M.P)
    for (j0, i0, h, w), pw in zip(wins, ref):
        # trim m cells on every side that is not the physical boundary
        jl = 0 if j0 == 0 else m
        jh = h if j0 + h == N2 else h - m
        il = 0 if i0 == 0 else m
        ih = w if i0 + w == N2 else w - m
        a = got[j0 + jl:j0 + jh, i0 + il:i0 + ih]
        b = pw[jl:jh, il:ih]
        assert min(a.shape) >= 768, (a.shape, j0, i0)
        assert np.array_equal(a, b), ((j0, i0), np.argwhere(a != b)[:5])


def test_ns_dcavity_16384_two_steps(golden):
    """BASELINE config 5 per GPU: a6 dcavity.par read as 2D at 16384^2"""
    prm = orc.read_par(os.path.join(golden, "a6_dcavity.par"))
    prm.update(imax=16384, jmax=16384, itermax=20)
    ns = orc.NS(prm)
    steps_ref, iters_ref, _ = ns.run(solver=1, max_steps=2)
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


def test_decomposed_8_ranks_32768_windows():
    """BASELINE config 4 at 8 GPUs: the 4 x 2 split of 32768^2 that bench.py
    --gpus 8 runs (one rank's block 8192 x 16384: T = 8, chained passes with
    their automatic geometry -- main and edge kernels, work stealing --,
    pipelined passes with the slot reserve, 2T-deep exchanges), as 8
    in-process ranks on the one GPU of the test box; windows at the physical
    corners and where two and four rank blocks meet, bit for bit against the
    oracle run on the window (see test_full_size_32768_windows)"""
    import threading
    n, k, world = 32768, 20, 8
    m = 2 * k + 2
    C, W = 812, 768 + 2 * m
    N2 = n + 2
    dx = 1.0 / n
    cid = b"LOCAL:bench8"
    outs, errs = [None] * world, []

    def body(r):
        try:
            with M.Grid(n, n, dx, dx, OMEGA, 1e-300, k, device=0, nranks=world, rank=r,
                        comm_id=cid) as g:
                g.poisson_init(1.0, 1.0, 2)
                p0, rhs = g.download(M.P), g.download(M.RHS)
                it, _ = g.solve_rb()
                assert g.get_tuning(M.TUNE_TB_CHAIN) == 1  # chained on a 2^27-cell block
                outs[r] = (g.loc, p0, rhs, g.download(M.P), it, g.stats()["iters_per_pass"])
        except BaseException as e:
            errs.append((r, repr(e)))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
        assert not t.is_alive(), "rank thread hung"
    assert not errs, errs
    assert all(o[4] == k for o in outs)
    assert all(o[5] == 8 for o in outs)  # T of a 2^27-cell block (misor_api.hip)
    assert tuple(outs[0][0].dims) == (4, 2) and (outs[0][0].ni, outs[0][0].nj) == (8192, 16384)

    def assemble(idx):
        glob = np.empty((N2, N2))
        for o in outs:
            loc, a = o[0], o[idx]
            nb = list(loc.neighbours)
            i0, j0 = (0 if nb[0] < 0 else 1), (0 if nb[2] < 0 else 1)
            i1 = loc.ni + 1 if nb[1] < 0 else loc.ni
            j1 = loc.nj + 1 if nb[3] < 0 else loc.nj
            glob[loc.joff + j0:loc.joff + j1 + 1, loc.ioff + i0:loc.ioff + i1 + 1] = \
                a[j0:j1 + 1, i0:i1 + 1]
        return glob

    p0, rhs = assemble(1), assemble(2)
    h = W // 2
    # (j0, i0, h, w), j0 + i0 even: four physical corners; the junction of four
    # blocks (j = 16384, i = 8192); a vertical boundary (i = 16384) inside a
    # block row; the horizontal boundary (j = 16384) at the physical left side
    wins = [(0, 0, C, C), (0, N2 - C, C, C), (N2 - C, 0, C, C), (N2 - C, N2 - C, C, C),
            (16384 - h, 8192 - h, W, W), (8000 - h, 16384 - h, W, W), (16384 - h, 0, W, C)]
    ref = [window_oracle(p0, rhs, j0, i0, hh, w, k, dx, dx) for (j0, i0, hh, w) in wins]
    del p0, rhs
    got = assemble(3)
    outs.clear()
    for (j0, i0, hh, w), pw in zip(wins, ref):
        jl = 0 if j0 == 0 else m
        jh = hh if j0 + hh == N2 else hh - m
        il = 0 if i0 == 0 else m
        ih = w if i0 + w == N2 else w - m
        a = got[j0 + jl:j0 + jh, i0 + il:i0 + ih]
        b = pw[jl:jh, il:ih]
        assert min(a.shape) >= 768, (a.shape, j0, i0)
        assert np.array_equal(a, b), ((j0, i0), np.argwhere(a != b)[:5])
