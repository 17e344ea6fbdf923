"""Whole-field parity at the configurations the driver times (BASELINE configs
4 and 5), every cell compared -- not windows.

Config 4 (2D Poisson red-black SOR, 32768^2, bench.py --steps 20 --warmup 5,
the driver's setting, BENCH_r04.json): the bench runs a warm-up solve of 5
iterations and one of 20, then times a third solve of 20 iterations (the short
pass plan: two 10-iteration passes of the split-ring kernel, TB variant 13,
misor_api.hip solve_rb_from).  The test replays exactly that sequence on one
Grid, asserts that the timed solve ran that kernel and plan, downloads the field the timed solve starts from, and
checks the WHOLE 32770^2 result (ghosts included) bit for bit, and res to
1e-12, against the multi-core restatement of solveRB
(assignment-4/src/solver.c:179-238; oracle/oracle_mt.c, p bit-identical to
the single-thread restatement) started from that same field.  A block skipped
or computed twice anywhere -- persistent queues, chained runs and work
stealing decide at run time which workgroup computes which block -- fails it.

Config 4 at 2, 4 and 8 GPUs: the splits of bench.py --gpus N (2 x 1: the short
plan on 2^29-cell blocks; 2 x 2: 16384^2 = 2^28-cell blocks, the short plan
(chained split ring), pipelined; 4 x 2: one rank's block 8192 x 16384, chained split-ring
passes of 10 iterations) as N
in-process ranks on the one GPU (pipelined loop, 2T-deep exchanges); the
assembled field against the same oracle.

Config 5 at 8 GPUs: dcavity NS on the 8-rank global grid 65536 x 32768 (16384^2
per rank, bench.py --workload ns --gpus 8), two time steps with the pressure
solve capped at 20 iterations, as 8 in-process ranks, against a ONE-rank GPU
run of the same global grid (2^31 cells, ~121 GB of fields): identical
per-step iteration counts and p, u, v bit for bit (the reference's int
indexing cannot run this grid, SURVEY 0.6, so the 1-rank GPU run is the
oracle here; its kernels are checked against the restatement at 16384^2 in
test_bench_configs_gpu.py).
"""
import os
import threading

import numpy as np
import pytest

import ns_gpu_driver as D
import orc
import pymisor as M

pytestmark = pytest.mark.gpu

OMEGA = 1.9
STEPS, WARMUP = 20, 5  # the driver's bench setting (BENCH_r04.json: --steps 20 --warmup 5)


def host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def owned(loc):
    """(j0, j1, i0, i1) inclusive: interior + the physical ghost sides"""
    nb = list(loc.neighbours)
    i0 = 0 if nb[0] < 0 else 1
    i1 = loc.ni + 1 if nb[1] < 0 else loc.ni
    j0 = 0 if nb[2] < 0 else 1
    j1 = loc.nj + 1 if nb[3] < 0 else loc.nj
    return j0, j1, i0, i1


def put(glob, loc, blk):
    j0, j1, i0, i1 = owned(loc)
    glob[loc.joff + j0:loc.joff + j1 + 1, loc.ioff + i0:loc.ioff + i1 + 1] = \
        blk[j0:j1 + 1, i0:i1 + 1]


def first_diff(a, b):
    bad = np.argwhere(a != b)
    return bad[:5], len(bad)


def test_fullfield_32768_bench_sequence():
    n = 32768
    dx = 1.0 / n
    with M.Grid(n, n, dx, dx, OMEGA, 1e-300, STEPS) as g:
        g.poisson_init(1.0, 1.0, 2)
        g.solve_rb(itermax=WARMUP)   # bench.py: warm-up solves
        g.solve_rb(itermax=STEPS)
        p = g.download(M.P)
        rhs = g.download(M.RHS)
        g.enable_timing(True)  # as bench.py: per-pass events, stats from here
        g.reset_stats()
        it, res = g.solve_rb(itermax=STEPS)  # the timed solve
        st = g.stats()
        T = st["iters_per_pass"]
        got = g.download(M.P)
    assert it == STEPS
    # the kernel and plan bench.py times: two 10-iteration passes of the
    # chained split ring (sor_tbh.h rb_tbhc_kernel)
    assert (T, st["tb_variant"], st["timed_passes"], st["chained"]) == (10, 13, 2, 1), st
    it_ref, res_ref = orc.solve_rb_mt(p, rhs, dx, dx, OMEGA, 1e-300, STEPS, host_threads())
    del rhs
    assert it_ref == STEPS
    assert np.array_equal(got, p), (T, first_diff(got, p))
    assert abs(res - res_ref) <= 1e-12 * res_ref, (res, res_ref)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_fullfield_32768_ranks(world):
    """8 ranks: 2^27-cell blocks, two 10-iteration passes of the chained split
    ring; 4 ranks (2^28-cell blocks) and 2 ranks (2^29): the short pass plan
    (two 10-iteration split-ring passes)"""
    n = 32768
    dx = 1.0 / n
    cid = ("LOCAL:full%d" % world).encode()
    outs, errs = [None] * world, []

    def body(r):
        try:
            with M.Grid(n, n, dx, dx, OMEGA, 1e-300, STEPS, device=0, nranks=world, rank=r,
                        comm_id=cid) as g:
                g.poisson_init(1.0, 1.0, 2)
                g.solve_rb(itermax=WARMUP)
                g.solve_rb(itermax=STEPS)
                p0, rhs = g.download(M.P), g.download(M.RHS)
                it, res = g.solve_rb(itermax=STEPS)
                chain = g.get_tuning(M.TUNE_TB_CHAIN)
                st = g.stats()
                outs[r] = [g.loc, p0, rhs, g.download(M.P), it, res, chain,
                           (st["iters_per_pass"], st["tb_variant"], st["chained"])]
        except BaseException as e:
            errs.append((r, repr(e)))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
        assert not t.is_alive(), "rank thread hung"
    assert not errs, errs
    assert all(o[4] == STEPS for o in outs)
    if world == 8:
        assert all(o[6] == 1 for o in outs)  # chained passes on a 2^27-cell block
        assert tuple(outs[0][0].dims) == (4, 2) and (outs[0][0].ni, outs[0][0].nj) == (8192, 16384)
        # the chained split ring: T = 10 passes on the 2^27-cell blocks
        assert all(o[7] == (10, 13, 1) for o in outs), [o[7] for o in outs]
    elif world == 4:
        assert all(o[6] == 0 for o in outs)  # 2^28 cells: T = 8 passes would not be chained
        assert tuple(outs[0][0].dims) == (2, 2) and (outs[0][0].ni, outs[0][0].nj) == (16384, 16384)
        # the short plan: two chained split-ring passes
        assert all(o[7] == (10, 13, 1) for o in outs), [o[7] for o in outs]
    else:  # the short plan: 2 passes of the split ring (decomposed 2^29 blocks)
        assert all(o[7][:2] == (10, 13) for o in outs), [o[7] for o in outs]
    p = np.empty((n + 2, n + 2))
    rhs = np.empty((n + 2, n + 2))
    got = np.empty((n + 2, n + 2))
    for o in outs:
        put(p, o[0], o[1])
        put(rhs, o[0], o[2])
        put(got, o[0], o[3])
        o[1] = o[2] = o[3] = None
    res = outs[0][5]
    it_ref, res_ref = orc.solve_rb_mt(p, rhs, dx, dx, OMEGA, 1e-300, STEPS, host_threads())
    del rhs
    assert it_ref == STEPS
    assert np.array_equal(got, p), first_diff(got, p)
    # per-rank partial sums all-reduced: the rounding order differs from the
    # reference's single loop, not the value
    assert abs(res - res_ref) <= 1e-12 * res_ref, (res, res_ref)


def test_fullfield_ns_dcavity_8_ranks_global_grid(golden):
    """config 5 at 8 GPUs: 65536 x 32768 global, 8 ranks vs 1 rank"""
    prm = orc.read_par(os.path.join(golden, "a6_dcavity.par"))
    prm.update(imax=65536, jmax=32768, itermax=20)
    g = D.ns_grid(prm)
    try:
        steps1, iters1, _ = D.run(g, prm, max_steps=2)
        ref = {f: g.download(f) for f in (M.P, M.U, M.V)}
    finally:
        g.close()
    assert steps1 == 2

    world = 8
    cid = b"LOCAL:ns8full"
    outs, errs = [None] * world, []

    def body(r):
        try:
            gr = D.ns_grid(prm, nranks=world, rank=r, comm_id=cid)
            try:
                steps, iters, _ = D.run(gr, prm, max_steps=2)
                loc = gr.loc
                j0, j1, i0, i1 = owned(loc)
                ok = {}
                for f in (M.P, M.U, M.V):
                    a = gr.download(f)[j0:j1 + 1, i0:i1 + 1]
                    b = ref[f][loc.joff + j0:loc.joff + j1 + 1, loc.ioff + i0:loc.ioff + i1 + 1]
                    ok[f] = bool(np.array_equal(a, b))
                    del a
                outs[r] = (steps, list(iters), ok, tuple(loc.dims), (loc.ni, loc.nj))
            finally:
                gr.close()
        except BaseException as e:
            errs.append((r, repr(e)))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
        assert not t.is_alive(), "rank thread hung"
    assert not errs, errs
    assert outs[0][3] == (4, 2) and outs[0][4] == (16384, 16384)
    for r, (steps, iters, ok, _, _) in enumerate(outs):
        assert steps == 2 and iters == list(iters1), (r, iters, list(iters1))
        assert all(ok.values()), (r, ok)
