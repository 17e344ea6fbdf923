"""Decomposed red-black SOR on the GPU kernels: partition independence.

The ranks of a 2D decomposition (misor_decompose: MPI_Dims_create +
sizeOfRank, assignment-5/skeleton/src/solver.c:30-32,445-473) run as host
threads of one process on the single MI355X of the test box, joined by
libmisor's in-process transport (comm_id "LOCAL:<name>").  Everything but the
transport -- 2-deep halo regions, pack/unpack kernels, the halo-ring red
recomputation, physical-side ghost copies, the all-reduced residual and the
device-side convergence decision -- is the code the RCCL path runs.

Bar: the assembled p is bit-identical to the single-domain oracle (solveRB,
assignment-4/src/solver.c:179-238) with the same iteration count, for every
partition.
"""
import threading

import numpy as np
import pytest

import orc
import pymisor as M

pytestmark = pytest.mark.gpu

_gid = [0]


def run_ranks(world, fn, dims=(0, 0)):
    """fn(rank, loc) -> result, each rank in its own thread"""
    _gid[0] += 1
    cid = ("LOCAL:t%d" % _gid[0]).encode()
    out = [None] * world
    err = []

    def body(r):
        try:
            out[r] = fn(r, cid, dims)
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


def local_window(a, loc):
    return np.ascontiguousarray(a[loc.joff:loc.joff + loc.nj + 2, loc.ioff:loc.ioff + loc.ni + 2])


def assemble(parts, shape):
    glob = np.full(shape, np.nan)
    for loc, blk in parts:
        nb = list(loc.neighbours)
        i0 = 0 if nb[0] < 0 else 1
        i1 = loc.ni + 1 if nb[1] < 0 else loc.ni
        j0 = 0 if nb[2] < 0 else 1
        j1 = loc.nj + 1 if nb[3] < 0 else loc.nj
        glob[loc.joff + j0:loc.joff + j1 + 1, loc.ioff + i0:loc.ioff + i1 + 1] = \
            blk[j0:j1 + 1, i0:i1 + 1]
    return glob


@pytest.mark.parametrize("world,dims", [(2, (0, 0)), (2, (1, 2)), (3, (0, 0)), (4, (0, 0)),
                                        (4, (1, 4)), (6, (0, 0)), (8, (0, 0))])
@pytest.mark.parametrize("ni,nj,k", [(61, 43, 5), (300, 257, 3), (2100, 90, 2)])
@pytest.mark.parametrize("overlap", [1, 0], ids=["overlap", "serial"])
@pytest.mark.parametrize("T", [1, 2, 4, 6, 7, 8], ids=["t1", "t2", "t4", "t6", "t7", "t8"])
def test_fixed_sweeps_partition_independent(world, dims, ni, nj, k, overlap, T):
    rng = np.random.default_rng(ni + 31 * nj + world)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 20
    dx, dy = 1.1 / ni, 0.8 / nj
    want = p.copy()
    it_ref, res_ref = orc.solve_rb(want, rhs, dx, dy, 1.85, 1e-300, k)

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, dx, dy, 1.85, 1e-300, k, device=0, nranks=world, rank=r,
                    dims=dims, comm_id=cid) as g:
            g.set_tuning(M.TUNE_OVERLAP, overlap)
            g.set_tuning(M.TUNE_TSTEPS, T)  # 2T-deep halo per pass of T iterations
            g.upload(M.P, local_window(p, g.loc))
            g.upload(M.RHS, local_window(rhs, g.loc))
            it, res = g.solve_rb()
            return g.loc, g.download(M.P), it, res

    outs = run_ranks(world, rank_fn, dims)
    got = assemble([(o[0], o[1]) for o in outs], p.shape)
    for (_, _, it, res) in outs:
        assert it == k
        assert abs(res - res_ref) <= 1e-12 * abs(res_ref)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("T", [1, 3])
def test_poisson_par_converges_decomposed(golden, world, T):
    """poisson.par to convergence (2388 iterations) on 2 / 4 ranks"""
    z = np.load(golden + "/rb_poisson100.npz")

    def rank_fn(r, cid, dims):
        with M.Grid(100, 100, 0.01, 0.01, 1.9, 1e-6, 1000000, device=0, nranks=world, rank=r,
                    comm_id=cid) as g:
            g.set_tuning(M.TUNE_TSTEPS, T)
            g.poisson_init(1.0, 1.0, 2)
            it, res = g.solve_rb()
            return g.loc, g.download(M.P), it

    outs = run_ranks(world, rank_fn)
    assert all(o[2] == 2388 for o in outs)
    got = assemble([(o[0], o[1]) for o in outs], z["p"].shape)
    assert np.array_equal(got, z["p"])  # corners included: the corner ranks own them


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("T", [2, 3, 4, 5, 6])
def test_converges_mid_pass_decomposed(world, T):
    """convergence inside a pass of T iterations: every rank recomputes its
    last pass with fewer iterations from the untouched source buffer"""
    ni, nj = 300, 190
    p, rhs = orc.poisson_init(ni, nj)
    want = p.copy()
    eps = 3e-3
    it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.9, eps, 100000)
    assert it_ref % 12 != 0  # ends mid-pass for at least two of T = 2, 3, 4

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.9, eps, 100000, device=0, nranks=world,
                    rank=r, comm_id=cid) as g:
            g.set_tuning(M.TUNE_TSTEPS, T)
            g.poisson_init(1.0, 1.0, 2)
            it, res = g.solve_rb()
            return g.loc, g.download(M.P), it, res

    outs = run_ranks(world, rank_fn)
    for o in outs:
        assert o[2] == it_ref
        assert abs(o[3] - res_ref) <= 1e-12 * res_ref
    got = assemble([(o[0], o[1]) for o in outs], p.shape)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("T", [0, 4, 8], ids=["plan", "t4", "t8"])
def test_stop_mid_batch_then_solve_again(world, T):
    """The pipelined loop enqueues batches of passes and reads the loop state
    after each batch.  A solve that converges inside a batch must leave
    nothing of it queued (round-5 review: a part-2 launch of the next pass
    could still run after the hand-over and write a pressure buffer): solve to
    convergence, then at once two more solves on the same field (and, with the
    near band forced, an exact-tail solve), p bit for bit against the oracle
    running the same sequence."""
    ni, nj = 300, 190
    p, rhs = orc.poisson_init(ni, nj)
    dx, dy = 1.0 / ni, 1.0 / nj
    eps = 3e-3
    want = p.copy()
    seq = []
    it, res = orc.solve_rb(want, rhs, dx, dy, 1.9, eps, 100000)
    seq.append(it)
    for cap in (9, 23):  # continue from the converged field
        it, _ = orc.solve_rb(want, rhs, dx, dy, 1.9, eps, cap)
        seq.append(it)

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, dx, dy, 1.9, eps, 100000, device=0, nranks=world, rank=r,
                    comm_id=cid) as g:
            if T:
                g.set_tuning(M.TUNE_TSTEPS, T)
            g.poisson_init(1.0, 1.0, 2)
            got = [g.solve_rb()[0]]
            for cap in (9, 23):
                got.append(g.solve_rb(itermax=cap)[0])
            return g.loc, g.download(M.P), got

    outs = run_ranks(world, rank_fn)
    assert all(o[2] == seq for o in outs), (seq, [o[2] for o in outs])
    assert np.array_equal(assemble([(o[0], o[1]) for o in outs], p.shape), want)

    # a capped solve, then one with the near band forced (every iteration
    # recomputed by the exact tail after the batched passes stop before it)
    want2 = p.copy()
    seq2 = [orc.solve_rb(want2, rhs, dx, dy, 1.9, eps, 57)[0]]
    seq2.append(orc.solve_rb(want2, rhs, dx, dy, 1.9, eps, 40)[0])

    def rank_fn2(r, cid, dims):
        with M.Grid(ni, nj, dx, dy, 1.9, eps, 100000, device=0, nranks=world, rank=r,
                    comm_id=cid) as g:
            if T:
                g.set_tuning(M.TUNE_TSTEPS, T)
            g.poisson_init(1.0, 1.0, 2)
            got = [g.solve_rb(itermax=57)[0]]
            g.set_tuning(M.TUNE_NEAR_BAND, -30)
            got.append(g.solve_rb(itermax=40)[0])
            return g.loc, g.download(M.P), got

    outs = run_ranks(world, rank_fn2)
    assert all(o[2] == seq2 for o in outs), (seq2, [o[2] for o in outs])
    assert np.array_equal(assemble([(o[0], o[1]) for o in outs], p.shape), want2)


@pytest.mark.parametrize("world,dims", [(2, (0, 0)), (4, (0, 0)), (6, (3, 2)), (4, (1, 4))])
def test_gather_assembles_global_field(world, dims):
    """misor_gather (collectResult): rank 0 receives every rank's block incl.
    the physical ghost layer -- the whole (jmax+2) x (imax+2) field"""
    ni, nj = 97, 61
    rng = np.random.default_rng(world)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    want = p.copy()
    orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 5)

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 5, device=0, nranks=world, rank=r,
                    dims=dims, comm_id=cid) as g:
            g.upload(M.P, local_window(p, g.loc))
            g.upload(M.RHS, local_window(rhs, g.loc))
            g.solve_rb()
            return g.gather(M.P), g.gather(M.RHS)

    outs = run_ranks(world, rank_fn, dims)
    assert all(o[0] is None and o[1] is None for o in outs[1:])
    assert np.array_equal(outs[0][0], want)
    assert np.array_equal(outs[0][1], rhs)


def test_rccl_single_rank_path(golden):
    """nranks=1 with a real RCCL id: the decomposed code path (RCCL init and
    all-reduce on the comm stream, interior/boundary split launches) on the
    one GPU of the box -- RCCL cannot put two ranks on one device."""
    z = np.load(golden + "/rb_poisson100.npz")
    cid = M.comm_unique_id()
    with M.Grid(100, 100, 0.01, 0.01, 1.9, 1e-6, 1000000, device=0, nranks=1, rank=0,
                comm_id=cid) as g:
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb()
        assert it == 2388
        assert np.array_equal(g.download(M.P), z["p"])
    n = 3000
    p, rhs = orc.poisson_init(n, n)
    it_ref, res_ref = orc.solve_rb(p, rhs, 1.0 / n, 1.0 / n, 1.9, 1e-300, 3)
    with M.Grid(n, n, 1.0 / n, 1.0 / n, 1.9, 1e-300, 3, device=0, nranks=1, rank=0,
                comm_id=M.comm_unique_id()) as g:
        g.poisson_init(1.0, 1.0, 2)
        it, res = g.solve_rb()
        assert it == 3 and np.array_equal(g.download(M.P), p)
        assert abs(res - res_ref) <= 1e-12 * res_ref


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("T", [2, 6])
def test_consecutive_solves_rotate_buffers(world, T):
    """three solves in a row (7, 13, 25 iterations): the pipelined pass loop
    rotates three pressure buffers, so each solve starts from a different one;
    p after each solve is bit-identical to the single-domain oracle"""
    ni, nj = 410, 230
    rng = np.random.default_rng(7 * world + T)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 10
    dx, dy = 1.0 / ni, 1.3 / nj
    counts = (7, 13, 25)
    wants = []
    w = p.copy()
    for k in counts:
        orc.solve_rb(w, rhs, dx, dy, 1.8, 1e-300, k)
        wants.append(w.copy())

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, dx, dy, 1.8, 1e-300, 100, device=0, nranks=world, rank=r,
                    comm_id=cid) as g:
            g.set_tuning(M.TUNE_TSTEPS, T)
            g.upload(M.P, local_window(p, g.loc))
            g.upload(M.RHS, local_window(rhs, g.loc))
            got = []
            for k in counts:
                it, _ = g.solve_rb(itermax=k)
                assert it == k
                got.append(g.download(M.P))
            return g.loc, got

    outs = run_ranks(world, rank_fn)
    for s in range(len(counts)):
        got = assemble([(o[0], o[1][s]) for o in outs], p.shape)
        assert np.array_equal(got, wants[s]), (s, np.argwhere(got != wants[s])[:5])


def test_rccl_single_rank_pipelined_fixed_sweeps():
    """the pipelined pass loop on real RCCL streams (one rank): interior and
    edge launches, exchange and all-reduce on their own streams, 3 consecutive
    solves of many passes each, bit-identical to the oracle"""
    ni, nj = 1500, 1100
    p, rhs = orc.poisson_init(ni, nj)
    want = p.copy()
    with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.9, 1e-300, 100, device=0, nranks=1, rank=0,
                comm_id=M.comm_unique_id()) as g:
        g.poisson_init(1.0, 1.0, 2)
        for k in (31, 24, 50):
            it_ref, res_ref = orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.9, 1e-300, k)
            it, res = g.solve_rb(itermax=k)
            assert it == k == it_ref
            assert abs(res - res_ref) <= 1e-12 * res_ref
            assert np.array_equal(g.download(M.P), want)


@pytest.mark.parametrize("reserve", [0, 16, 500, 1 << 20])
def test_pipelined_reserve(reserve):
    """the pipelined loop's persistent interior launch leaves `reserve` of its
    workgroup slots to the other streams (misor_api.hip, SweepParams.reserve;
    at least 8 workgroups remain, so 2^20 runs the whole pass on 8 queue
    workers): p stays bit-identical over several passes and a remainder pass"""
    world, ni, nj, k, T = 4, 900, 700, 19, 4
    rng = np.random.default_rng(reserve % 1000 + 5)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2)) * 20
    dx, dy = 1.0 / ni, 1.0 / nj
    want = p.copy()
    orc.solve_rb(want, rhs, dx, dy, 1.7, 1e-300, k)

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, dx, dy, 1.7, 1e-300, k, device=0, nranks=world, rank=r,
                    dims=dims, comm_id=cid) as g:
            g.set_tuning(M.TUNE_TSTEPS, T)
            g.set_tuning(M.TUNE_TB_RESERVE, reserve)
            assert g.get_tuning(M.TUNE_TB_RESERVE) == reserve
            g.upload(M.P, local_window(p, g.loc))
            g.upload(M.RHS, local_window(rhs, g.loc))
            it, _ = g.solve_rb()
            return g.loc, g.download(M.P), it

    outs = run_ranks(world, rank_fn)
    assert all(o[2] == k for o in outs)
    got = assemble([(o[0], o[1]) for o in outs], p.shape)
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


@pytest.mark.parametrize("world,dims", [(2, (0, 0)), (4, (0, 0)), (6, (3, 2)), (8, (0, 0))])
@pytest.mark.parametrize("depth", [1, 2, 7])
def test_exchange_rank_fill(world, dims, depth):
    """the skeleton's printExchange check (assignment-5/skeleton/src/solver.c:38-66):
    every rank fills the cells it owns -- its interior plus the ghost cells on
    its physical sides -- with a code of (rank, global i, global j) and the
    rest of its array with -1; after misor_exchange at any depth every cell of
    every rank's (ni+2) x (nj+2) array holds the code its owner wrote for that
    global cell: own cells untouched, halo edges and corners from the 8
    neighbours (corner ghosts of a physical side from the neighbour that owns
    them)"""
    ni, nj = 61, 47

    def code(r, gi, gj):
        return r * 1e6 + gj * 1000.0 + gi

    def extent(loc):  # global cells a rank owns, (i0, i1, j0, j1) inclusive
        nb = list(loc.neighbours)
        return (loc.ioff + (0 if nb[0] < 0 else 1), loc.ioff + loc.ni + (1 if nb[1] < 0 else 0),
                loc.joff + (0 if nb[2] < 0 else 1), loc.joff + loc.nj + (1 if nb[3] < 0 else 0))

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-6, 10, device=0, nranks=world, rank=r,
                    dims=dims, comm_id=cid) as g:
            loc = g.loc
            i0, i1, j0, j1 = extent(loc)
            jj, ii = np.mgrid[0:loc.nj + 2, 0:loc.ni + 2]
            gi, gj = loc.ioff + ii, loc.joff + jj
            mine = (gi >= i0) & (gi <= i1) & (gj >= j0) & (gj <= j1)
            a = np.where(mine, code(r, gi, gj), -1.0)
            g.upload(M.U, a)
            g.exchange(M.U, depth)
            return loc, g.download(M.U)

    outs = run_ranks(world, rank_fn, dims)
    ext = [extent(o[0]) for o in outs]
    for r, (loc, got) in enumerate(outs):
        for j in range(loc.nj + 2):
            for i in range(loc.ni + 2):
                gi, gj = loc.ioff + i, loc.joff + j
                own = [q for q, (a0, a1, b0, b1) in enumerate(ext)
                       if a0 <= gi <= a1 and b0 <= gj <= b1]
                assert len(own) == 1, (gi, gj, own)
                assert got[j, i] == code(own[0], gi, gj), (r, i, j, got[j, i], own[0])


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("T", [1, 4, 8])
def test_halo_after_solve(world, T):
    """A solve leaves the final field's halo to its next reader (misor_api.hip
    p_halo): a download of p after a decomposed solve holds, in every cell of
    the 2-deep halo, the neighbour's new value -- the whole local window of the
    oracle's field, ghosts included -- and so does adaptUV's read of it (the
    NS tests)"""
    ni, nj = 300, 190
    rng = np.random.default_rng(world * 10 + T)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    want = p.copy()
    orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.9, 1e-300, 2 * T + 1)

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.9, 1e-300, 2 * T + 1, device=0, nranks=world,
                    rank=r, comm_id=cid) as g:
            g.set_tuning(M.TUNE_TSTEPS, T)
            g.upload(M.P, local_window(p, g.loc))
            g.upload(M.RHS, local_window(rhs, g.loc))
            it, _ = g.solve_rb()
            return g.loc, g.download(M.P), it

    for loc, blk, it in run_ranks(world, rank_fn):
        assert it == 2 * T + 1
        w = local_window(want, loc)
        # rows / columns 0 and n+1 of the window: the physical ghost copy or
        # the neighbour's cells (the window's four corners left out)
        assert np.array_equal(blk[1:-1, :], w[1:-1, :]), (loc.ioff, loc.joff)
        assert np.array_equal(blk[:, 1:-1], w[:, 1:-1]), (loc.ioff, loc.joff)


@pytest.mark.parametrize("world", [2, 4])
def test_part2_on_comm_stream(world):
    """The pipelined loop's part 2 (on the communication stream right behind
    its exchange) gives the oracle's field, bit for bit, over several passes
    and a partial last one"""
    ni, nj, T = 420, 260, 4
    sweeps = 3 * T + 1
    rng = np.random.default_rng(world * 7 + 1)
    p = rng.standard_normal((nj + 2, ni + 2))
    rhs = rng.standard_normal((nj + 2, ni + 2))
    want = p.copy()
    orc.solve_rb(want, rhs, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, sweeps)

    def rank_fn(r, cid, dims):
        with M.Grid(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, sweeps, device=0, nranks=world,
                    rank=r, comm_id=cid) as g:
            g.set_tuning(M.TUNE_TSTEPS, T)
            assert g.get_tuning(M.TUNE_OVERLAP) == 1
            g.upload(M.P, local_window(p, g.loc))
            g.upload(M.RHS, local_window(rhs, g.loc))
            it, _ = g.solve_rb()
            return g.loc, g.download(M.P), it

    for loc, blk, it in run_ranks(world, rank_fn):
        assert it == sweeps
        w = local_window(want, loc)
        assert np.array_equal(blk[1:-1, 1:-1], w[1:-1, 1:-1]), (loc.ioff, loc.joff)
