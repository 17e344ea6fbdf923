"""Multi-rank CPU model of the decomposed red-black SOR (gloo, world 2 and 4).

This is the algorithm libmisor runs over RCCL (DESIGN.md "Multi-GPU"),
restated on the CPU with the oracle's arithmetic:
  per iteration
    1. 2-deep halo exchange of p with all 8 neighbours (here: every rank
       publishes the cells it owns -- interior + physical ghosts -- and reads
       its halo ring back from the owners);
    2. red pass over the owned cells PLUS the 1-deep halo ring on sides that
       have a neighbour (the neighbour's boundary red values, recomputed
       redundantly from the 2-deep halo: no second exchange per iteration);
    3. black pass over the owned cells;
    4. Neumann ghost copy on physical sides only (rows, then columns);
    5. allreduce of sum r^2 (owned cells), res = sum/(imax*jmax).
Decomposition from libmisor's host-only misor_decompose (MPI_Dims_create +
sizeOfRank rules).  Colour parity is GLOBAL (i+j).  The result must equal the
single-domain solveRB bit for bit with the same iteration count, for any
partition -- the property the GPU path relies on.
"""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import orc
import pymisor as M

H = 2  # halo depth


def owned_range(loc):
    """cells a rank is authoritative for: interior + ghost cells on physical sides"""
    nb = list(loc.neighbours)
    ilo = 0 if nb[0] < 0 else 1
    ihi = loc.ni + 1 if nb[1] < 0 else loc.ni
    jlo = 0 if nb[2] < 0 else 1
    jhi = loc.nj + 1 if nb[3] < 0 else loc.nj
    return ilo, ihi, jlo, jhi


def worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imax, jmax, dims, itermax, eps, seed = case
        rng = np.random.default_rng(seed)
        pg = rng.standard_normal((jmax + 2, imax + 2))
        rhsg = rng.standard_normal((jmax + 2, imax + 2)) * 50.0
        dx, dy, omega = 1.0 / imax, 1.5 / jmax, 1.8
        idx2, idy2, factor = orc.sor_constants(dx, dy, omega)

        loc = M.decompose(world, rank, imax, jmax, dims)
        ni, nj, io, jo = loc.ni, loc.nj, loc.ioff, loc.joff
        # local array with a 2-deep ring: local (li, lj) at [lj + H, li + H]
        shape = (nj + 2 + 2 * H, ni + 2 + 2 * H)
        p = np.zeros(shape)
        rhs = np.zeros(shape)

        def window(a_glob, a_loc):
            for lj in range(-H, nj + 2 + H - 1):
                gj = jo + lj
                if not (0 <= gj <= jmax + 1):
                    continue
                for li in range(-H, ni + 2 + H - 1):
                    gi = io + li
                    if 0 <= gi <= imax + 1:
                        a_loc[lj + H, li + H] = a_glob[gj, gi]

        window(pg, p)
        window(rhsg, rhs)
        ilo, ihi, jlo, jhi = owned_range(loc)
        nb = list(loc.neighbours)
        r_ilo = 1 if nb[0] < 0 else 0
        r_ihi = ni if nb[1] < 0 else ni + 1
        r_jlo = 1 if nb[2] < 0 else 0
        r_jhi = nj if nb[3] < 0 else nj + 1

        def exchange():
            own = p[jlo + H:jhi + H + 1, ilo + H:ihi + H + 1].copy()
            allv = [None] * world
            dist.all_gather_object(allv, (io + ilo, jo + jlo, own))
            glob = np.full((jmax + 2, imax + 2), np.nan)
            for (gi0, gj0, blk) in allv:
                glob[gj0:gj0 + blk.shape[0], gi0:gi0 + blk.shape[1]] = blk
            # refresh every non-owned cell of the local array that is a global cell
            for lj in range(-H, nj + 2 + H - 1):
                for li in range(-H, ni + 2 + H - 1):
                    if ilo <= li <= ihi and jlo <= lj <= jhi:
                        continue
                    gi, gj = io + li, jo + lj
                    if 0 <= gi <= imax + 1 and 0 <= gj <= jmax + 1:
                        p[lj + H, li + H] = glob[gj, gi]

        stride = shape[1]
        it, res = 0, 1.0
        while res >= eps * eps and it < itermax:
            exchange()
            s = orc.lib().orc_rb_pass_range(stride, H, r_ilo, r_ihi, r_jlo, r_jhi, 1, ni, 1,
                                            nj, io, jo, 0, idx2, idy2, factor,
                                            orc._ptr(p), orc._ptr(rhs))
            s += orc.lib().orc_rb_pass_range(stride, H, 1, ni, 1, nj, 1, ni, 1, nj, io, jo, 1,
                                             idx2, idy2, factor, orc._ptr(p), orc._ptr(rhs))
            # ghost copy on physical sides: rows first, then columns
            if nb[2] < 0:
                p[0 + H, 1 + H:ni + 1 + H] = p[1 + H, 1 + H:ni + 1 + H]
            if nb[3] < 0:
                p[nj + 1 + H, 1 + H:ni + 1 + H] = p[nj + H, 1 + H:ni + 1 + H]
            if nb[0] < 0:
                p[1 + H:nj + 1 + H, 0 + H] = p[1 + H:nj + 1 + H, 1 + H]
            if nb[1] < 0:
                p[1 + H:nj + 1 + H, ni + 1 + H] = p[1 + H:nj + 1 + H, ni + H]
            allres = [None] * world
            dist.all_gather_object(allres, s)
            res = sum(allres) / (imax * jmax)  # rank-order sum
            it += 1

        own = p[jlo + H:jhi + H + 1, ilo + H:ihi + H + 1].copy()
        allv = [None] * world
        dist.all_gather_object(allv, (io + ilo, jo + jlo, own))
        if rank == 0:
            glob = pg.copy()  # corners never change
            for (gi0, gj0, blk) in allv:
                glob[gj0:gj0 + blk.shape[0], gi0:gi0 + blk.shape[1]] = blk
            q.put((it, res, glob))
    finally:
        dist.destroy_process_group()


CASES = [
    # imax, jmax, dims, itermax, eps, seed
    (23, 17, (0, 0), 9, 1e-300, 1),
    (40, 31, (2, 1), 6, 1e-300, 2),
    (30, 30, (1, 2), 200, 1e-3, 3),
]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", CASES)
def test_decomposed_rb_equals_single_domain(world, case):
    imax, jmax, dims, itermax, eps, seed = case
    if world == 4 and dims != (0, 0):
        dims = (2, 2) if dims == (2, 1) else (1, 4)
    case = (imax, jmax, dims, itermax, eps, seed)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + world * 7 + seed
    procs = [ctx.Process(target=worker, args=(r, world, port, case, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    import queue
    import time
    t0 = time.time()
    while True:
        try:
            it, res, glob = q.get(timeout=2)
            break
        except queue.Empty:
            bad = [pr.exitcode for pr in procs if pr.exitcode not in (None, 0)]
            assert not bad and time.time() - t0 < 240, ("worker failed", bad)
    for pr in procs:
        pr.join(60)
        assert pr.exitcode == 0

    rng = np.random.default_rng(seed)
    p = rng.standard_normal((jmax + 2, imax + 2))
    rhs = rng.standard_normal((jmax + 2, imax + 2)) * 50.0
    it_ref, res_ref = orc.solve_rb(p, rhs, 1.0 / imax, 1.5 / jmax, 1.8, eps, itermax)
    assert it == it_ref
    assert np.array_equal(glob, p)
    assert abs(res - res_ref) <= 1e-12 * abs(res_ref)
