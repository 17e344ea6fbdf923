"""Multi-rank CPU model of the decomposed 3D solve (gloo, world 2 and 3).

The algorithm libmisor runs for assignment-6's 3D solve over RCCL (DESIGN.md
6b), restated on the CPU with numpy in the reference's expression order:
slabs of planes along k (misor3_decompose); per iteration
  1. red update of the owned planes PLUS the halo planes a neighbour owns
     (recomputed redundantly from the 2-deep halo), global colours i+j+k;
  2. black update of the owned planes;
  3. Neumann face copy: x and y faces everywhere, k faces on physical sides;
  4. sum of r^2 over owned cells, all-reduced; res = (res + sum) / N;
  5. 2-deep halo exchange of p (whole planes).
The gathered p must equal the single-domain 3D oracle (oracle/oracle3d.c, the
restatement pinned to assignment-6's own build) bit for bit with the same
iteration count.
"""
import os
import queue
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import orc3
import pymisor as M

H = 2


def colour_update(p, rhs, planes, I, J, colour, gk0, idx2, idy2, idz2, factor):
    """update the cells of one colour (0: i+j+k odd = the reference's pass 0)
    on local planes `planes` (storage index = local k + H - 1); returns sum r^2
    over the mask `own` planes handled by the caller"""
    sums = {}
    for lk in planes:
        s = lk + H - 1
        c = p[s, 1:J + 1, 1:I + 1]
        tx = (p[s, 1:J + 1, 2:I + 2] - 2.0 * c) + p[s, 1:J + 1, 0:I]
        ty = (p[s, 2:J + 2, 1:I + 1] - 2.0 * c) + p[s, 0:J, 1:I + 1]
        tz = (p[s + 1, 1:J + 1, 1:I + 1] - 2.0 * c) + p[s - 1, 1:J + 1, 1:I + 1]
        r = rhs[s, 1:J + 1, 1:I + 1] - ((tx * idx2 + ty * idy2) + tz * idz2)
        jj, ii = np.meshgrid(np.arange(1, J + 1), np.arange(1, I + 1), indexing="ij")
        mask = ((ii + jj + gk0 + lk) & 1) == (1 if colour == 0 else 0)
        new = c - (factor * r)
        p[s, 1:J + 1, 1:I + 1] = np.where(mask, new, c)
        sums[lk] = float(np.sum(np.where(mask, r * r, 0.0)))
    return sums


def worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I, J, K, itermax, eps, seed = case
        rng = np.random.default_rng(seed)
        pg = rng.standard_normal((K + 2, J + 2, I + 2))
        rhsg = rng.standard_normal((K + 2, J + 2, I + 2))
        dx, dy, dz, omega = 1.0 / I, 1.0 / J, 1.0 / K, 1.8
        dx2, dy2, dz2 = dx * dx, dy * dy, dz * dz
        idx2, idy2, idz2 = 1.0 / dx2, 1.0 / dy2, 1.0 / dz2
        factor = omega * 0.5 * (dx2 * dy2 * dz2) / (dy2 * dz2 + dx2 * dz2 + dx2 * dy2)
        kl, ko = M.decompose3(world, rank, K)
        lo, hi = rank == 0, rank == world - 1
        # storage planes -1 .. kl+2 (local k), global plane = ko + local k
        p = np.zeros((kl + 2 * H, J + 2, I + 2))
        rhs = np.zeros_like(p)
        for lk in range(-1, kl + 3):
            gk = ko + lk
            if 0 <= gk <= K + 1:
                p[lk + H - 1] = pg[gk]
                rhs[lk + H - 1] = rhsg[gk]

        def exchange():
            own_lo = 0 if lo else 1
            own_hi = kl + 1 if hi else kl
            mine = (ko + own_lo, p[own_lo + H - 1:own_hi + H].copy())
            allv = [None] * world
            dist.all_gather_object(allv, mine)
            glob = {}
            for (g0, blk) in allv:
                for t in range(blk.shape[0]):
                    glob[g0 + t] = blk[t]
            for lk in list(range(-1, own_lo)) + list(range(own_hi + 1, kl + 3)):
                if ko + lk in glob:
                    p[lk + H - 1] = glob[ko + lk]

        red_planes = range(1 if lo else 0, kl + 1 if hi else kl + 2)
        it, res = 0, 1.0
        while res >= eps * eps and it < itermax:
            s_red = colour_update(p, rhs, red_planes, I, J, 0, ko, idx2, idy2, idz2, factor)
            s_blk = colour_update(p, rhs, range(1, kl + 1), I, J, 1, ko, idx2, idy2, idz2,
                                  factor)
            # face copy: x, y faces of owned planes; k faces on physical sides
            for lk in range(1, kl + 1):
                s = lk + H - 1
                p[s, 1:J + 1, 0] = p[s, 1:J + 1, 1]
                p[s, 1:J + 1, I + 1] = p[s, 1:J + 1, I]
                p[s, 0, 1:I + 1] = p[s, 1, 1:I + 1]
                p[s, J + 1, 1:I + 1] = p[s, J, 1:I + 1]
            if lo:
                p[H - 1 + 0, 1:J + 1, 1:I + 1] = p[H - 1 + 1, 1:J + 1, 1:I + 1]
            if hi:
                p[H - 1 + kl + 1, 1:J + 1, 1:I + 1] = p[H - 1 + kl, 1:J + 1, 1:I + 1]
            local = sum(s_red[lk] for lk in range(1, kl + 1)) + sum(s_blk.values())
            allres = [None] * world
            dist.all_gather_object(allres, local)
            res = (res + sum(allres)) / (I * J * K)
            it += 1
            exchange()
        own_lo = 0 if lo else 1
        own_hi = kl + 1 if hi else kl
        allv = [None] * world
        dist.all_gather_object(allv, (ko + own_lo, p[own_lo + H - 1:own_hi + H].copy()))
        if rank == 0:
            glob = pg.copy()
            for (g0, blk) in allv:
                glob[g0:g0 + blk.shape[0]] = blk
            q.put((it, res, glob))
    finally:
        dist.destroy_process_group()


CASES = [(9, 7, 10, 6, 1e-300, 1), (12, 8, 13, 5, 1e-300, 2)]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES)
def test_decomposed_3d_equals_single_domain(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000) + world * 11 + case[-1]
    procs = [ctx.Process(target=worker, args=(r, world, port, case, q)) for r in range(world)]
    for pr in procs:
        pr.start()
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

    I, J, K, itermax, eps, seed = case
    rng = np.random.default_rng(seed)
    prm = dict(imax=I, jmax=J, kmax=K, xlength=1.0, ylength=1.0, zlength=1.0, re=100.0,
               gamma=0.9, tau=0.5, omg=1.8, eps=eps, itermax=itermax, gx=0.0, gy=0.0,
               gz=0.0, dt=0.0, te=0.0, bcLeft=1, bcRight=1, bcBottom=1, bcTop=1, bcFront=1,
               bcBack=1, name="dcavity")
    ns = orc3.NS3(prm)
    ns.p[...] = rng.standard_normal((K + 2, J + 2, I + 2))
    ns.rhs[...] = rng.standard_normal((K + 2, J + 2, I + 2))
    it_ref, res_ref = ns.solve()
    assert it == it_ref == itermax
    assert np.array_equal(glob, ns.p)
    assert res == pytest.approx(res_ref, rel=1e-12)
