"""Python replay of the NS time loop (assignment-5/sequential/src/main.c:37-60)
on the libmisor C ABI, for the GPU parity tests.  The product driver is the C
host program (practical-parallel-algorithms-with-mpi_amd/host/main_ns.c); this
mirror exists so tests can look at per-step iteration counts and fields."""
import numpy as np

import pymisor as M


def ns_grid(prm, device=0, nranks=1, rank=0, dims=(0, 0), comm_id=None):
    imax, jmax = int(prm["imax"]), int(prm["jmax"])
    dx, dy = prm["xlength"] / imax, prm["ylength"] / jmax
    g = M.Grid(imax, jmax, dx, dy, prm["omg"], prm["eps"], int(prm["itermax"]), device=device,
               nranks=nranks, rank=rank, dims=dims, comm_id=comm_id)
    g.ns_setup(prm)
    g.fill(M.U, prm["u_init"])
    g.fill(M.V, prm["v_init"])
    g.fill(M.P, prm["p_init"])
    g.set_dt(prm["dt"])
    return g


def dt_bound(prm):
    """initSolver, assignment-5/sequential/src/solver.c:113-116"""
    dx = prm["xlength"] / prm["imax"]
    dy = prm["ylength"] / prm["jmax"]
    inv = 1.0 / (dx * dx) + 1.0 / (dy * dy)
    return 0.5 * prm["re"] * 1.0 / inv


def run(g, prm, max_steps=-1, solver="rb"):
    """returns (steps, per-step iterations, t); solver "rb" = solveRB (the
    production path), "lex" = the reference's lexicographic `solve`
    (assignment-5/sequential/src/solver.c:140-191)"""
    tau, te = prm["tau"], prm["te"]
    dtb = dt_bound(prm)
    dt = prm["dt"]
    t, nt, iters = 0.0, 0, []
    while t <= te and (max_steps < 0 or nt < max_steps):
        if tau > 0.0:
            dt = g.compute_timestep(dtb, tau)
        g.call("set_boundary_conditions")
        g.call("set_special_boundary_condition")
        g.call("compute_fg")
        g.call("compute_rhs")
        if nt % 100 == 0:
            g.call("normalize_pressure")
        it, _ = g.solve_rb() if solver == "rb" else g.solve_lex(M.LEX_SEQ)
        iters.append(it)
        g.call("adapt_uv")
        t += dt
        nt += 1
    return nt, np.array(iters, dtype=np.int32), t
