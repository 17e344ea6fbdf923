#!/usr/bin/env python3
"""Headline benchmark: red-black SOR MLUP/s + % of HBM roofline, 32768^2 grid
(BASELINE.json metric; SURVEY 8d config 4 -- strong scaling 1/2/4/8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 32768]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A "step" is one red+black SOR iteration (one fused sweep launch, the
reference's solveRB loop body, assignment-4/src/solver.c:197-234) over the
whole global grid.  The Poisson problem is assignment-4's problem 2 init
(p = sin(4 pi x) + sin(4 pi y), rhs = sin(2 pi x)), omega 1.9, with eps so
small that exactly K iterations run (convergence at 32768^2 needs ~2e8
sweeps).  Fields are initialised on the device before the timed
region; the timed region is K iterations, barrier + device sync on both
sides, max over ranks.  Rank 0 prints ONE JSON line.

A launch (a "pass") of the default temporally blocked kernel performs T
complete iterations (sor_tb.hip; T = iters_per_pass): it reads p and rhs once
and writes p once per T iterations.

roofline (the binding roof, frac <= 1): the algorithmic HBM bytes of ONE pass
are 24 B per cell (read p, read rhs, write p: SURVEY 8d's 24 B/LUP with the
T iterations of the pass sharing one read/write of the fields), so achieved =
24 B x local cells / the kernel's average launch duration, measured with HIP
events recorded around every pass on the library's stream
(misor_enable_timing); peak = 8000 GB/s (MI355X HBM3E, MI355X_MICROARCH.md).
traffic = HBM bytes per launch from the PMC profile committed under profiles/
for this size and T (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
MI355X_MICROARCH.md) of every pass length the timed solve launches (its
pass split, in config.pass_split), weighted by launches, or null.
floors_ms: the launch's HBM floor (24 B x cells at 8 TB/s) and its FP64 VALU
floor (FP64 operations per lattice update of the form that runs -- 9 with the
power-of-two spacing identity, else 11 -- at 16 lanes/clk/SIMD x 1024 SIMDs x
2.4 GHz).  The iteration-equivalent
rate (24 B/LUP x T iterations / launch time, > 8 TB/s because T iterations
share one pass) is reported separately under iteration_equivalent.

Warm-up: besides --warmup iterations, every kernel instantiation the timed
region launches (T and the remainder steps % T) runs once before timing.

cpu_baseline: the reference's own solveRB (assignment-4/src/solver.c:179-238,
compiled in place by oracle/Makefile into oracle/_ref/libref.so) on one host
core, on the bench's own 32768^2 grid (the device's fields after the timed
solve), 3 sweeps per run, best of 3 runs and their median,
the solve timed alone; falls back to the C restatement
(oracle/liboracle.so, kind "port") when _ref is absent.
cpu_baseline_multicore: the restatement over the cores the job is granted
(pthreads over row bands), same grid, 10 sweeps per run, best of 3 and median.
cpu_baseline_mpi: the reference's own MPI pressure solve
(assignment-5/skeleton/src/solver.c:586-661: a halo exchange and a residual
MPI_Allreduce per iteration; compiled from its sources with MPICH by
oracle/Makefile `mpi`) under mpirun on the granted host cores, 8192^2, best
of 3 and median; {"mpi": "absent"} where mpirun or the build is missing.
The CPU baselines run on rank 0 at every N (rank 0's own block at N > 1).

N > 1: one process per GPU.  Under torch.distributed.run (the driver) the
launcher's RANK / LOCAL_RANK / WORLD_SIZE are used and WORLD_SIZE must equal
--gpus (else exit 2); without a launcher, --gpus N > 1 spawns the N workers
itself (this parent never touches the GPU: each worker selects its device
before its first GPU call) and exits with their worst status.  Before timing,
every N > 1 run solves a 2048^2 grid decomposed over the same ranks, gathers p
on rank 0 and compares it bit for bit with a single-domain solve there
(`parity`); `rccl_ranks` is the rank count of the bench grid's communicator
as RCCL reports it (ncclCommCount).  --dry-run stops each worker before any
GPU call and prints the rank assignment (tests/test_bench_cpu.py).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

PEAK_GBS = 8000.0
BYTES_PER_LUP = 24.0
# waves each SIMD runs of the temporally blocked kernels (launch bounds)
WAVES_PER_SIMD = {"rb_tb_kernel": 2, "rb_tbc_kernel": 2, "rb_tbh_kernel": 2, "rb_tbhc_kernel": 2}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def runs_summary(vals):
    """best of the runs and their median"""
    v = sorted(vals)
    med = v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
    return v[-1], med


def cpu_baseline(p, rhs, sweeps=3, runs=3):
    """The reference's own solveRB (assignment-4/src/solver.c:179-238, compiled
    in place by oracle/Makefile into oracle/_ref/libref.so) on one host core,
    on the bench's own grid: the fields the GPU holds after the timed solve,
    `sweeps` iterations per run, each run from its own copy of that field, the
    solve timed alone (init excluded, as assignment-4/src/main.c:33-35 times
    solve()); best of `runs` and their median.  Falls back to
    the C restatement (oracle/liboracle.so, kind "port") when _ref is absent."""
    import orc

    n = p.shape[1] - 2
    kind = "reference" if orc.have_ref() else "port"
    lup = float(n) * (p.shape[0] - 2) * sweeps
    rates, secs = [], []
    for _ in range(runs):
        q = p.copy()
        if kind == "reference":
            it, sec = orc.ref_solve_rb_arrays(q, rhs, 1.0 / n, 1.0 / n, 1.9, 1e-300, sweeps)
        else:
            t1 = time.perf_counter()
            it, _ = orc.solve_rb(q, rhs, 1.0 / n, 1.0 / n, 1.9, 1e-300, sweeps)
            sec = time.perf_counter() - t1
        del q
        assert it == sweeps
        rates.append(lup / sec / 1e6)
        secs.append(sec)
    best, med = runs_summary(rates)
    return {"value": round(best, 2), "median": round(med, 2), "runs": [round(r, 2) for r in rates],
            "unit": "MLUP/s", "cores": 1, "kind": kind, "cpu": cpu_model(),
            "sample": "solveRB on the bench's %dx%d grid (its fields after the timed solve), "
                      "%d sweeps per run, best of %d runs (%s s solve each, init excluded; "
                      "median in 'median'), 1 host core"
                      % (n, p.shape[0] - 2, sweeps, runs, "/".join("%.2f" % t for t in secs))}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        return None


def cpu_baseline_multicore(p, rhs, sweeps=10, runs=3):
    """solveRB on every host core the affinity mask allows (no MPI
    on the box, so pthreads over row bands, oracle/oracle_mt.c -- the
    restatement, p bit-identical to the single-core solve), on the bench's own
    grid; `sweeps` iterations per run, each from its own copy of the field,
    best of `runs` and their median"""
    import orc

    n = p.shape[1] - 2
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    # threads: the cores this process may actually run on at once -- the
    # affinity mask, capped by a cgroup CPU quota and by OMP_NUM_THREADS (the
    # GPU box shows its whole machine in the mask but grants a share of it,
    # which it states in OMP_NUM_THREADS; 256 threads there ran at 1.8x one)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = max(1, min(aff, 256, quota or 256, int(omp) if omp.isdigit() and int(omp) > 0 else 256))
    lup = float(n) * (p.shape[0] - 2) * sweeps
    rates, secs = [], []
    for _ in range(runs):
        q = p.copy()
        t1 = time.perf_counter()
        it, _ = orc.solve_rb_mt(q, rhs, 1.0 / n, 1.0 / n, 1.9, 1e-300, sweeps, threads)
        sec = time.perf_counter() - t1
        del q
        assert it == sweeps
        rates.append(lup / sec / 1e6)
        secs.append(sec)
    best, med = runs_summary(rates)
    return {"value": round(best, 1), "median": round(med, 1), "runs": [round(r, 1) for r in rates],
            "unit": "MLUP/s", "cores": threads,
            "kind": "port", "cpu": cpu_model(), "nproc": os.cpu_count(), "affinity": aff,
            "cgroup_cpus": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample": "solveRB on the bench's %dx%d grid, %d sweeps per run, best of %d runs "
                      "(%s s each; median in 'median'), %d threads over row bands "
                      "(oracle/oracle_mt.c); the GPU box lists its whole machine in the "
                      "affinity mask but grants this job a share of it (OMP_NUM_THREADS=%s)"
                      % (n, p.shape[0] - 2, sweeps, runs, "/".join("%.2f" % t for t in secs),
                         threads, os.environ.get("OMP_NUM_THREADS"))}


def pmc_summary(size, nranks, T, chain, kernel="rb_tb_kernel"):
    """The committed PMC summary (tools/pmc_summary.py) of the same launch shape
    -- size, ranks, iterations per pass, chained kernel or not -- or {} (the
    latest file in name order wins)."""
    best = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if (d.get("size") == size and d.get("nranks", 1) == nranks
                and d.get("iters_per_pass", 1) == T and "bytes_per_launch" in d
                and bool(d.get("chain", False)) == bool(chain)
                and ("::%s<" % kernel) in d.get("kernel", "::rb_tb_kernel<")):
            best = dict(d, file=os.path.basename(path))
    return best


def pass_split(steps, T):
    """Iterations of each pass of a solve capped at `steps` (misor_api.hip
    misor_solve_rb_n: ceil(steps / T) passes, as even as possible)"""
    n = -(-steps // T)
    base, extra = divmod(steps, n)
    return [base + 1] * extra + [base] * (n - extra)


# assignment-6/dcavity.par read as 2D, sizes set per GPU
DCAVITY = dict(name="dcavity", xlength=1.0, ylength=1.0, re=1000.0, gx=0.0, gy=0.0,
               u_init=0.0, v_init=0.0, p_init=0.0, dt=0.02, tau=0.5, eps=1e-3, omg=1.8,
               gamma=0.9, bcLeft=1, bcRight=1, bcBottom=1, bcTop=1)


def run_ns(args, world, rank, local_rank, dist, torch):
    """BASELINE config 5: dcavity NS weak scaling, size^2 cells per GPU, the
    pressure solve capped at --itermax iterations, fixed time steps.  A step is
    one time step of assignment-5/sequential/src/main.c:43-60 (dt all-reduce,
    BCs, computeFG, computeRHS, normalizePressure every 100 steps, solve,
    adaptUV) over the whole global grid."""
    import pymisor as M

    dims = list(M.decompose(world, 0, 1 << 20, 1 << 20).dims)
    imax, jmax = args.size * dims[0], args.size * dims[1]
    prm = dict(DCAVITY, imax=imax, jmax=jmax, itermax=args.itermax)
    dx, dy = prm["xlength"] / imax, prm["ylength"] / jmax
    comm_id = None
    if world > 1:
        obj = [M.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    g = M.Grid(imax, jmax, dx, dy, prm["omg"], prm["eps"], prm["itermax"], device=local_rank,
               nranks=world, rank=rank, comm_id=comm_id)
    if args.tb_variant >= 0:  # (the variant first: T = 10 needs the split ring)
        g.set_tuning(M.TUNE_TB_VARIANT, args.tb_variant)
    if args.tsteps > 0:
        g.set_tuning(M.TUNE_TSTEPS, args.tsteps)
    g.set_tuning(M.TUNE_RES_LITE, args.res_lite)
    g.ns_setup(prm)
    for f, v in ((M.U, prm["u_init"]), (M.V, prm["v_init"]), (M.P, prm["p_init"])):
        g.fill(f, v)
    g.set_dt(prm["dt"])
    inv = 1.0 / (dx * dx) + 1.0 / (dy * dy)
    dt_bound = 0.5 * prm["re"] * 1.0 / inv  # solver.c:113-116
    state = {"nt": 0, "iters": 0}

    def step():
        g.compute_timestep(dt_bound, prm["tau"])
        g.call("set_boundary_conditions")
        g.call("set_special_boundary_condition")
        g.call("compute_fg")
        g.call("compute_rhs")
        if state["nt"] % 100 == 0:
            g.call("normalize_pressure")
        it, _ = g.solve_rb()
        g.call("adapt_uv")
        state["nt"] += 1
        return it

    def barrier():
        torch.cuda.synchronize()
        g.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    g.enable_timing(True)
    g.reset_stats()
    barrier()
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        iters += step()
    barrier()
    elapsed = time.perf_counter() - t0
    st = g.stats()
    solve_ms = st["sweep_ms"]
    # per launch, HIP events on the library's stream: the solve's passes, the
    # fused computeFG + computeRHS, the fused adaptUV + max |u|, |v| partials
    pass_ms = st["sweep_ms"] / max(st["timed_passes"], 1)
    fg_ms = st["ns_ms"][0] / max(st["ns_calls"][0], 1)
    ad_ms = st["ns_ms"][1] / max(st["ns_calls"][1], 1)
    T_ns, passes_ns = st["iters_per_pass"], st["timed_passes"]
    # normalizePressure runs every 100 steps (main.c:49): in the warm-up step
    # 0, not in the timed steps -- timed here, after the timed region, on
    # the field the steps left (3 calls)
    g.reset_stats()
    for _ in range(3):
        g.call("normalize_pressure")
    g.synchronize()
    st2 = g.stats()
    norm_ms = st2["ns_ms"][2] / max(st2["ns_calls"][2], 1)
    if dist is not None:
        tt = torch.tensor([elapsed, solve_ms, pass_ms, fg_ms, ad_ms, norm_ms],
                          dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, solve_ms, pass_ms, fg_ms, ad_ms, norm_ms = tt.tolist()
    cells = float(imax) * float(jmax)
    out = {
        "metric": "dcavity NS weak scaling: pressure-solve MLUP/s within full time steps",
        "value": round(cells * iters / elapsed / 1e6, 1),
        "unit": "MLUP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (dcavity initial state u = v = p = 0, generated on device)",
        "config": {"workload": "2D NS lid-driven cavity (assignment-6 dcavity.par as 2D), "
                               "%dx%d global = %d^2 per GPU, pressure solve capped at %d "
                               "iterations, 1 time step = 1 step" % (imax, jmax, args.size,
                                                                       args.itermax),
                   "imax": imax, "jmax": jmax, "decomposition": "%dx%d" % tuple(dims),
                   "baseline_config": 5},
        "pressure_iterations": iters,
        "solve_kernel_ms_per_step": round(solve_ms / args.steps, 3),
        "other_ms_per_step": round(elapsed / args.steps * 1e3 - solve_ms / args.steps, 3),
    }
    # rooflines per launch (HBM, 8 TB/s): the dominant kernel -- the solve's
    # pass, 24 B per local cell (p in, rhs in, p out) -- and every streaming
    # kernel of the step with its algorithmic bytes per cell:
    # fg_rhs 40 (u, v in; f, g, rhs out), adapt_absmax 40 (f, g, p in; u, v
    # out), normalizePressure 32 (max |p| 8, exact sum 8, subtract 16).  traffic:
    # the committed PMC summary of this command (tools/ns_pmc_summary.py)
    lc = float(g.loc.ni) * float(g.loc.nj)
    pm = ns_pmc_summary(args.size, world)
    kp = pm.get("kernels", {})

    def roof(nbytes, ms, kname):
        ach = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else None
        tr = kp.get(kname, {}).get("bytes_per_launch")
        return {"bound": "hbm", "achieved": round(ach, 1) if ach else None, "peak": PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / PEAK_GBS, 4) if ach else None,
                "traffic": tr, "traffic_ratio": round(tr / nbytes, 4) if tr else None,
                "kernel_ms": round(ms, 4), "bytes_per_launch": nbytes}

    # the solve's passes: the register-ring kernel (T <= 8) or the split ring
    # (variant 13); the PMC summary's traffic applies only to its own kernel
    tbv_ns = st.get("tb_variant", 0)
    solve_kernel = "rb_tbhc_kernel" if tbv_ns == 13 else "rb_tb_kernel"
    if pm.get("solve_kernel") and pm.get("solve_kernel") != solve_kernel:
        kp = {k: v for k, v in kp.items() if k != pm.get("solve_kernel")}
    out["config"]["tb_variant"] = tbv_ns
    out["config"]["residual_lower_bounds"] = {"on": bool(g.get_tuning(M.TUNE_RES_LITE)),
                                              "misses": st.get("lite_misses", 0)}
    out["roofline"] = dict(roof(24.0 * lc, pass_ms, solve_kernel),
                           kernel="pressure solve pass (%s, %d iterations per pass, %d passes in "
                                  "the timed steps)" % (solve_kernel, T_ns, passes_ns))
    # the solve pass's VALU issue (SQ_ACTIVE_INST_VALU per wave x 2 waves per
    # SIMD, the committed PMC summary): >= 0.85 -- VALU-bound (the 10-iteration
    # split-ring passes, as the headline's)
    vb = kp.get(solve_kernel, {}).get("valu_busy_per_wave")
    if vb is not None:
        out["roofline"]["valu_busy_per_simd"] = round(2 * vb, 3)
        if 2 * vb >= 0.85:
            out["roofline"]["bound"] = "valu"
    out["kernels"] = {
        "fg_rhs_kernel": dict(roof(40.0 * lc, fg_ms, "fg_rhs_kernel"),
                              what="computeFG + computeRHS fused (solver.c:360-436, 122-138)"),
        "adapt_absmax_kernel": dict(roof(40.0 * lc, ad_ms, "adapt_absmax_kernel"),
                                    what="adaptUV + the next dt's max |u|, |v| (:438-455, "
                                         ":193-202)"),
        "normalize_pressure": dict(roof(32.0 * lc, norm_ms, "normalize_pressure"),
                                   what="normalizePressure (:204-217): absmax2 + exact_sum + "
                                        "sub_mean, timed after the timed steps (3 calls)"),
    }
    if pm:
        out["roofline"]["traffic_source"] = pm.get("file")
    if rank == 0 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline_ns(g.loc.ni, g.loc.nj)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    g.close()
    return out


def ns_pmc_summary(size, nranks):
    """the committed PMC summary of bench.py --workload ns at this size
    (tools/ns_pmc_summary.py), latest in name order, or {}"""
    best = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_ns*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("size") == size and d.get("nranks", 1) == nranks and "kernels" in d:
            best = dict(d, file=os.path.basename(path))
    return best


def cpu_baseline_ns(ni, nj, itermax=3, steps=1):
    """The reference's own NS step (assignment-5/sequential/src/main.c:43-60:
    computeTimestep, BCs, computeFG, computeRHS, normalizePressure, solveRB of
    assignment-4 -- the composed RB-NS oracle of SURVEY 0.4 -- and adaptUV;
    oracle/_ref/libref.so) on one host core, on the bench's dcavity grid
    (rank 0's block at N > 1), a bounded sample: `steps` step(s) with the
    solve capped at `itermax` iterations.  value = cells x iterations / step
    time of the sample; the solve's time per iteration and the rest of the
    step are reported beside it."""
    import orc

    if not orc.have_ref():
        return {"value": None, "kind": "reference", "error": "oracle/_ref/libref.so not built"}
    par = os.path.join(ROOT, "tests", "golden", "a6_dcavity.par")
    n, solve_s, step_s, sweeps = orc.ref_ns_timed(par, ni, nj, itermax, steps)
    cells = float(ni) * float(nj)
    per_it = solve_s / max(sweeps, 1)
    other = (step_s - solve_s) / max(n, 1)
    return {"value": round(cells * sweeps / step_s / 1e6, 2), "unit": "MLUP/s", "cores": 1,
            "kind": "reference", "cpu": cpu_model(),
            "solve_s_per_iteration": round(per_it, 4),
            "solve_MLUPs": round(cells / per_it / 1e6, 2),
            "other_s_per_step": round(other, 3),
            "sample": "the reference's NS step (sequential solver.c + assignment-4 solveRB, "
                      "oracle/_ref) on %dx%d dcavity, %d step(s) with the solve capped at %d "
                      "iterations (%.2f s; %.2f s of it in solveRB), 1 host core, "
                      "initSolver untimed" % (ni, nj, n, itermax, step_s, solve_s)}


# assignment-6/dcavity.par (the 3D solver's own configuration)
DCAVITY3D = dict(name="dcavity", xlength=1.0, ylength=1.0, zlength=1.0, re=1000.0, gx=0.0,
                 gy=0.0, gz=0.0, u_init=0.0, v_init=0.0, w_init=0.0, p_init=0.0, dt=0.02,
                 te=10.0, tau=0.5, itermax=1000, eps=1e-3, omg=1.8, gamma=0.9, bcLeft=1,
                 bcRight=1, bcBottom=1, bcTop=1, bcFront=1, bcBack=1)


def cpu_baseline3d(n, iters=100):
    """the reference's own 3D solve (assignment-6/src/solver.c:175-297 compiled
    in place, oracle/_ref/libref3d.so) on one host core, n^3 cells x `iters`
    iterations from a random state; None where the build is absent"""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import numpy as np
        import orc3
        if not orc3.have_ref3():
            return None
    except Exception as e:  # pragma: no cover
        log("cpu_baseline3d unavailable: %s" % e)
        return None
    import tempfile
    rng = np.random.default_rng(0)
    shape = (n + 2, n + 2, n + 2)
    st = {f: rng.standard_normal(shape) * 1e-3 for f in orc3.FIELDS}
    with tempfile.NamedTemporaryFile("w", suffix=".par", delete=False) as fh:
        fh.write("name dcavity\nimax %d\njmax %d\nkmax %d\nitermax %d\neps 1e-300\n"
                 "omg 1.8\nre 1000\n" % (n, n, n, iters))
        par = fh.name
    t0 = time.perf_counter()
    _, it = orc3.ref3_call(par, (0, 0, 0), "solve", 0.02, st)
    el = time.perf_counter() - t0
    os.unlink(par)
    return {"value": round(float(n) ** 3 * it / el / 1e6, 1), "unit": "MLUP/s", "cores": 1,
            "kind": "reference",
            "sample": "assignment-6 solve (oracle/_ref/libref3d.so), %d^3 cells x %d "
                      "iterations, random state" % (n, it)}


def run_ns3d(args, world, rank, local_rank, dist, torch):
    """assignment-6's 3D NS (dcavity.par) weak scaling: --size^3 cells per GPU,
    the global box size x size x (size*N) split into N slabs of planes (RCCL
    halos and residual all-reduce).  A step is one time step of
    assignment-6/src/main.c:45-60 over the whole box."""
    import pymisor as M

    n = args.size
    prm = dict(DCAVITY3D, imax=n, jmax=n, kmax=n * world, itermax=args.itermax or 1000)
    comm_id = None
    if world > 1:
        obj = [M.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    g = M.Grid3(prm, device=local_rank, nranks=world, rank=rank, comm_id=comm_id)
    for f, v in ((M.U3, prm["u_init"]), (M.V3, prm["v_init"]), (M.W3, prm["w_init"]),
                 (M.P3, prm["p_init"])):
        g.fill(f, v)
    g.set_dt(prm["dt"])

    def step():
        g.compute_timestep()
        for fn in ("set_boundary_conditions", "set_special_boundary_condition", "compute_fg",
                   "compute_rhs"):
            g.call(fn)
        it, _ = g.solve()
        g.call("adapt_uvw")
        return it

    def barrier():
        torch.cuda.synchronize()
        g.call("synchronize")
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    g.enable_timing(True)
    barrier()
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        iters += step()
    barrier()
    elapsed = time.perf_counter() - t0
    solve_ms, solve_iters = g.solve_time()
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.tolist()[0]
    cells = float(n) ** 3  # per GPU
    iters_all = iters * world  # every rank runs the same iterations over its slab
    out = {
        "metric": "3D dcavity NS (assignment-6): pressure-solve MLUP/s within full time steps",
        "value": round(cells * iters_all / elapsed / 1e6, 1),
        "unit": "MLUP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (dcavity initial state u = v = w = p = 0, generated on device)",
        "config": {"workload": "3D NS lid-driven cavity (assignment-6 dcavity.par), %d^3 "
                               "cells per GPU, %dx%dx%d global in %d slabs along k, "
                               "1 time step = 1 step" % (n, n, n, n * world, world),
                   "imax": n, "jmax": n, "kmax": n * world, "itermax": prm["itermax"],
                   "decomposition": "%d slabs" % world},
        "pressure_iterations": iters,
    }
    if solve_ms > 0:
        # the solve's kernels (two colour passes + loop test per iteration),
        # HIP events on the library's stream; 24 B/LUP algorithmic (p in, rhs
        # in, p out), one LUP = one cell updated once
        ach = 24.0 * cells * solve_iters / (solve_ms / 1e3) / 1e9
        traffic = None
        for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc3d*.json"))):
            d = json.load(open(path))
            if d.get("size") == n and "bytes_per_launch" in d:
                traffic = d["bytes_per_launch"]
        fused = g.get_tuning(M.TUNE3_SWEEP) == 1
        resident = g.get_tuning(M.TUNE3_RESIDENT) == 1
        if resident:
            # p never leaves the CUs, so no HBM roofline applies; the 24 B/LUP
            # rate is kept under its own name as a streaming-equivalent rate
            out["roofline"] = {"bound": "latency/LDS", "achieved": None, "peak": 8000.0,
                               "unit": "GB/s", "frac": None, "traffic": None,
                               "streaming_equivalent_GBs": round(ach, 1),
                               "kernel": "3D solve: k3_resident1 (the whole solve in one "
                                         "cooperative launch, p resident in LDS, one grid "
                                         "barrier and one exchange per iteration)",
                               "solve_ms_per_iteration": round(solve_ms / solve_iters, 5)}
        else:
            out["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0,
                               "unit": "GB/s", "frac": round(ach / 8000.0, 4),
                               "traffic": traffic if fused else None,
                               "kernel": ("3D solve: k3_sweep (one fused red+black launch) + "
                                          "k3_finish per iteration" if fused else
                                          "3D solve: k3_rb_pass x2 + k3_finish per iteration"),
                               "solve_ms_per_iteration": round(solve_ms / solve_iters, 5)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline3d(min(n, 128))
    g.close()
    return out


def run_poisson_local(args, N):
    """The decomposed leg of the headline bench with N in-process ranks on ONE
    GPU (libmisor's LOCAL: transport, host threads of this process): the same
    Grid code, pass loop and comm timing as N processes over RCCL, so the
    N > 1 JSON line (comm block, overlap) is produced and checked where only
    one GPU exists.  Not a scaling measurement (the ranks share the GPU).
    --check: the gathered p after the timed solve against a 1-rank solve of
    the same iterations, bit for bit."""
    import threading

    import numpy as np
    import pymisor as M

    n = args.size
    pdims = list(M.decompose(N, 0, 1 << 20, 1 << 20).dims) if args.scaling == "weak" else [1, 1]
    imax, jmax = n * pdims[0], n * pdims[1]
    cid = ("LOCAL:bench%d" % os.getpid()).encode()
    bar = threading.Barrier(N)
    res = [None] * N
    err = []
    total_iters = max(args.warmup, 1) + 2 * args.steps

    def body(r):
        try:
            g = M.Grid(imax, jmax, 1.0 / n, 1.0 / n, 1.9, 1e-300, args.steps, device=0,
                       nranks=N, rank=r, comm_id=cid)
            if args.tsteps > 0:
                g.set_tuning(M.TUNE_TSTEPS, args.tsteps)
            g.poisson_init(float(pdims[0]), float(pdims[1]), 2)
            g.solve_rb(itermax=max(args.warmup, 1))
            g.solve_rb(itermax=args.steps)
            g.enable_timing(True)
            g.reset_stats()
            g.synchronize()
            bar.wait()
            t0 = time.perf_counter()
            it, _ = g.solve_rb(itermax=args.steps)
            g.synchronize()
            bar.wait()
            el = time.perf_counter() - t0
            st = g.stats()
            p = g.gather(M.P) if args.check else None
            res[r] = dict(it=it, el=el, st=st, p=p, dims=tuple(g.loc.dims),
                          cells=g.loc.ni * g.loc.nj, T=st["iters_per_pass"])
            g.close()
        except BaseException as e:  # surfaced in the main thread
            err.append((r, repr(e)))
            bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise RuntimeError("local ranks failed: %s" % err)
    assert all(x["it"] == args.steps for x in res)
    elapsed = max(x["el"] for x in res)
    passes = max(max(x["st"]["timed_passes"], 1) for x in res)
    kern_ms = max(x["st"]["sweep_ms"] / max(x["st"]["timed_passes"], 1) for x in res)
    halo = max(x["st"]["halo_ms"] / max(x["st"]["halos"], 1) for x in res)
    ared = max(x["st"]["allreduce_ms"] / max(x["st"]["allreduces"], 1) for x in res)
    comm = max((x["st"]["halo_ms"] + x["st"]["allreduce_ms"]) / passes for x in res)
    wall = elapsed * 1e3 / passes
    exposed = max(0.0, wall - kern_ms)
    out = {
        "metric": "red-black SOR MLUP/s + % HBM roofline at 1/2/4/8 MI355X, 32768^2 grid",
        "value": round(float(imax) * jmax * args.steps / elapsed / 1e6, 1),
        "unit": "MLUP/s", "n_gpus": 1, "local_ranks": N, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (assignment-4 problem-2 fields, generated on device)",
        "config": {"workload": "2D Poisson red-black SOR (solveRB), %dx%d interior cells, %d "
                               "in-process ranks on ONE GPU (plumbing check of the decomposed "
                               "path; not a scaling number)" % (imax, jmax, N),
                   "imax": imax, "jmax": jmax, "decomposition": "%dx%d" % res[0]["dims"],
                   "iters_per_pass": res[0]["T"], "baseline_config": 4},
        "comm": {"halo_ms_per_exchange": round(halo, 4), "allreduce_ms_per_call": round(ared, 4),
                 "sweep_ms_per_pass": round(kern_ms, 4), "wall_ms_per_pass": round(wall, 4),
                 "comm_ms_per_pass": round(comm, 4),
                 "overlap": round(1.0 - min(1.0, exposed / comm), 3) if comm > 0 else None,
                 "transport": "in-process LOCAL: device copies + events (stands in for RCCL)",
                 "note": "max over ranks; overlap = 1 - (wall - sweep span) / comm time per pass"},
    }
    if args.check:
        with M.Grid(imax, jmax, 1.0 / n, 1.0 / n, 1.9, 1e-300, total_iters, device=0) as g1:
            if args.tsteps > 0:
                g1.set_tuning(M.TUNE_TSTEPS, args.tsteps)
            g1.poisson_init(float(pdims[0]), float(pdims[1]), 2)
            it1, _ = g1.solve_rb(itermax=total_iters)
            ref = g1.download(M.P)
        same = bool(np.array_equal(res[0]["p"], ref)) and it1 == total_iters
        out["check"] = {"iterations": total_iters, "p_bit_identical_to_1_rank": same}
    return out


def spawn_workers(n, dry_run):
    """--gpus N > 1 without a launcher: start N workers of this script with the
    environment torch.distributed.run would give them (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT).  This process never
    imports torch or touches the GPU; it waits for the workers, stops the rest
    when one fails, and returns their worst exit status.  Rank 0's stdout is
    this script's stdout (the JSON line), the other ranks' goes to stderr; with
    --dry-run every worker's line is collected into one JSON line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        out = subprocess.PIPE if dry_run else (None if r == 0 else sys.stderr)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=out))
    rcs = [None] * n
    outs = [b""] * n
    if dry_run:
        for r, p in enumerate(procs):
            outs[r], _ = p.communicate(timeout=120)
            rcs[r] = p.returncode
    else:
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
            if any(rc not in (None, 0) for rc in rcs):  # one failed: stop the others
                for r, p in enumerate(procs):
                    if rcs[r] is None:
                        p.terminate()
                for r, p in enumerate(procs):
                    if rcs[r] is None:
                        try:
                            rcs[r] = p.wait(timeout=30)
                        except subprocess.TimeoutExpired:
                            p.kill()
                            rcs[r] = p.wait()
                break
            time.sleep(0.2)
    worst = max((abs(rc) for rc in rcs), default=0)
    if dry_run:
        workers = [json.loads(o.decode().strip().splitlines()[-1]) for o in outs if o.strip()]
        print(json.dumps({"dry_run": True, "spawned": n, "master_port": port,
                          "exit_codes": rcs, "workers": workers}), flush=True)
    elif worst:
        log("bench workers exited with %s" % rcs)
    return worst


def parity_check(world, rank, local_rank, dist, n=2048, iters=30):
    """Before timing an N > 1 run: a n^2 problem-2 solve of `iters` iterations
    decomposed over the same ranks (its own RCCL communicator), p gathered on
    rank 0 (misor_gather, the skeleton's collectResult) and compared bit for
    bit with a single-domain solve of the same grid on rank 0's GPU, with the
    iteration counts and residuals.  Returns the record on rank 0, else None."""
    import numpy as np
    import pymisor as M

    obj = [M.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    g = M.Grid(n, n, 1.0 / n, 1.0 / n, 1.9, 1e-300, iters, device=local_rank, nranks=world,
               rank=rank, comm_id=obj[0])
    g.poisson_init(1.0, 1.0, 2)
    it, res = g.solve_rb()
    nr = g.comm_ranks()
    dims = "%dx%d" % tuple(g.loc.dims)
    p = g.gather(M.P)
    g.close()
    if rank != 0:
        return None
    with M.Grid(n, n, 1.0 / n, 1.0 / n, 1.9, 1e-300, iters, device=local_rank) as g1:
        g1.poisson_init(1.0, 1.0, 2)
        it1, res1 = g1.solve_rb()
        ref = g1.download(M.P)
    same = bool(np.array_equal(p, ref))
    return {"grid": "%dx%d" % (n, n), "decomposition": dims, "iterations": [it, it1],
            "p_bit_identical_to_1_rank": same and it == it1,
            "res_rel_diff": abs(res - res1) / abs(res1) if res1 else abs(res - res1),
            "rccl_ranks": nr,
            "note": "gathered p of the decomposed RCCL solve vs a single-domain solve on rank 0, "
                    "before the timed region"}


def cpu_baseline_mpi(cores, n=8192, sweeps=50, runs=3):
    """The reference's MPI pressure solve (assignment-5/skeleton/src/solver.c:
    586-661: per iteration an exchange of p, MPI_Neighbor_alltoallw :155, a
    lexicographic sweep and MPI_Allreduce of the residual :651), built from its
    own sources with MPICH (oracle/Makefile `mpi`, driver oracle/ref_mpi_glue.c),
    under mpirun with `cores` ranks on this host, n^2 problem-2 fields, `sweeps`
    iterations per run; the north star's communication-pattern CPU baseline.
    {"mpi": "absent"} when mpirun or the build is missing."""
    import shutil
    import subprocess

    exe = os.path.join(ROOT, "oracle", "_ref", "ref-skel-solve")
    mpirun = "/opt/conda/bin/mpirun" if os.path.exists("/opt/conda/bin/mpirun") else \
        shutil.which("mpirun")
    if not mpirun or not os.path.exists(exe):
        return {"value": None, "mpi": "absent",
                "mpirun": mpirun, "build": os.path.exists(exe)}
    cmd = [mpirun, "-launcher", "fork", "-np", str(cores), exe, str(n), str(n), str(sweeps),
           str(runs)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp")
    if r.returncode != 0:
        return {"value": None, "mpi": mpirun, "error": (r.stderr or r.stdout)[-400:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": d["mlups_best"], "median": d["mlups_median"], "unit": "MLUP/s",
            "cores": cores, "ranks": d["ranks"], "dims": d["dims"], "kind": "reference",
            "mpi": mpirun, "cpu": cpu_model(),
            "sample": "assignment-5/skeleton solve (lexicographic SOR, halo exchange + "
                      "MPI_Allreduce every iteration) on %dx%d, %d sweeps per run, best of %d "
                      "(%.2f s; median %.2f s), mpirun -np %d (MPICH, one rank per core)"
                      % (n, n, sweeps, runs, d["best_s"], d["median_s"], cores)}


def granted_cores():
    """the cores this process may run on at once: the affinity mask capped by a
    cgroup CPU quota and OMP_NUM_THREADS (the GPU box lists its whole machine in
    the mask but grants a share of it, stated in OMP_NUM_THREADS)"""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(aff, 256, quota or 256, int(omp) if omp.isdigit() and int(omp) > 0 else 256))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=140)
    ap.add_argument("--warmup", type=int, default=7)
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tsteps", type=int, default=0,
                    help="iterations per kernel launch (0: library default)")
    ap.add_argument("--tb-variant", type=int, default=-1,
                    help="temporally blocked kernel variant (-1: library default)")
    ap.add_argument("--res-lite", type=int, choices=(0, 1), default=1,
                    help="residual lower bounds of the 10-iteration passes (MISOR_TUNE_RES_LITE; "
                         "0: every iteration's residual counted in full, for A/B)")
    ap.add_argument("--workload", choices=("poisson", "ns", "ns3d"), default="poisson",
                    help="poisson: the headline metric (config 4); ns: config 5, "
                         "dcavity NS weak scaling (--size cells^2 per GPU); ns3d: "
                         "assignment-6's 3D dcavity (--size cells^3, default 128)")
    ap.add_argument("--itermax", type=int, default=0,
                    help="ns: pressure-solve cap (default 100); ns3d: default 1000 (.par)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="poisson: strong (default: the --size^2 grid split over the GPUs, "
                         "BASELINE config 4) or weak (--size^2 cells per GPU: the global grid "
                         "is the process grid times --size^2, same spacing 1/--size)")
    ap.add_argument("--local-ranks", type=int, default=0,
                    help="poisson, one process: N in-process ranks on this one GPU (the "
                         "decomposed path's plumbing; not a scaling measurement)")
    ap.add_argument("--check", action="store_true",
                    help="with --local-ranks: gathered p bit for bit against one rank")
    ap.add_argument("--dry-run", action="store_true",
                    help="stop before any GPU call; print this worker's rank assignment")
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip the pre-timing 2048^2 decomposed-vs-single parity solve")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process spawns the N workers and never touches the GPU
        sys.exit(spawn_workers(args.gpus, args.dry_run))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("error: WORLD_SIZE=%d but --gpus %d: launch one process per GPU "
            "(torch.distributed.run --nproc-per-node %d, or no launcher at all)"
            % (world, args.gpus, args.gpus))
        sys.exit(2)
    if args.dry_run:
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world_size": world,
                          "gpus": args.gpus, "master_addr": os.environ.get("MASTER_ADDR"),
                          "master_port": os.environ.get("MASTER_PORT"),
                          "device": "cuda:%d" % local_rank}), flush=True)
        return

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    if args.workload in ("ns", "ns3d"):
        if args.size == 32768 and "--size" not in sys.argv:
            args.size = 16384 if args.workload == "ns" else 128
        if args.workload == "ns":
            args.itermax = args.itermax or 100
            out = run_ns(args, world, rank, local_rank, dist, torch)
        else:
            out = run_ns3d(args, world, rank, local_rank, dist, torch)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps(out), flush=True)
        return

    if args.local_ranks > 1 and world == 1:
        out = run_poisson_local(args, args.local_ranks)
        print(json.dumps(out), flush=True)
        return

    import pymisor as M

    n = args.size
    # strong: n^2 over all GPUs; weak: n^2 per GPU, the process grid's extent
    # in cells, on a domain of dims[0] x dims[1] unit squares (spacing 1/n
    # either way, so the power-of-two form of the sweep applies to both)
    pdims = list(M.decompose(world, 0, 1 << 20, 1 << 20).dims) if args.scaling == "weak" \
        else [1, 1]
    imax, jmax = n * pdims[0], n * pdims[1]
    comm_id = None
    if world > 1:
        obj = [M.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    g = M.Grid(imax, jmax, 1.0 / n, 1.0 / n, 1.9, 1e-300, args.steps, device=local_rank,
               nranks=world, rank=rank, comm_id=comm_id)
    if args.tb_variant >= 0:
        g.set_tuning(M.TUNE_TB_VARIANT, args.tb_variant)
    if args.tsteps > 0:
        g.set_tuning(M.TUNE_TSTEPS, args.tsteps)
    g.set_tuning(M.TUNE_RES_LITE, args.res_lite)
    g.poisson_init(float(pdims[0]), float(pdims[1]), 2)
    local_cells = g.loc.ni * g.loc.nj
    rccl_ranks = g.comm_ranks() if world > 1 else None
    parity = None
    if world > 1 and not args.no_parity:
        parity = parity_check(world, rank, local_rank, dist)

    def barrier():
        torch.cuda.synchronize()
        g.synchronize()
        if dist is not None:
            dist.barrier()

    # warm-up: --warmup iterations, then a solve of the timed length, so every
    # kernel instantiation the timed solve launches has run once (the library
    # splits a capped solve into passes of as even a length as it can)
    g.solve_rb(itermax=max(args.warmup, 1))
    g.solve_rb(itermax=args.steps)
    g.enable_timing(True)
    g.reset_stats()
    barrier()
    t0 = time.perf_counter()
    it, res = g.solve_rb(itermax=args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    st = g.stats()
    assert it == args.steps, (it, args.steps)

    T = st["iters_per_pass"]
    # per launch (pass) of the sweep kernel, HIP events on the library's stream;
    # iterations per launch averaged over the timed launches (a capped solve's
    # last pass runs only the remaining iterations when --steps % T != 0)
    passes = max(st["timed_passes"], 1)
    iters_launch = st["timed_sweeps"] / passes
    if dist is not None:
        tt = torch.tensor([elapsed, st["sweep_ms"] / passes],
                          dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = tt.tolist()
    else:
        kern_ms = st["sweep_ms"] / passes

    total_lup = float(imax) * float(jmax) * args.steps
    mlups = total_lup / elapsed / 1e6
    # one pass moves at least p in, rhs in, p out: 24 B per local cell
    hbm_min = BYTES_PER_LUP * local_cells
    achieved = hbm_min / (kern_ms * 1e-3) / 1e9  # GB/s per GPU
    iter_eq = hbm_min * iters_launch / (kern_ms * 1e-3) / 1e9
    # FP64 operations per update of the form the kernel runs: 11 in the
    # reference's expression, 9 with the power-of-two spacing identity
    # (sor_tb.h resid<true>, used when 1/dx^2 == 1/dy^2 == 2^m, m >= 1)
    idx2, idy2 = 1.0 / (1.0 / n) ** 2, 1.0 / (1.0 / n) ** 2
    pow2 = idx2 == idy2 and math.frexp(idx2)[0] == 0.5 and idx2 >= 2.0 and T > 1
    fp64_ops = 9 if pow2 else 11
    fp64_floor_ms = fp64_ops * local_cells * iters_launch / (16 * 1024 * 2.4e9) * 1e3
    dims = "%dx%d" % tuple(g.loc.dims)
    chain = T > 1 and st.get("chained", 0) == 1
    split = pass_split(args.steps, T)
    if len(split) != st["timed_passes"]:
        split = None
    # the passes' kernel: the library's pass plan picks the split-ring kernel
    # (TB variants 12 / 13, sor_tbh.h) for short capped solves (misor_api.hip)
    tbv = st.get("tb_variant", 0)
    kernel = (("rb_tbhc_kernel" if chain else "rb_tbh_kernel") if tbv in (12, 13) else
              "rb_tbc_kernel" if chain else "rb_tb_kernel") if T > 1 else "rb_sweep_kernel"
    # traffic / VALU of the timed launches: the committed PMC summaries of each
    # pass length the split contains, weighted by its launches (null if one is
    # missing)
    traffic, valu, pmc_files = None, None, []
    if split:
        pm = {t: pmc_summary(n, world, t, chain, kernel) for t in set(split)}
        if all(pm[t] for t in pm):
            traffic = sum(pm[t]["bytes_per_launch"] for t in split) / len(split)
            pmc_files = sorted(pm[t]["file"] for t in pm)
            if all(pm[t].get("sq", {}).get("valu_insts") for t in pm):
                valu = {"insts_per_launch": sum(pm[t]["sq"]["valu_insts"] for t in split) /
                        len(split),
                        "valu_busy_per_wave": round(sum(pm[t]["sq"].get("active_inst_valu", 0)
                                                        for t in split) / len(split), 3),
                        "source": "PMC summaries of the same launch shapes: " +
                                  ", ".join(pmc_files)}
    if split:
        counts = {t: split.count(t) for t in sorted(set(split), reverse=True)}
        split_txt = " + ".join("%d x %d" % (c, t) for t, c in counts.items())
    else:
        split_txt = "%d" % T
    out = {
        "metric": "red-black SOR MLUP/s + % HBM roofline at 1/2/4/8 MI355X, 32768^2 grid",
        "value": round(mlups, 1),
        "unit": "MLUP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (assignment-4 problem-2 fields, generated on device)",
        "config": {"workload": "2D Poisson red-black SOR (solveRB), %dx%d interior cells, "
                               "fixed %d iterations per timed region, 1 iteration = 1 step, "
                               "passes (kernel launches) of %s iterations" % (
                                   imax, jmax, args.steps, split_txt),
                   "iters_per_pass": T, "pass_split": split, "tb_variant": tbv,
                   "imax": imax, "jmax": jmax, "omega": 1.9, "problem": 2,
                   "decomposition": dims, "baseline_config": 4,
                   # the 10-iteration passes' residual lower bounds (MISOR_TUNE_RES_LITE):
                   # same p / iterations / res bits; misses = solves that fell back
                   "residual_lower_bounds": {"on": bool(g.get_tuning(M.TUNE_RES_LITE)),
                                             "misses": st.get("lite_misses", 0)}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_ratio": round(traffic / hbm_min, 4) if traffic else None,
                     "kernel": kernel,
                     "iters_per_launch": round(iters_launch, 3), "kernel_ms": round(kern_ms, 4),
                     "bytes_per_launch": hbm_min,
                     "floors_ms": {"hbm": round(hbm_min / (PEAK_GBS * 1e9) * 1e3, 4),
                                   "fp64_valu": round(fp64_floor_ms, 4),
                                   "fp64_ops_per_update": fp64_ops},
                     "iteration_equivalent": {
                         "GBs": round(iter_eq, 1), "per_lup_bytes": BYTES_PER_LUP,
                         "note": "24 B/LUP x iterations per launch / launch time; exceeds "
                                 "the HBM peak because one pass carries T iterations"}},
    }
    if world > 1:
        # the decomposed loop's communication (HIP events on the stream that
        # runs it, misor_stats): per exchange / all-reduce, and how much of it
        # the interior sweeps hide -- per pass, the wall time beyond the sweep
        # kernels' own span is the exposed communication (max over ranks)
        passes_all = max(st["timed_passes"], 1)
        vals = [st["halo_ms"] / max(st["halos"], 1), st["allreduce_ms"] / max(st["allreduces"], 1),
                st["sweep_ms"] / passes_all, elapsed * 1e3 / passes_all,
                (st["halo_ms"] + st["allreduce_ms"]) / passes_all]
        tt = torch.tensor(vals, dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        halo, ared, comp, wall, comm = tt.tolist()
        exposed = max(0.0, wall - comp)
        out["comm"] = {"halo_ms_per_exchange": round(halo, 4),
                       "allreduce_ms_per_call": round(ared, 4),
                       "sweep_ms_per_pass": round(comp, 4), "wall_ms_per_pass": round(wall, 4),
                       "comm_ms_per_pass": round(comm, 4),
                       "overlap": round(1.0 - min(1.0, exposed / comm), 3) if comm > 0 else None,
                       "transport": "RCCL send/recv (pack/unpack kernels) + ncclAllReduce",
                       "note": "max over ranks; overlap = 1 - (wall - sweep span) / comm time "
                               "per pass"}
    if pmc_files:
        out["roofline"]["traffic_source"] = pmc_files
    # the VALU roof beside the HBM one: the algorithmic FP64 operations of the
    # launch at the FP64 vector peak (16 lanes/clk/SIMD x 1024 SIMDs x 2.4 GHz)
    # against the launch time
    out["roofline"]["valu_frac"] = round(fp64_floor_ms / kern_ms, 4) if kern_ms > 0 else None
    if valu:
        # what actually bounds the temporally blocked kernel: VALU issue
        # (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES per wave, x waves per SIMD); a
        # launch whose SIMDs issue VALU work >= 85% of their cycles is VALU-bound
        wps = WAVES_PER_SIMD.get(kernel, 2)
        valu["waves_per_simd"] = wps
        valu["valu_busy_per_simd"] = round(valu["valu_busy_per_wave"] * wps, 3)
        out["roofline"]["valu"] = valu
        if valu["valu_busy_per_simd"] >= 0.85:
            out["roofline"]["bound"] = "valu"
    if world > 1:
        out["rccl_ranks"] = rccl_ranks
        if parity is not None:
            out["parity"] = parity
    if not args.no_cpu_baseline:
        # the bench's own grid (rank 0's block at N > 1): the fields the device
        # holds after the timed solve.  (A download of p exchanges its halo
        # first on a decomposed grid, a collective: every rank takes part.)
        hp = g.download(M.P)
        if rank == 0:
            hrhs = g.download(M.RHS)
            try:
                out["cpu_baseline"] = cpu_baseline(hp, hrhs)
            except Exception as e:  # reported, never fatal for the GPU number
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
            try:
                out["cpu_baseline_multicore"] = cpu_baseline_multicore(hp, hrhs)
            except Exception as e:
                out["cpu_baseline_multicore"] = {"value": None, "error": repr(e)}
            del hrhs
            try:
                out["cpu_baseline_mpi"] = cpu_baseline_mpi(granted_cores())
            except Exception as e:
                out["cpu_baseline_mpi"] = {"value": None, "error": repr(e)}
            for key in ("cpu_baseline", "cpu_baseline_multicore", "cpu_baseline_mpi"):
                cb = out[key]
                out["config"][key + "_sample"] = "%s; %s cores (%s)" % (
                    cb.get("sample"), cb.get("cores"), cb.get("kind"))
            if world > 1:
                out["config"]["cpu_baseline_block"] = "rank 0's block %dx%d" % (
                    hp.shape[1] - 2, hp.shape[0] - 2)
        del hp
    g.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
