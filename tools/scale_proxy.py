#!/usr/bin/env python3
"""Compute-side strong-scaling proxy on ONE GPU.

For N = 1, 2, 4, 8 the 32768^2 bench grid is split as bench.py splits it
(misor_decompose); this script times ONE rank's block (rank 0's ni x nj) as a
single-rank solve on this GPU, for several temporally-blocked row heights, and
prints the compute-only efficiency t(1) / (N * t(N)).  Communication is not
modelled (the box has one GPU); what this isolates is the loss from smaller
grids: fewer workgroups per launch, wave quantisation, the last partial round.

    python tools/scale_proxy.py [--size 32768] [--rows 0,128,192] [--sweeps 24]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
import pymisor as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--rows", default="0,96,128,160,192")
    ap.add_argument("--sweeps", type=int, default=24)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--base-ms", type=float, default=0.0,
                    help="N=1 ms per iteration to compute eff against (default: first row)")
    ap.add_argument("--tsteps", default="6", help="iterations per pass to try")
    ap.add_argument("--lib", default="", help="load this libmisor.so instead (A/B runs)")
    ap.add_argument("--shapes", default="",
                    help="explicit local blocks NIxNJ[:N],... instead of the decomposition of --ranks")
    ap.add_argument("--variants", default="-1", help="TB variants to try (-1: default)")
    ap.add_argument("--res-lite", type=int, choices=(0, 1), default=1,
                    help="residual lower bounds of the 10-iteration passes (MISOR_TUNE_RES_LITE)")
    ap.add_argument("--remap", default="1", help="XCD-aware block remap settings to try")
    ap.add_argument("--persistent", default="1", help="work-queue launch settings to try")
    ap.add_argument("--chain", default="-1",
                    help="chained-pass settings to try (TUNE_TB_CHAIN; -1: automatic)")
    ap.add_argument("--reserve", default="16",
                    help="slots a pipelined interior launch leaves free (--comm), settings to try")
    ap.add_argument("--no-timing", action="store_true", help="no per-pass HIP events (wall only)")
    ap.add_argument("--torch-pg", action="store_true",
                    help="also hold a one-rank torch.distributed NCCL process group (as bench.py "
                         "does at N > 1)")
    ap.add_argument("--comm", action="store_true",
                    help="one-rank RCCL communicator: the decomposed, pipelined pass loop "
                         "(comm stream, all-reduce, split launches) without neighbours")
    ap.add_argument("--sides", default=None,
                    help="with --comm: the block's PHYSICAL sides (of LRBT; e.g. LB for "
                         "rank 0 of the 4 x 2 split): the others are treated as bordering "
                         "another rank (MISOR_PROXY_SIDES: halo cones, split launches, "
                         "self-exchanges through the one-rank communicator; timing only)")
    args = ap.parse_args()
    if args.sides is not None:
        # the proxy exists only in the experiment build (csrc/misor_api.hip
        # MISOR_PROXY): make -C practical-parallel-algorithms-with-mpi_amd ab
        # B=build_proxy L=lib_proxy XFLAGS=-DMISOR_PROXY
        args.comm = True
        os.environ["MISOR_PROXY_SIDES"] = args.sides or "-"
        if not args.lib:
            args.lib = os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd", "lib_proxy",
                                    "libmisor.so")
    if args.lib:
        M.LIBPATH = os.path.abspath(args.lib)
    n = args.size
    if args.torch_pg:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0,
                                world_size=1, device_id=torch.device("cuda", 0))
        dist.barrier()
    combos = [(int(t), int(v), int(r), int(x), int(pp), int(rv), int(ch))
              for t in args.tsteps.split(",")
              for v in args.variants.split(",") for r in args.rows.split(",")
              for x in args.remap.split(",") for pp in args.persistent.split(",")
              for rv in args.reserve.split(",") for ch in args.chain.split(",")]
    base = args.base_ms or None
    print("%-2s %-12s %2s %2s %5s %10s %10s %10s %6s" % (
        "N", "local", "T", "v", "rows", "ms/iter", "wall/iter", "MLUP/s/GPU", "eff"), flush=True)
    if args.shapes:
        cases = []
        for sh in args.shapes.split(","):
            dims, _, nr = sh.partition(":")
            a, b = dims.split("x")
            cases.append((int(nr or (n * n) // (int(a) * int(b))), int(a), int(b)))
    else:
        cases = []
        for N in [int(x) for x in args.ranks.split(",")]:
            L = M.decompose(N, 0, n, n)
            cases.append((N, L.ni, L.nj))
    for N, ni, nj in cases:
        g = M.Grid(ni, nj, 1.0 / n, 1.0 / n, 1.9, 1e-300, args.sweeps, device=0,
                   comm_id=M.comm_unique_id() if args.comm else None)
        g.poisson_init(1.0, 1.0, 2)
        g.enable_timing(not args.no_timing)
        g.solve_rb(itermax=args.sweeps)  # warm-up
        v0 = g.get_tuning(M.TUNE_TB_VARIANT)
        g.solve_rb(itermax=args.sweeps)  # the first timed solve of a process runs slow
        res = {c: ([], []) for c in combos}
        hrow, tgot = {}, {}
        applied = None
        for _ in range(args.rounds):
            for c in combos:
                T, v, r, x, pp, rv, ch = c
                if c == applied:  # (re-applying rebuilds the plans: host work in the timing)
                    g.reset_stats()
                    g.synchronize()
                    t0 = time.perf_counter()
                    g.solve_rb(itermax=args.sweeps)
                    g.synchronize()
                    wall = time.perf_counter() - t0
                    st = g.stats()
                    tgot[c] = st["iters_per_pass"]  # (a balanced split of the solve: <= T)
                    res[c][0].append(st["sweep_ms"] / max(st["timed_sweeps"], 1))
                    res[c][1].append(wall * 1e3 / args.sweeps)
                    continue
                applied = c
                try:
                    g.set_tuning(M.TUNE_TB_CHAIN, ch)
                except M.MisorError:  # an older library (--lib A/B runs): no chained passes
                    if ch != -1:
                        raise
                g.set_tuning(M.TUNE_TB_PERSISTENT, pp)
                g.set_tuning(M.TUNE_TB_RESERVE, rv)
                g.set_tuning(M.TUNE_XCD_REMAP, x)
                # (the variant first where T exceeds what the current one runs)
                if T > 8:
                    g.set_tuning(M.TUNE_TB_VARIANT, v0 if v < 0 else v)
                    g.set_tuning(M.TUNE_TSTEPS, T)
                else:
                    g.set_tuning(M.TUNE_TSTEPS, T)
                    g.set_tuning(M.TUNE_TB_VARIANT, v0 if v < 0 else v)
                g.set_tuning(M.TUNE_TB_ROWS, r)
                g.set_tuning(M.TUNE_RES_LITE, args.res_lite)
                hrow[c] = g.get_tuning(M.TUNE_TB_ROWS)
                g.solve_rb(itermax=args.sweeps)  # (plans of the new setting built)
                g.reset_stats()
                g.synchronize()
                t0 = time.perf_counter()
                g.solve_rb(itermax=args.sweeps)
                g.synchronize()
                wall = time.perf_counter() - t0
                st = g.stats()
                tgot[c] = st["iters_per_pass"]  # (a balanced split of the solve: <= T)
                res[c][0].append(st["sweep_ms"] / max(st["timed_sweeps"], 1))
                res[c][1].append(wall * 1e3 / args.sweeps)
        for c in combos:
            T, v, r, x, pp, rv, ch = c
            ms = float(np.median(res[c][0]))
            wall = float(np.median(res[c][1]))
            if ms <= 0:  # --no-timing: wall clock only
                ms = wall
            mlups = ni * nj / (ms * 1e-3) / 1e6
            if base is None:
                base = ms * N
            eff = base / (N * ms)
            print("%-2d %-12s %2d %2d %5d %10.4f %10.4f %10.0f %6.3f  remap=%d persistent=%d "
                  "reserve=%d chain=%d T/pass=%d" % (N, "%dx%d" % (ni, nj), T, v, hrow[c], ms, wall,
                                                      mlups, eff, x, pp, rv, ch, tgot[c]),
                  flush=True)
        g.close()


if __name__ == "__main__":
    main()
