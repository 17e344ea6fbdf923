#!/usr/bin/env python3
"""A/B of the 3D resident solve (assignment-6's 128^3 dcavity time step) between
two library builds, each in its own child process per round, alternated:
solve device time per iteration (misor3 timing) and wall ms per time step.

    python tools/ab3d.py --libs main:,old:practical-parallel-algorithms-with-mpi_amd/lib_x/libmisor.so
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, n, steps):
    sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
    sys.path.insert(0, ROOT)
    import pymisor as M
    if lib:
        M.LIBPATH = os.path.abspath(lib)
    import bench
    prm = dict(bench.DCAVITY3D, imax=n, jmax=n, kmax=n, itermax=1000)
    g = M.Grid3(prm, device=0)
    for f, v in ((M.U3, 0.0), (M.V3, 0.0), (M.W3, 0.0), (M.P3, 0.0)):
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

    for _ in range(2):
        step()
    g.enable_timing(True)
    g.call("synchronize")
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    g.call("synchronize")
    wall = (time.perf_counter() - t0) * 1e3 / steps
    ms, its = g.solve_time()
    print(json.dumps({"us_iter": ms * 1e3 / its, "ms_step": wall, "p": float(g.download(M.P3).sum())}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="main:")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child is not None:
        return child(a.child, a.n, a.steps)
    res = {}
    for _ in range(a.rounds):
        for spec in a.libs.split(","):
            label, lib = spec.split(":", 1)
            out = subprocess.run([sys.executable, __file__, "--child", lib, "--n", str(a.n),
                                  "--steps", str(a.steps)], capture_output=True, text=True,
                                 timeout=600)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit("child failed: %s" % spec)
            res.setdefault(label, []).append(json.loads(out.stdout.strip().splitlines()[-1]))
    for label, v in res.items():
        us = sorted(x["us_iter"] for x in v)
        ms = sorted(x["ms_step"] for x in v)
        print("%-6s solve us/iteration med %.3f min %.3f | ms/step med %.3f | p sums %s" % (
            label, us[len(us) // 2], us[0], ms[len(ms) // 2], sorted({x["p"] for x in v})))


if __name__ == "__main__":
    main()
