#!/usr/bin/env python3
"""Interleaved A/B of solve configurations -- library build x TB variant x T --
each in its own child process per round (tools/ab_env.py's child), rounds
alternated; prints ms per iteration (HIP events around every pass) and
whether p is identical across configurations.

    python tools/ab_libs.py --size 32768 --passes 4 --rounds 3 \
        main::0:8 main::6:10 x0:practical-parallel-algorithms-with-mpi_amd/lib_x0/libmisor.so:6:10
    (label:lib:variant:T; an empty lib = the in-tree build)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--ni", type=int, default=0)
    ap.add_argument("--nj", type=int, default=0)
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    res, hashes = {}, set()
    for r in range(a.rounds):
        for c in a.configs:
            label, lib, variant, T = c.split(":")
            cmd = [sys.executable, os.path.join(ROOT, "tools", "ab_env.py"), "--child",
                   "--size", str(a.size), "--tsteps", T, "--passes", str(a.passes),
                   "--ni", str(a.ni), "--nj", str(a.nj), "--variant", variant, "--rows", "0"]
            if lib:
                cmd += ["--lib", os.path.join(ROOT, lib)]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit("child failed for %s" % c)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res.setdefault(c, []).append((d["ms_iter"], d.get("wall_iter", 0.0)))
            hashes.add((T, d["hash"]))
        print("round %d done" % r, file=sys.stderr, flush=True)
    cells = float(a.ni or a.size) * (a.nj or a.size)
    for c, v in res.items():
        ms = sorted(x[0] for x in v)
        wl = sorted(x[1] for x in v)
        print("%-60s ms/iter (events) med %.4f min %.4f | wall med %.4f  MLUP/s (wall) %.0f" % (
            c, ms[len(ms) // 2], ms[0], wl[len(wl) // 2], cells / (wl[len(wl) // 2] * 1e-3) / 1e6))
    by_t = {}
    for t, h in hashes:
        by_t.setdefault(t, set()).add(h)
    print("identical p across configurations of equal T: %s" %
          all(len(v) == 1 for v in by_t.values()))


if __name__ == "__main__":
    main()
