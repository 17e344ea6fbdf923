#!/usr/bin/env python3
"""Timeline of one chained temporally blocked pass (diagnostics).

    MISOR_CHAIN_TRACE=1 python tools/chain_trace.py [--shape 8192x16384] [--T 8] [--rows 0]

Runs a few warm-up passes, then one traced pass of T iterations, and prints:
the pass span, how busy the workgroups were, when they ran out of work, the
block durations by kind (a run's first block -- warm-up included -- or a
chained one; edge columns or not) and the number of active workgroups over
time.  Clock: the 100 MHz wall clock (10 ns ticks).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "practical-parallel-algorithms-with-mpi_amd"))
import pymisor as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8192x16384")
    ap.add_argument("--size", type=int, default=32768, help="spacing 1/size")
    ap.add_argument("--T", type=int, default=8)
    ap.add_argument("--variant", type=int, default=-1, help="TB variant (13: the split ring)")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--passes", type=int, default=3, help="traced solves (last one kept)")
    ap.add_argument("--per-solve", type=int, default=1, help="passes per solve (the last traced)")
    a = ap.parse_args()
    os.environ["MISOR_CHAIN_TRACE"] = "1"
    ni, nj = (int(x) for x in a.shape.split("x"))
    g = M.Grid(ni, nj, 1.0 / a.size, 1.0 / a.size, 1.9, 1e-300, a.T * a.per_solve, device=0)
    g.poisson_init(1.0, 1.0, 2)
    g.set_tuning(M.TUNE_TB_CHAIN, 1)
    if a.variant >= 0:
        g.set_tuning(M.TUNE_TB_VARIANT, a.variant)
    g.set_tuning(M.TUNE_TSTEPS, a.T)
    if a.rows:
        g.set_tuning(M.TUNE_TB_ROWS, a.rows)
    H = g.get_tuning(M.TUNE_TB_ROWS)
    spans = []
    g.enable_timing(True)
    for _ in range(a.passes):
        g.reset_stats()
        g.solve_rb(itermax=a.T * a.per_solve)
        tr = g.chain_trace()
        t0, t1 = tr[:, 0].min(), tr[:, 1].max()
        spans.append((t1 - t0) * 10e-6)
    st = g.stats()
    print("last solve: %d passes, %.3f ms per pass (HIP events)" % (
        st["timed_passes"], st["sweep_ms"] / max(st["timed_passes"], 1)))
    g.close()
    st = tr[:, 0].astype(np.int64)
    en = tr[:, 1].astype(np.int64)
    wg = (tr[:, 2] & 0xffffffff).astype(np.int64)
    first = (tr[:, 2] >> np.uint64(32)).astype(bool)
    t0 = st.min()
    st, en = st - t0, en - t0
    span = en.max()
    dur = (en - st) * 10e-3  # us
    print("shape %s T %d rows %d: %d blocks, %d workgroups, %d runs (%d beyond one per "
          "workgroup)" % (a.shape, a.T, H, len(st), len(set(wg)), first.sum(),
                          first.sum() - len(set(wg))))
    print("pass spans (ms): %s" % ", ".join("%.3f" % x for x in spans))
    print("block us: chained median %.1f p90 %.1f | run start median %.1f p90 %.1f" % (
        np.median(dur[~first]), np.percentile(dur[~first], 90), np.median(dur[first]),
        np.percentile(dur[first], 90)))
    last_end = {}
    busy = {}
    for w, s, e in zip(wg, st, en):
        last_end[w] = max(last_end.get(w, 0), e)
        busy[w] = busy.get(w, 0) + (e - s)
    le = np.array(sorted(last_end.values())) * 10e-6
    b = np.array(list(busy.values())) * 10e-6
    print("workgroup last block end (ms): min %.3f p10 %.3f median %.3f p90 %.3f max %.3f" % (
        le.min(), np.percentile(le, 10), np.median(le), np.percentile(le, 90), le.max()))
    print("busy fraction of the span: mean %.3f min %.3f" % (b.mean() / (span * 10e-6),
                                                           b.min() / (span * 10e-6)))
    # runs: per workgroup, its blocks in time order; a run = a first block and
    # the chained ones after it
    order = np.lexsort((st, wg))
    runs = []
    cur = None
    for i in order:
        if first[i] or cur is None or cur[0] != wg[i]:
            if cur is not None:
                runs.append(cur)
            cur = [wg[i], st[i], 0]
        cur[2] += 1
    runs.append(cur)
    # block durations by position in the run and by column kind
    pos = np.zeros(len(st), dtype=np.int64)
    prev_w, k = None, 0
    for i in order:
        k = 0 if (first[i] or wg[i] != prev_w) else k + 1
        pos[i] = k
        prev_w = wg[i]
    nbx = int(np.ceil(ni / (4 * (128 - 4 * a.T))))
    col = np.arange(len(st)) % nbx
    edge = (col == 0) | (col == nbx - 1)
    print("block us by position in run: %s; edge columns median %.1f, others %.1f" % (
        ", ".join("%d: %.1f (p90 %.1f, n %d)" % (q, np.median(dur[pos == q]),
                                                 np.percentile(dur[pos == q], 90),
                                                 (pos == q).sum())
                  for q in range(4) if (pos == q).any()) +
        ", 4+: %.1f (p90 %.1f)" % (np.median(dur[pos >= 4]), np.percentile(dur[pos >= 4], 90)),
        np.median(dur[edge]), np.median(dur[~edge])))
    # durations over time (when in the pass a block ran)
    tb = np.linspace(0, span, 11)
    print("median block us per 10%% of the span (non-edge, chained): %s" % " ".join(
        "%.0f" % np.median(dur[(st >= tb[q]) & (st < tb[q + 1]) & ~edge & ~first])
        if ((st >= tb[q]) & (st < tb[q + 1]) & ~edge & ~first).any() else "-" for q in range(10)))
    rl = np.array([r[2] for r in runs])
    rs = np.array([r[1] for r in runs]) * 10e-6
    late = rs > 0.05 * span * 10e-6
    print("runs: %d; blocks per run: initial median %.0f, stolen median %.0f p10 %.0f p90 %.0f; "
          "steals started at (ms) p10 %.3f median %.3f p90 %.3f max %.3f" % (
              len(runs), np.median(rl[~late]) if (~late).any() else 0,
              np.median(rl[late]) if late.any() else 0,
              np.percentile(rl[late], 10) if late.any() else 0,
              np.percentile(rl[late], 90) if late.any() else 0,
              *(np.percentile(rs[late], [10, 50, 90]).tolist() + [rs.max()] if late.any()
                else [0, 0, 0, 0])))
    # active workgroups over time (20 bins)
    edges = np.linspace(0, span, 21)
    act = []
    for k in range(20):
        lo, hi = edges[k], edges[k + 1]
        ov = np.clip(np.minimum(en, hi) - np.maximum(st, lo), 0, None).sum()
        act.append(ov / (hi - lo))
    print("active workgroups per 5%% of the span: %s" % " ".join("%.0f" % x for x in act))
    # the blocks that ended last
    idx = np.argsort(en)[-8:]
    print("last blocks (L, start us, end us, first-of-run):",
          [(int(i), round(st[i] * 1e-2, 1), round(en[i] * 1e-2, 1), bool(first[i])) for i in idx])


if __name__ == "__main__":
    main()
