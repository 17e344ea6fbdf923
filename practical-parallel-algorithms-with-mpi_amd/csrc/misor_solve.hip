// misor_solve.hip -- the solve loop of the C ABI: batched passes with a
// device-resident convergence flag, the pipelined decomposed loop (interior
// and halo parts, exchange and all-reduce overlapped), the exact tail near the
// threshold, and the lexicographic solver entry (misor_grid.h).

#include "misor_grid.h"

// ---------------------------------------------------------------------------
// solve loop
// ---------------------------------------------------------------------------

static int ensure_events(misor_grid* g, size_t n) {
    while (g->ev.size() < n) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        g->ev.push_back(e);
    }
    return MISOR_OK;
}

int solve_rb_from(misor_grid* g, int itermax, int it0, double res0, int* iters,
                         double* res, bool* hand_off);
static int exact_tail(misor_grid* g, int itermax, int it0, double res0, int* iters, double* res,
                      bool* hand_off);

// The batched passes and the exact tail (below) hand the solve to each other
// (*hand_off) with the iterations done and the last residual; this loop runs
// them in turn, so the hand-overs of a long solve need no stack.
int misor_solve_rb_n(misor_grid* g, int itermax, int* iters, double* res) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    HIPCHK(hipSetDevice(g->device));
    int it = 0;
    double r = 1.0;  // solver.c:196
    for (bool tail = false;; tail = !tail) {
        bool hand_off = false;
        const int rc = tail ? exact_tail(g, itermax, it, r, &it, &r, &hand_off)
                            : solve_rb_from(g, itermax, it, r, &it, &r, &hand_off);
        if (rc) return rc;
        if (!hand_off) break;
    }
    if (iters) *iters = it;
    if (res) *res = r;
    return MISOR_OK;
}

// ---------------------------------------------------------------------------
// The loop test near its threshold (partition independence).
// The residual of a pass is a sum of per-workgroup (and, decomposed, per-rank)
// partials, so its last bits depend on the partition -- as the reference's own
// MPI_Allreduce of per-rank sums (assignment-5/skeleton/src/solver.c:651) does.
// An iteration count can only depend on that when res lies within a few ulps
// of eps^2.  The loop-test kernels therefore stop the solve BEFORE any
// iteration whose res lies within near_rel * eps^2 of eps^2 (DevState::near;
// far outside the rounding spread, so every partition stops at the same
// iteration), the pass is recomputed up to there from its untouched source,
// and exact_tail takes over: one sweep per iteration that stores r^2 of every
// cell, whose sum is formed exactly (fixed-point 128-bit limbs per cell --
// each truncation a function of the cell alone -- added in any order and
// all-reduced exactly, ns_kernels.hip exact_sum), so res and the loop test are
// bit for bit the same on every partition.  Once 2T consecutive iterations
// are outside the band again the batched passes resume.  Only solves that come
// near the threshold pay for it.
// ---------------------------------------------------------------------------
static int exact_residual(misor_grid* g, double cells, double* out) {
    NsLaunch L{};  // the reduction region: interior + physical ghost cells (zero in rsq)
    L.s = g->stream;
    L.pitch = g->pitch;
    L.ni = g->loc.ni;
    L.nj = g->loc.nj;
    L.wall_left = g->loc.neighbours[0] < 0;
    L.wall_right = g->loc.neighbours[1] < 0;
    L.wall_bottom = g->loc.neighbours[2] < 0;
    L.wall_top = g->loc.neighbours[3] < 0;
    const int nb = reduce_blocks(L.ni, L.nj);
    launch_absmax2(L, g->rsq, g->rsq, g->red_partials);
    launch_finish_reduce(g->stream, g->red_partials, nb, kReduceMax, 2, g->red_out);
    HIPCHK(hipGetLastError());
    if (g->dist) {
        int rc = allreduce(g, g->red_out, 1, 1);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(g->red_host, g->red_out, sizeof(double), hipMemcpyDeviceToHost,
                          g->stream));
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    int E = 0;
    (void)frexp(g->red_host[0], &E);
    launch_exact_sum(L, g->rsq, E, g->red_partials, g->red_out);
    HIPCHK(hipGetLastError());
    if (g->dist) {
        int rc = allreduce(g, g->red_out, 3, 0);  // integer limbs < 2^53: exact
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(g->red_host, g->red_out, 3 * sizeof(double), hipMemcpyDeviceToHost,
                          g->stream));
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    *out = exact_sum_value(g->red_host, E) / cells;  // solver.c:229
    return MISOR_OK;
}

// iterations it0 + 1 .. of solveRB from the current field, one sweep each with
// the exact residual and the loop test on the host (solver.c:197)
static int exact_tail(misor_grid* g, int itermax, int it0, double res0, int* iters, double* res,
                      bool* hand_off) {
    const double epssq = g->desc.eps * g->desc.eps;
    const double cells = (double)g->desc.imax * (double)g->desc.jmax;
    if (!g->rsq) {
        if (hipMalloc(&g->rsq, (size_t)g->elems * sizeof(double)) != hipSuccess) {
            g->rsq = nullptr;
            return fail(MISOR_ENOMEM, "exact residual buffer allocation failed");
        }
        HIPCHK(hipMemsetAsync(g->rsq, 0, (size_t)g->elems * sizeof(double), g->stream));
    }
    // the sweep kernel runs while the device state says not done
    DevState s{};
    s.it = it0;
    s.res = res0;
    s.epssq = epssq;
    s.itermax = itermax;
    s.nband = -1.0;
    *g->st_host = s;
    HIPCHK(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice, g->stream));
    SweepParams sp = g->sp;  // the default sweep variant's geometry
    if (sp.variant != kDefaultSweepVariant) {
        sp.variant = kDefaultSweepVariant;
        sp.rows_per_block = pick_rows_per_block(g->loc.ni, g->loc.nj, sweep_waves(sp.variant));
        int nby = 0, nbx = 0;
        sp.nblocks = sweep_partials(g->loc.ni, g->loc.nj, sp.rows_per_block,
                                    sweep_waves(sp.variant), &nbx, &nby);
        sp.nbx = nbx;
        if (sp.nblocks > g->partials_cap) {
            int rc = ensure_partials(g, sp.nblocks);
            if (rc) return rc;
        }
    }
    sp.part = 0;
    int it = it0, far = 0;
    double r = res0;
    const int T = effective_tsteps(g);
    while ((r >= epssq) && (it < itermax)) {
        double* src = pbuf(g, g->cur);
        double* dst = pbuf(g, g->cur + 1);
        if (g->dist) {
            int rc = exchange(g, src, 2);  // the sweep reads the 2-deep halo
            if (rc) return rc;
        }
        launch_sweep_rsq(g->stream, sp, src, dst, g->fld[kRhs], g->partials, g->st, g->rsq);
        HIPCHK(hipGetLastError());
        g->cur = (g->cur + 1) % g->np;
        int rc = exact_residual(g, cells, &r);
        if (rc) return rc;
        ++it;
        g->stats.launches += 1;
        // back to the batched passes after 2T iterations outside the band
        far = fabs(r - epssq) > g->near_rel * epssq ? far + 1 : 0;
        if (far >= 2 * T && (r >= epssq) && (it < itermax)) {
            *hand_off = true;  // back to solve_rb_from (misor_solve_rb_n)
            break;
        }
    }
    g->p_stale = g->dist;  // (p_halo)
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    g->stats.sweeps += it - it0;
    g->last_iters = it;
    *iters = it;
    *res = r;
    return MISOR_OK;
}

int solve_rb_from(misor_grid* g, int itermax, int it0, double res0, int* iters,
                         double* res, bool* hand_off) {
    const double epssq = g->desc.eps * g->desc.eps;
    DevState s0{};
    s0.it = it0;
    s0.res = res0;
    s0.epssq = epssq;
    s0.itermax = itermax;
    // (eps^2 = 0 -- e.g. eps = 1e-300 -- has no threshold to come near: res >= 0
    // always continues the loop)
    s0.nband = g->near_rel > 0.0 && epssq > 0.0 ? g->near_rel * epssq : -1.0;
    s0.done = !((res0 >= epssq) && (it0 < itermax));  // loop test of solver.c:197
    if (s0.done) {
        *iters = it0;
        *res = res0;
        return MISOR_OK;
    }
    *g->st_host = s0;
    HIPCHK(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice,
                          g->stream));
    const double cells = (double)g->desc.imax * (double)g->desc.jmax;
    if (!g->dist && g->small_solve && small_solve_fits(g->loc.ni, g->loc.nj)) {
        double* p = pbuf(g, g->cur);
        if (g->timing) {
            int rc = ensure_events(g, 2);
            if (rc) return rc;
            HIPCHK(hipEventRecord(g->ev[0], g->stream));
        }
        launch_solve_small(g->stream, p, g->fld[kRhs], g->loc.ni, g->loc.nj, g->pitch,
                           g->sp.idx2, g->sp.idy2, g->sp.coef, cells, g->st);
        HIPCHK(hipGetLastError());
        if (g->timing) HIPCHK(hipEventRecord(g->ev[1], g->stream));
        HIPCHK(hipMemcpyAsync(g->st_host, g->st, sizeof(DevState), hipMemcpyDeviceToHost,
                              g->stream));
        {
            int rc_ = wait_stream(g, g->stream);
            if (rc_) return rc_;
        }
        const int it = g->st_host->it;
        if (g->timing) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, g->ev[0], g->ev[1]));
            g->stats.sweep_ms += ms;
            g->stats.timed_sweeps += it - it0;
        }
        g->stats.launches += 1;
        if (g->st_host->near) {
            // the kernel left p untouched: run it again up to the iteration
            // before the near one, then the exact tail
            const double rn = g->st_host->res;
            DevState s1 = s0;
            s1.itermax = it;
            s1.nband = -1.0;
            *g->st_host = s1;
            HIPCHK(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice,
                                  g->stream));
            launch_solve_small(g->stream, p, g->fld[kRhs], g->loc.ni, g->loc.nj, g->pitch,
                               g->sp.idx2, g->sp.idy2, g->sp.coef, cells, g->st);
            HIPCHK(hipGetLastError());
            g->stats.sweeps += it - it0;
            *hand_off = true;  // the exact tail from iteration it (misor_solve_rb_n)
            *iters = it;
            *res = rn;
            return MISOR_OK;
        }
        g->stats.sweeps += it - it0;
        g->last_iters = it;
        *iters = it;
        *res = g->st_host->res;
        return MISOR_OK;
    }
    // multi-block path: passes of T iterations (T = 1: single-iteration sweep
    // kernel; T >= 2: temporally blocked kernel, sor_tb.hip)
    //
    // The short plan: a pass costs about the same for any T <= 8 (it streams
    // its fields; profiles/r04_tcurve.txt), so a solve capped at few iterations
    // is cheapest in as few passes as possible.  The split-ring kernel runs
    // kShortT = 10 iterations a pass at ~1.4 x the time of a T = 8 pass
    // (profiles/r04_ab_splitring.txt): where its passes times 1.4 undercut the
    // default's pass count -- 9-10 and 17-20 iterations (the driver's
    // 20-iteration solve: 2 passes instead of 7 + 7 + 6) -- the solve takes it.
    // With the chained split ring (round 5) a T = 10 pass costs about a T = 8
    // one on the blocks where configure_tb sets short_all, so there every solve
    // of more than 8 iterations takes it.
    const int todo0 = itermax - it0;
    const bool all = g->short_all || (g->short_all_lite && g->res_lite);
    const bool shortp = g->short_plan && effective_tsteps(g) == kDefaultTsteps &&
                        (all ? todo0 > kDefaultTsteps
                                      : 7LL * ((todo0 + kShortT - 1) / kShortT) <
                                            5LL * ((todo0 + kDefaultTsteps - 1) / kDefaultTsteps));
    const int T = shortp ? kShortT : effective_tsteps(g);
    SweepParams tpl = g->tp;  // the plan's geometry
    if (shortp) {
        tpl.variant = kShortTbVariant;
        tb_geometry(g, T, tpl);
    }
    // time the communication steps of the loop (collected after each batch)
    g->comm_timing = g->timing && g->dist;
    g->cev_used[0] = g->cev_used[1] = 0;
    // halo of src each pass needs: 2T, one row more for the skewed split ring
    // (its leading stages run one row ahead of the trailing ones; the top rows
    // of their residual windows at a neighbour above read row nj + 2T + 1)
    const int depth = 2 * T + (T >= 2 && tpl.variant == kHrTbVariant && 2 * T < g->max_depth);
    // Residual lower bounds (MISOR_TUNE_RES_LITE): on one rank, a
    // kShortT-iteration split-ring pass counts r^2 of its iterations but the
    // last on one row in S of its steady chunks (sor_tbh.h hrs_step LITE), one
    // FP64 FMA per update fewer on a VALU-bound pass.  Each such sum is a lower
    // bound of the iteration's residual; the loop test (rb_partsum_kernel) takes
    // it only where it proves the loop goes on -- >= eps^2, outside the near
    // band, before itermax -- and otherwise stops the pass before that
    // iteration (DevState::lite_miss): the pass is redone from its source up to
    // there and the rest of the solve counts every cell.  The pass's last
    // iteration is always counted in full, so res after every pass is exact.
    // (one rank: the loop test in the last workgroup of the partial sums;
    // decomposed: the decide kernel after the all-reduce -- the sum of the
    // ranks' lower bounds is one)
    const bool lite_on = g->res_lite && !g->lite_block && T > 1 && (g->dist || g->finish2);
    auto lite_pass = [&](int Tp, int force) {
        return lite_on && force == 0 && Tp == kShortT && tpl.variant == kHrTbVariant;
    };
    auto lite_mask = [&](int Tp) { return lite_pass(Tp, 0) ? (1 << (Tp - 1)) - 1 : 0; };
    const int nparts = T == 1 ? g->nparts : tb_parts(tpl);
    double* const rhs = g->fld[kRhs];
    auto pass = [&](hipStream_t s, int part, const double* src, double* dst, int Tp, int force,
                    double* partials) -> int {
        if (T == 1) {
            SweepParams sp = g->sp;
            sp.part = part;
            launch_sweep(s, sp, src, dst, rhs, partials, g->st);
        } else {
            SweepParams tp = tpl;
            tp.part = part;
            // the interior blocks of an overlapped pass leave workgroup slots to the
            // halo exchange, the residual all-reduce + loop test and the edge blocks
            // on the other streams: a persistent launch holds every slot it gets
            // until the pass is over, so without them the exchange would only start
            // at the end of the interior blocks
            tp.reserve = part == 1 ? g->tb_reserve : 0;
            if (Tp != T) tb_geometry(g, Tp, tp);  // narrower cone: wider strips
            tp.lite = lite_pass(Tp, force) ? 1 : 0;
            if (tp.chain) {  // chained runs, work stealing (parts 0 / 1 and 2 concurrently)
                const misor_grid::ChainPlan* pl = nullptr;
                int rc = chain_plan(g, tp.variant, Tp, part, &pl);
                if (rc) return rc;
                const int k = part == 2 ? 1 : 0;
                tp.seg_cap = kChainSegCap;
                tp.trace = part == 2 ? nullptr : g->chain_trace;
                if (tp.trace) g->chain_trace_last = tp.nblocks;
                auto use = [&](SweepParams& q, const misor_grid::ChainList& L) {
                    q.seg_tmpl = L.tmpl;
                    q.nseg0 = L.nseg0;
                    q.chain_blocks = L.blocks;
                    for (int x = 0; x < 9; ++x) q.seg_run[x] = L.run[x];
                };
                const int eg = pl->edge.nseg0;  // edge workgroups: one per initial segment
                // Where the two kernels run: the main kernel forked to xstream,
                // the edge kernel on s.  The other way round (the edge kernel on
                // xstream, launched first or after the main one) its 16-odd
                // workgroups did not start until the main kernel's workgroups
                // retired, in every pass of a multi-pass solve but the first,
                // though its slots were free (profiles/r03_chain_xmode.txt: 8.5-8.9
                // ms per 32768^2 pass against 6.0).
                SweepParams te = tp;
                use(te, pl->edge);
                te.chain_edge = 1;
                te.reserve = std::max(0, tb_resident(Tp, tp.variant) - eg);
                SweepParams tm = tp;
                use(tm, pl->main);
                tm.chain_edge = 0;
                if (part == 1 && pl->reserve >= 0) tm.reserve = pl->reserve;
                tm.reserve += pl->edge.blocks > 0 ? eg : 0;
                const bool has_e = pl->edge.blocks > 0, has_m = pl->main.blocks > 0;
                // (no edge list: the main kernel alone, on s)
                const bool fork = has_e && has_m;
                hipStream_t ms = fork ? g->xstream[k] : s;
                if (fork) {
                    // A whole pass: the edge kernel's workgroups go on to steal
                    // from the main list once the edge list is done (its 2.5x
                    // block cost is an estimate: its kernel ended ~2.5 ms before
                    // the main one in a 6.6 ms 32768^2 pass, its slots idle), so
                    // the main list's work area is initialised here, before
                    // either kernel starts.  Not in a pipelined pass's parts:
                    // there the edge slots, once free, are part 2's
                    // (profiles/r06_edge_steal_ab.txt: the 8-GPU rank's loop 3%
                    // slower with them stealing)
                    if (part == 0) {
                        launch_chain_init(s, g->tb_work[k], pl->main.tmpl, pl->main.nseg0,
                                          tm.seg_cap);
                        tm.no_init = 1;
                        te.alt_work = g->tb_work[k];
                        te.alt_nseg0 = pl->main.nseg0;
                    }
                    HIPCHK(hipEventRecord(g->ev_fork[k], s));
                    HIPCHK(hipStreamWaitEvent(g->xstream[k], g->ev_fork[k], 0));
                }
                if (has_e)
                    launch_tb(s, Tp, te, src, dst, rhs, partials, g->st, force, g->tb_work[2 + k]);
                if (has_m)
                    launch_tb(ms, Tp, tm, src, dst, rhs, partials, g->st, force, g->tb_work[k]);
                if (fork) {
                    HIPCHK(hipEventRecord(g->ev_join[k], g->xstream[k]));
                    HIPCHK(hipStreamWaitEvent(s, g->ev_join[k], 0));
                }
                return MISOR_OK;
            }
            // persistent work-queue launch on the grid stream (whole passes and
            // interior blocks); the boundary blocks of a split pass are few
            int* q = (g->tb_persistent && part != 2 && s == g->stream) ? g->tb_queue : nullptr;
            launch_tb(s, Tp, tp, src, dst, rhs, partials, g->st, force, q);
        }
        return MISOR_OK;
    };
    const int cur0 = g->cur;
    long long launched = 0;  // passes enqueued
    const int rhs_depth = T == 1 ? 1 : depth;
    if (g->dist && g->rhs_halo < rhs_depth) {  // the halo-ring updates read rhs outside the block
        int rc = exchange(g, rhs, rhs_depth);
        if (rc) return rc;
        g->rhs_halo = rhs_depth;
    }
    // Pipelined decomposed passes (T >= 2, overlap on; three pressure buffers):
    // pass k reads src_k = pbuf(k), writes pbuf(k+1), which is the source of
    // pass k-2 -- so pass k waits for the loop test of pass k-2 only (a pass that
    // overshoots convergence is recomputed from its source), and the all-reduce
    // + loop test of pass k-1 run while pass k sweeps.  Within a pass the
    // interior blocks (part 1, main stream) and the edge blocks (part 2, on
    // cstream: those whose cone reads src's halo; they alone write dst's send
    // region) run concurrently; the exchange of dst's halo for pass k+1 follows
    // the edge blocks on cstream, and so overlaps the interior blocks.
    const bool pipelined = g->dist && g->overlap && T > 1;
    // (the exchange of the first source follows the first pass's interior
    // launch on the host: RCCL's host side of a grouped send / receive takes
    // ~0.1 ms, which the interior blocks need not wait for --
    // profiles/r05_decomposed_loop_trace.csv)
    bool first_x = pipelined;
    if (pipelined) {
        HIPCHK(hipEventRecord(g->ev_s, g->stream));  // state upload, rhs halo, prior work
        HIPCHK(hipStreamWaitEvent(g->cstream, g->ev_s, 0));
    }
    // passes plan the iterations still to do (it0 of them are done: a solve
    // resumed after an exact tail)
    const int todo = itermax - it0;
    const long long max_passes = (todo + T - 1) / T;
    // iterations pass k performs.  The cap takes max_passes passes of at most T
    // iterations (no pass overshoots it); they are made as even as possible --
    // `extra` passes of base + 1, the rest of base -- because a pass costs
    // nearly as much with fewer iterations (a T' = 4 pass at 32768^2 is
    // HBM-bound at 5.06 ms against 5.41 for T = 8), so 20 iterations run as
    // 7 + 7 + 6 rather than 8 + 8 + 4.  A solve that converges earlier stops
    // at the same iteration either way.
    const long long base = todo / max_passes;
    const long long extra = todo % max_passes;
    auto t_of = [&](long long k) -> int { return (int)(base + (k < extra ? 1 : 0)); };
    auto nparts_of = [&](int Tk) -> int {
        if (T == 1 || Tk == T) return nparts;
        SweepParams tp = tpl;
        tb_geometry(g, Tk, tp);
        return tb_parts(tp);
    };
    // iterations covered by the first p passes, and the passes that cover `it`
    auto covered = [&](long long p) -> long long { return p * base + std::min(p, extra); };
    auto passes_for = [&](long long it) -> long long {
        const long long head = extra * (base + 1);  // iterations of the longer passes
        if (it <= head) return (it + base) / (base + 1);
        return std::min(extra + (it - head + base - 1) / base, max_passes);
    };
    // passes enqueued before the host reads the loop state: as many as the last
    // solve took (rounded up: a solve capped at itermax = 100 with T = 8 --
    // NS config 5 -- enqueues its 13 passes at once), at least 8
    const int last_passes = (g->last_iters + T - 1) / T;
    int batch = last_passes > 8 ? last_passes : 8;
    for (;;) {
        if (batch > max_passes - launched) batch = (int)(max_passes - launched);
        if (batch < 1) batch = 1;
        if (g->timing) {
            int rc = ensure_events(g, 2 * (size_t)batch);
            if (rc) return rc;
        }
        for (int b = 0; b < batch && pipelined; ++b) {
            const long long k = launched + b;
            const int Tk = t_of(k);
            const double* src = pbuf(g, cur0 + k);
            double* dst = pbuf(g, cur0 + k + 1);
            double* part = g->partials + (k & 1) * (long long)g->partials_cap;
            // interior blocks: after pass k-1 (this stream, plus the edge blocks:
            // waited on at the end of the previous iteration) and decide k-2
            if (k >= 2) HIPCHK(hipStreamWaitEvent(g->stream, g->ev_dk[k & 1], 0));
            if (g->timing) HIPCHK(hipEventRecord(g->ev[2 * b], g->stream));
            {
                int rc_ = pass(g->stream, 1, src, dst, Tk, 0, part);
                if (rc_) return rc_;
            }
            HIPCHK(hipEventRecord(g->ev_i[k & 1], g->stream));
            // Part 2 (the blocks whose cone reads the halo) on the comm stream,
            // right behind what it waits for: pass k+1's part 2 is enqueued here,
            // after pass k's exchange, loop test and part 1 (its source is pass
            // k's result), so no cross-stream wait stands between the exchange
            // and it.  (On a stream of its own, waiting for the exchange on the
            // comm stream and the interior blocks on this one, the second pass's
            // part 2 started ~0.5 ms late on the 8-GPU rank block:
            // profiles/r05_decomposed_loop_trace*.)  The first pass of a batch
            // enqueues its own part 2: the previous batch's last pass leaves it
            // out, so nothing of a batch is still queued on the comm stream
            // behind the decide the host reads -- a solve that stops there (or a
            // near-threshold hand-off to exact_tail, whose state upload would
            // re-arm the device flag) leaves no pending launch that could still
            // write a pressure buffer.
            int rc = MISOR_OK;
            if (first_x) {  // the solve's first pass: src's halo, then its part 2
                first_x = false;
                rc = exchange(g, const_cast<double*>(src), depth, g->cstream);
                if (rc) return rc;
            }
            if (b == 0) {
                rc = pass(g->cstream, 2, src, dst, Tk, 0, part);
                if (rc) return rc;
                HIPCHK(hipEventRecord(g->ev_e2[k & 1], g->cstream));
            }
            if (k + 1 < max_passes) {  // dst's halo (part 2 of pass k, above, wrote its send region)
                rc = exchange(g, dst, depth, g->cstream);
                if (rc) return rc;
            }
            HIPCHK(hipStreamWaitEvent(g->cstream, g->ev_i[k & 1], 0));
            // the pass's residual sums for the all-reduce: the two-level sum (many
            // workgroups, the last one writing st->sum) -- one workgroup summing
            // every block partial took 70-100 us, after the last pass on the
            // solve's critical path (profiles/r05_decomposed_loop_trace.csv)
            launch_finish2(g->cstream, part, nparts_of(Tk), Tk, g->st, cells,
                           g->partials + 2 * (long long)g->partials_cap, g->tb_queue + 10, 0);
            rc = allreduce(g, g->st->sum, Tk, 0, g->cstream);
            if (rc) return rc;
            launch_decide(g->cstream, g->st, Tk, cells, lite_mask(Tk));
            HIPCHK(hipEventRecord(g->ev_dk[k & 1], g->cstream));
            if (k + 1 < max_passes && b + 1 < batch) {  // pass k+1's part 2: after both parts of pass k
                const long long k1 = k + 1;
                double* part1 = g->partials + (k1 & 1) * (long long)g->partials_cap;
                rc = pass(g->cstream, 2, dst, pbuf(g, cur0 + k1 + 1), t_of(k1), 0, part1);
                if (rc) return rc;
                HIPCHK(hipEventRecord(g->ev_e2[k1 & 1], g->cstream));
            }
            // pass k+1's interior blocks read what part 2 of pass k wrote
            HIPCHK(hipStreamWaitEvent(g->stream, g->ev_e2[k & 1], 0));
            if (g->timing) HIPCHK(hipEventRecord(g->ev[2 * b + 1], g->stream));
            if (b == batch - 1)  // the host reads the loop state after the last decide
                HIPCHK(hipStreamWaitEvent(g->stream, g->ev_dk[k & 1], 0));
        }
        for (int b = 0; b < batch && g->dist && g->overlap && !pipelined; ++b) {
            // Overlapped pass k.  comm stream: [wait pass k-1] all-reduce and
            // decide of k-1, exchange of src_k.  compute stream: interior blocks
            // of pass k (no halo reads) meanwhile, then [wait exchange] boundary
            // blocks, partial sums.  (T = 1 only: T >= 2 takes the pipelined
            // loop above.)  An interior pass launched after convergence (decide
            // k-1 still in flight) only writes a buffer that is not the result.
            const long long k = launched + b;
            const int Tk = t_of(k);
            const double* src = pbuf(g, cur0 + k);
            double* dst = pbuf(g, cur0 + k + 1);
            HIPCHK(hipEventRecord(g->ev_s, g->stream));
            HIPCHK(hipStreamWaitEvent(g->cstream, g->ev_s, 0));
            if (b > 0) {  // pass k-1 of this batch (the previous batch closed its own)
                int rc = allreduce(g, g->st->sum, t_of(k - 1), 0, g->cstream);
                if (rc) return rc;
                launch_decide(g->cstream, g->st, t_of(k - 1), cells);
                if (T > 1) {
                    HIPCHK(hipEventRecord(g->ev_d, g->cstream));
                    HIPCHK(hipStreamWaitEvent(g->stream, g->ev_d, 0));
                }
            }
            int rc = exchange(g, const_cast<double*>(src), depth, g->cstream);
            if (rc) return rc;
            HIPCHK(hipEventRecord(g->ev_x, g->cstream));
            if (g->timing) HIPCHK(hipEventRecord(g->ev[2 * b], g->stream));
            {
                int rc_ = pass(g->stream, 1, src, dst, Tk, 0, g->partials);
                if (rc_) return rc_;
            }
            HIPCHK(hipStreamWaitEvent(g->stream, g->ev_x, 0));
            {
                int rc_ = pass(g->stream, 2, src, dst, Tk, 0, g->partials);
                if (rc_) return rc_;
            }
            if (g->timing) HIPCHK(hipEventRecord(g->ev[2 * b + 1], g->stream));
            launch_finish(g->stream, g->partials, nparts_of(Tk), Tk, g->st, cells, 0);
            if (b == batch - 1) {  // close the batch: all-reduce + decide of the last one
                HIPCHK(hipEventRecord(g->ev_s, g->stream));
                HIPCHK(hipStreamWaitEvent(g->cstream, g->ev_s, 0));
                rc = allreduce(g, g->st->sum, Tk, 0, g->cstream);
                if (rc) return rc;
                launch_decide(g->cstream, g->st, Tk, cells);
                HIPCHK(hipEventRecord(g->ev_x, g->cstream));
                HIPCHK(hipStreamWaitEvent(g->stream, g->ev_x, 0));
            }
        }
        for (int b = 0; b < batch && !(g->dist && g->overlap); ++b) {
            const long long k = launched + b;
            const int Tk = t_of(k);
            const double* src = pbuf(g, cur0 + k);
            double* dst = pbuf(g, cur0 + k + 1);
            if (g->dist) {  // 2T-deep halo of src: one exchange per pass
                int rc = exchange(g, const_cast<double*>(src), depth);
                if (rc) return rc;
            }
            if (g->timing) HIPCHK(hipEventRecord(g->ev[2 * b], g->stream));
            {
                int rc_ = pass(g->stream, 0, src, dst, Tk, 0, g->partials);
                if (rc_) return rc_;
            }
            if (g->timing) HIPCHK(hipEventRecord(g->ev[2 * b + 1], g->stream));
            if (g->dist) {
                launch_finish(g->stream, g->partials, nparts_of(Tk), Tk, g->st, cells, 0);
                int rc = allreduce(g, g->st->sum, Tk, 0);
                if (rc) return rc;
                launch_decide(g->stream, g->st, Tk, cells, lite_mask(Tk));
            } else if (g->finish2) {  // the loop test in the last workgroup (tb_queue[9])
                launch_finish2(g->stream, g->partials, nparts_of(Tk), Tk, g->st, cells,
                               g->partials + 2 * (long long)g->partials_cap, g->tb_queue + 9, 1,
                               lite_mask(Tk));
            } else {
                launch_finish(g->stream, g->partials, nparts_of(Tk), Tk, g->st, cells, 1);
            }
        }
        HIPCHK(hipGetLastError());
        launched += batch;
        g->stats.launches += batch;
        HIPCHK(hipMemcpyAsync(g->st_host, g->st, sizeof(DevState), hipMemcpyDeviceToHost,
                              g->stream));
        {
            int rc_ = wait_stream(g, g->stream);
            if (rc_) return rc_;
        }
        if (g->comm_timing) {
            int rc = collect_comm_times(g);
            if (rc) return rc;
        }
        if (g->timing) {
            // passes after convergence exit at once; count only the real ones
            const long long real_before = launched - batch;
            const long long real_end = passes_for(g->st_host->it - it0);
            for (int b = 0; b < batch; ++b) {
                if (real_before + b >= real_end) break;
                float ms = 0.f;
                HIPCHK(hipEventElapsedTime(&ms, g->ev[2 * b], g->ev[2 * b + 1]));
                g->stats.sweep_ms += ms;
                g->stats.timed_sweeps += t_of(real_before + b);
                g->stats.timed_passes++;
            }
        }
        if (g->st_host->done) break;
        if (launched >= max_passes) break;  // cannot happen: done covers it
        batch = batch < 512 ? 2 * batch : 1024;
    }
    const int it = g->st_host->it;
    const long long passes = passes_for(it - it0);
    const int over = (int)(covered(passes) - (it - it0));
    g->cur = (int)((cur0 + passes) % g->np);
    if (over > 0) {
        // the last pass ran past the iteration that ended the loop: redo it
        // with T - over iterations from its source (untouched since)
        const double* src = pbuf(g, cur0 + passes - 1);
        {
            int rc_ = pass(g->stream, 0, src, pbuf(g, g->cur), t_of(passes - 1) - over, 1, g->partials);
            if (rc_) return rc_;
        }
        HIPCHK(hipGetLastError());
    }
    g->comm_timing = false;
    g->p_stale = g->dist;  // the final field's halo: exchanged by its next reader (p_halo)
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    g->last_iters = it;
    g->stats.sweeps += it - it0;
    g->stats.iters_per_pass = T;
    g->stats.tb_variant = T == 1 ? -1 : tpl.variant;
    g->stats.chained = T > 1 && tpl.chain ? 1 : 0;
    if (g->st_host->lite_miss) {
        // a residual lower bound proved nothing: the field is the state after
        // `it` iterations (the pass redone above), the rest counts every cell
        g->stats.lite_misses++;
        g->lite_block = true;
        const int rc = solve_rb_from(g, itermax, it, g->st_host->res, iters, res, hand_off);
        g->lite_block = false;
        return rc;
    }
    // stopped before an iteration near the threshold: the exact tail goes on
    // from it (misor_solve_rb_n)
    if (g->st_host->near) *hand_off = true;
    *iters = it;
    *res = g->st_host->res;
    return MISOR_OK;
}

int misor_solve_lex(misor_grid* g, int xorder, int* iters, double* res) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    if (g->desc.nranks != 1)
        return fail(MISOR_ESTATE, "lexicographic SOR has no decomposed form (use red-black)");
    if (g->desc.variant != MISOR_SOLVE_RB)
        return fail(MISOR_ESTATE, "lexicographic SOR uses the solveRB factor (variant RB)");
    HIPCHK(hipSetDevice(g->device));
    const double epssq = g->desc.eps * g->desc.eps;
    DevState s0{};
    s0.res = 1.0;
    s0.epssq = epssq;
    s0.itermax = g->desc.itermax;
    *g->st_host = s0;
    HIPCHK(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice,
                          g->stream));
    const double cells = (double)g->desc.imax * (double)g->desc.jmax;
    launch_solve_lex(g->stream, pbuf(g, g->cur), g->fld[kRhs], g->loc.ni, g->loc.nj, g->pitch,
                     g->sp.idx2, g->sp.idy2, g->sp.coef, cells, xorder != 0, g->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(g->st_host, g->st, sizeof(DevState), hipMemcpyDeviceToHost,
                          g->stream));
    HIPCHK(hipStreamSynchronize(g->stream));
    const int it = g->st_host->it;
    g->last_iters = it;
    g->stats.sweeps += it;
    if (iters) *iters = it;
    if (res) *res = g->st_host->res;
    return MISOR_OK;
}

int misor_solve_rb(misor_grid* g, int* iters, double* res) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    return misor_solve_rb_n(g, g->desc.itermax, iters, res);
}
