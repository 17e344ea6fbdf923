// misor_plan.hip -- launch geometry of the sweeps: rows per block, the
// single-sweep configuration, the temporally blocked passes (T, variant,
// block geometry, the short pass plan) and the segment lists of chained
// passes (misor_grid.h).

#include "misor_grid.h"

int pick_rows_per_block(int ni, int nj, int waves) {
    // enough workgroups to fill 256 CUs several times, but long enough row
    // marches that the two redundant halo rows per block stay cheap
    const int strips = (ni + kStripCells - 1) / kStripCells;
    const int nbx = (strips + waves - 1) / waves;
    const int target_blocks = 2048;
    int want_nby = (target_blocks + nbx - 1) / nbx;
    int h = (nj + want_nby - 1) / want_nby;
    if (h < 4) h = 4;
    if (h > 16) h = 16;  // measured optimum at 32768^2 (profiles/r01_tune_rows.txt)
    return h;
}

int ensure_partials(misor_grid* g, int n) {
    if (n <= g->partials_cap) return MISOR_OK;
    if (g->partials) (void)hipFree(g->partials);
    g->partials = nullptr;
    g->partials_cap = 0;
    // two slots of n (by pass parity) + the two-level finish's chunk sums
    if (hipMalloc(&g->partials, sizeof(double) * (2 * (size_t)n + kMaxT * kFinishChunks)) !=
        hipSuccess)
        return fail(MISOR_ENOMEM, "partials allocation failed");
    g->partials_cap = n;
    return MISOR_OK;
}

// (re)derive the sweep launch geometry; partials are sized for the largest
int configure_sweep(misor_grid* g, int variant, int rows, int remap) {
    if (variant < 0 || variant >= kNumSweepVariants) return fail(MISOR_EINVAL, "bad variant");
    SweepParams& sp = g->sp;
    const int waves = sweep_waves(variant);
    sp.variant = variant;
    sp.rows_per_block = rows > 0 ? rows : pick_rows_per_block(g->loc.ni, g->loc.nj, waves);
    if (sp.rows_per_block < 1) sp.rows_per_block = 1;
    sp.xcd_remap = remap;
    int nby = 0;
    g->nparts = sweep_partials(g->loc.ni, g->loc.nj, sp.rows_per_block, waves, &g->nbx, &nby);
    g->nby = nby;
    sp.nbx = g->nbx;
    sp.nblocks = g->nparts;
    g->tp.xcd_remap = remap;
    return ensure_partials(g, g->nparts);
}

// T that a multi-block solve uses: the requested one, limited so that the
// 2T-deep halo of a decomposed run fits inside the smallest neighbour block
int effective_tsteps(const misor_grid* g) {
    int T = g->tsteps;
    if (T < 1) T = 1;
    if (T > kMaxT) T = kMaxT;
    if (g->dist) {
        const int mi = g->desc.imax / g->loc.dims[0], mj = g->desc.jmax / g->loc.dims[1];
        while (T > 1 && (2 * T > mi || 2 * T > mj || 2 * T > g->max_depth)) --T;
    }
    return T;
}

// Block height H of a pass of T iterations.  A block streams H + 4T rows for
// its H, so tall blocks waste less; short ones give a launch more workgroups.
// With one workgroup per block, round-1 measurements put the optimum near 192
// rows (profiles/r01_shape_sweep*.txt); with the persistent work-queue passes
// (the 64 workgroups of an XCD stream neighbouring blocks of one block row,
// and the pass ends on a band of short blocks) taller blocks pay off: 384 rows
// 0.796 vs 0.821 ms per iteration at 32768^2, 576-768 within noise of 384,
// 1536 slower (profiles/r02_tb_rows_persistent.txt).  H is a multiple of the
// static ring's S slots (sor_tb.hip: interior blocks march in chunks of S
// steps); smaller grids halve it until the launch has ~1024 workgroups.  The last block row takes the rest
// (at most H rows) and marches in pairs.
static int pick_tb_rows(int ni, int nj, int T, int variant) {
    const long long nbx = tb_nbx(ni, T, variant);
    const int S = tb_ring_slots(T, variant);
    auto on_ring = [&](int h) { return S * std::max(1, (h + S / 2) / S); };
    // the tallest of the ladder that still gives the launch ~6 blocks per
    // resident workgroup (3000 blocks)
    int h = kTbRowLadder[0];
    for (int k = 0; k < kTbRowLadderLen; ++k) {
        h = kTbRowLadder[k];
        if (nbx * ((nj + on_ring(h) - 1) / on_ring(h)) >= 3000) break;
    }
    return on_ring(h);
}

// geometry of the temporally blocked pass with T iterations into `tp`: block
// columns and block rows.  Automatic geometry (no MISOR_TUNE_TB_ROWS request):
// blocks of pick_tb_rows' height H, then about two resident rounds of short
// ones (~32 rows) -- the work order takes them last, so the pass ends on
// blocks a sixth as long (the makespan of a persistent pass runs ~half a
// block past its average), at the cost of their extra halo rows -- and a last
// block row of one to two short-block heights (the rest; round 1 left up to H
// rows there, a long row-tested block at the very end of the order).
// (tools/scale_proxy.py, profiles/r02_small_rows.txt: the short band took one
// rank's 8192 x 16384 at 8 GPUs from 0.149 to 0.118 ms per iteration.)  A
// three-level form -- the bulk in 576-row blocks, one round of H, then the
// short band -- ran up to 1.7x slower on the small grids (the tall blocks
// hold their slots for a whole pass; profiles/r02_tb_levels.txt) and was
// dropped.  An explicit request gives uniform blocks of that height, the last
// row taking the rest.
bool chain_on(const misor_grid* g, int variant) {
    if (!g->tb_persistent) return false;
    // the split-ring passes are always chained runs (the warm-up rows they
    // save are VALU work of a VALU-bound pass, sor_tbh.h rb_tbhc_kernel; an
    // unchained form measured 2-15% slower, profiles/r05_hrsweep*.txt)
    if (variant == kHrTbVariant) return true;
    const bool want = g->tb_chain > 0 ||
                      (g->tb_chain < 0 && (long long)g->loc.ni * g->loc.nj < kChainCells);
    return want && variant == kDefaultTbVariant;
}

// T when none was requested: 8 on large local blocks; on small ones 8 with
// chained passes (the default there), 7 without (misor_internal.h)
int default_tsteps(const misor_grid* g, int variant) {
    const long long cells = (long long)g->loc.ni * g->loc.nj;
    return cells >= kTsteps8Cells || chain_on(g, variant) ? kDefaultTsteps : kSmallBlockTsteps;
}

// residual partials per stage of a pass: one per block, or one per block and
// wave for a chained pass (sor_tb.h chain_block_end)
int tb_parts(const SweepParams& tp) {
    return tp.chain ? tp.nblocks * tb_waves(tp.variant) : tp.nblocks;
}

void tb_geometry(const misor_grid* g, int T, SweepParams& tp) {
    const int nj = g->loc.nj, req = g->tb_rows_req;
    tp.nbx = tb_nbx(g->loc.ni, T, tp.variant);
    const int S = tb_ring_slots(T, tp.variant);
    tp.chain = chain_on(g, tp.variant);
    if (tp.chain) {
        // chained passes: short blocks (the unit of residual partials and of
        // work stealing), long runs; every block row but the last a multiple
        // of the ring
        const int rings = tp.variant == kHrTbVariant
                              ? (g->dist ? kHrChainRingsDist : kHrChainRingsPerBlock)
                              : kChainRingsPerBlock;
        int h = req > 0 ? S * std::max(1, (req + S / 2) / S) : rings * S;
        if (h > nj) h = nj;
        tp.rows_per_block = h;
        tp.nby = (nj + h - 1) / h;
        tp.nby_big = tp.nby - 1;
        tp.h_small = h;
        tp.nblocks = tp.nbx * tp.nby;
        return;
    }
    int h = req > 0 ? req : pick_tb_rows(g->loc.ni, nj, T, tp.variant);
    if (h > nj) h = nj;
    const int small_rows = kTbSmallRows;
    const double band_rounds = kTbSmallRounds;
    const int hs = S * std::max(1, (small_rows + S / 2) / S);
    int nbig = 0, ns = 0;
    if (req > 0 || hs >= h || nj < 4 * hs) {  // uniform blocks, the last takes the rest
        nbig = nj / h;
        if (nbig * h == nj && nbig > 0) --nbig;
    } else {
        const int band = std::min(
            (int)((band_rounds * tb_resident(T, tp.variant) + tp.nbx - 1) / tp.nbx), nj / 4 / hs);
        nbig = std::max(0, (nj - band * hs - hs) / h);
        ns = std::max(0, (nj - nbig * h) / hs - 1);  // the last row: [hs, 2 hs)
    }
    tp.rows_per_block = h;
    tp.nby_big = nbig;
    tp.h_small = hs;
    tp.nby = nbig + ns + 1;
    tp.nblocks = tp.nbx * tp.nby;
}

// The initial segment list of a chained pass (sor_tb.h rb_tbc_kernel) of Tp
// iterations, part `part`, built on first use.  Blocks in a part: all (0),
// those whose cone stays clear of the halo (1, sor_tb.h tb_block's test), the
// rest (2).  Along a column, blocks of steady-able rows (chain_rows_ok) form
// runs, each split into segments of about B / G blocks (B: blocks of the
// part, G: workgroups resident at once), so that the initial list gives every
// resident workgroup about one segment; every other block (cone at a
// physical bottom / top side, a last block off the ring) is a segment of its
// own.  The list is column-interleaved (segment s of every column, then s + 1
// ...): the XCD queues deal contiguous runs of it, so neighbouring columns --
// whose strips share 4T columns -- march side by side on one XCD.
void drop_chain_plans(misor_grid* g) {
    for (auto& v : g->chain_plan)
        for (auto& row : v)
            for (auto& pl : row) {
                (void)hipFree(pl.main.tmpl);
                (void)hipFree(pl.edge.tmpl);
                pl = misor_grid::ChainPlan{};
            }
}

// (variant: the configured one or the split ring of the short plan; the plan
// follows that variant's geometry: strip width, ring, block height)
int chain_plan(misor_grid* g, int variant, int Tp, int part,
                      const misor_grid::ChainPlan** out) {
    auto& pl = g->chain_plan[variant == kHrTbVariant ? 1 : 0][Tp][part];
    *out = &pl;
    if (pl.built) return MISOR_OK;
    SweepParams tp = g->tp;
    tp.variant = variant;
    tb_geometry(g, Tp, tp);
    const int W = tb_waves(tp.variant), OW = tb_out_width(Tp, tp.variant);
    const int S = tb_ring_slots(Tp, tp.variant);
    const int nbx = tp.nbx, nby = tp.nby;
    auto rows = [&](int by, int& j0, int& j1) {
        j0 = 1 + by * tp.rows_per_block;
        j1 = by == nby - 1 ? tp.nj + 1 : j0 + tp.rows_per_block;
    };
    // (the skewed split ring streams one row more each way: its leading
    // stages run a row ahead, and the residual they count reads it)
    const int sk = variant == kHrTbVariant && Tp >= 2 ? 1 : 0;
    auto interior = [&](int bx, int by) {
        int j0, j1;
        rows(by, j0, j1);
        const int lo = 1 + bx * W * OW - 2 * Tp;
        const int hi = 1 + (bx * W + W - 1) * OW - 2 * Tp + kStripCells - 1;
        return lo >= tp.int_lo_i && hi <= tp.int_hi_i && j0 - 2 * Tp - sk >= tp.int_lo_j &&
               j1 - 1 + 2 * Tp + sk <= tp.int_hi_j;
    };
    auto steady = [&](int by) {  // sor_tb.h chain_rows_ok
        int j0, j1;
        rows(by, j0, j1);
        return j0 - 2 * Tp >= tp.upd_lo_j && j1 - 1 + 2 * Tp <= tp.upd_hi_j &&
               (j1 - j0) % S == 0 && j1 > j0;
    };
    auto in_part = [&](int bx, int by) { return part == 0 || interior(bx, by) == (part == 1); };
    // a column with a strip at a physical left / right side marches the
    // general, lane-masked way (sor_tb.h chain_run's cols_in)
    auto edge_col = [&](int bx) {
        for (int w = 0; w < W; ++w) {
            const int c_out = 1 + (bx * W + w) * OW;
            if (c_out > tp.ni) break;
            const int c_ld = c_out - 2 * Tp;
            if (!(c_ld >= tp.upd_lo_i && c_ld + kStripCells - 1 <= tp.upd_hi_i &&
                  (c_out + OW - 1 <= tp.ni || (tp.ni & 1) == 0)))
                return true;
        }
        return false;
    };
    // Cost model, in steady-block units: a block of an edge column costs
    // kChainEdgeCost (kSteadyEdge chunks), a block of a row that is not
    // steady-able (a segment of its own) that much plus its 4T warm-up rows.
    // The segments are cut so that each costs about (total / resident
    // workgroups): every workgroup starts one at once and they end together.
    const double E = variant == kHrTbVariant ? (g->dist ? kHrChainEdgeCostDist : kHrChainEdgeCost)
                                             : kChainEdgeCost;
    const int H = tp.rows_per_block;
    // The split ring's plan (round 5): main and edge lists, segments of cost /
    // resident workgroups, and the pipelined pass's part-2 slots sized to its
    // cost share (below): the 8-GPU rank block's pipelined loop 0.130-0.135
    // against 0.145-0.147 ms per iteration with physical left and bottom
    // sides, 0.130-0.131 against 0.136-0.138 with the bottom one only
    // (profiles/r05_reserve_ab.txt).  One list for both kinds of column with
    // exactly one item per workgroup measured 1-3% slower at 32768^2 and on
    // the 8-GPU rank block (profiles/r05_hr_plan_ab.txt: edge-column blocks ran
    // 1.4x longer among the main list's) and was removed.
    const bool sized = variant == kHrTbVariant && part != 0;
    std::vector<unsigned long long> singles;
    double cost = 0;
    long long Bm = 0, Be = 0;
    for (int bx = 0; bx < nbx; ++bx) {
        const bool ecol = edge_col(bx);
        for (int by = 0; by < nby; ++by) {
            if (!in_part(bx, by)) continue;
            if (!steady(by)) {
                singles.push_back(chain_word(bx, by, by + 1));
                cost += E * (H + 4.0 * Tp) / H;
                ++Bm;
            } else {
                cost += ecol ? E : 1.0;
                ++(ecol ? Be : Bm);
            }
        }
    }
    const int G = std::max(8, tb_resident(Tp, tp.variant));
    // a pipelined pass's parts (1: interior blocks, 2: the blocks whose cone
    // reads the halo, launched once the exchange is in): part 2 runs beside
    // part 1 on the slots part 1 leaves free, so those are sized to its share
    // of the pass's cost (at least MISOR_TUNE_TB_RESERVE, which also serves the
    // exchange's kernels) and each part's items to its slots -- part 2's
    // blocks then run as chained runs of the border columns instead of one
    // warmed-up block per slot at the end of the pass
    int Gp = G;
    if (sized) {
        double c12[3] = {0, 0, 0};
        for (int bx = 0; bx < nbx; ++bx) {
            const bool ecol = edge_col(bx);
            for (int by = 0; by < nby; ++by)
                c12[interior(bx, by) ? 1 : 2] +=
                    !steady(by) ? E * (H + 4.0 * Tp) / H : ecol ? E : 1.0;
        }
        const int R = std::min(G / 2, std::max(g->tb_reserve,
                                               (int)llround(G * c12[2] / (c12[1] + c12[2]))));
        pl.reserve = R;
        Gp = std::max(8, part == 1 ? G - R : R);
    }
    double per = std::max(1.0, cost / Gp);  // cost of one segment
    // segments of one steady run of n blocks of cost c1 each
    auto pieces = [&](int n, double c1) {
        return std::min(n, std::max(1, (int)llround(n * c1 / per)));
    };
    auto each_run = [&](auto&& fn) {  // fn(bx, by, n, edge column)
        for (int bx = 0; bx < nbx; ++bx) {
            const bool ecol = edge_col(bx);
            for (int by = 0; by < nby;) {
                if (!in_part(bx, by) || !steady(by)) {
                    ++by;
                    continue;
                }
                int e = by;
                while (e < nby && in_part(bx, e) && steady(e)) ++e;
                fn(bx, by, e - by, ecol);
                by = e;
            }
        }
    };
    std::vector<unsigned long long> edge, inner;  // inner: column-interleaved
    std::vector<std::vector<unsigned long long>> col(nbx);
    each_run([&](int bx, int by, int n, bool ecol) {
        const int k = pieces(n, ecol ? E : 1.0);
        for (int q = 0; q < k; ++q) {
            const unsigned long long w = chain_word(
                bx, by + (int)((long long)n * q / k), by + (int)((long long)n * (q + 1) / k));
            if (ecol) edge.push_back(w);
            else col[bx].push_back(w);
        }
    });
    for (size_t q = 0;; ++q) {
        bool any = false;
        for (int bx = 0; bx < nbx; ++bx)
            if (q < col[bx].size()) {
                inner.push_back(col[bx][q]);
                any = true;
            }
        if (!any) break;
    }
    // XCD runs: the main list -- singles dealt round-robin first, then the
    // inner list in 8 contiguous parts; the edge list round-robin
    auto upload = [&](misor_grid::ChainList& L, const std::vector<unsigned long long>* xl,
                      long long blocks) -> int {
        std::vector<unsigned long long> list;
        for (int x = 0; x < 8; ++x) {
            L.run[x] = (int)list.size();
            list.insert(list.end(), xl[x].begin(), xl[x].end());
        }
        L.run[8] = (int)list.size();
        L.nseg0 = (int)list.size();
        L.blocks = (int)blocks;
        if (list.empty()) return MISOR_OK;
        if (hipMalloc(&L.tmpl, list.size() * sizeof(unsigned long long)) != hipSuccess ||
            hipMemcpy(L.tmpl, list.data(), list.size() * sizeof(unsigned long long),
                      hipMemcpyHostToDevice) != hipSuccess)
            return fail(MISOR_ENOMEM, "chain plan allocation failed");
        return MISOR_OK;
    };
    std::vector<unsigned long long> xm[8], xe[8];
    for (size_t k = 0; k < singles.size(); ++k) xm[k % 8].push_back(singles[k]);
    for (int x = 0; x < 8; ++x)
        for (size_t k = inner.size() * x / 8; k < inner.size() * (x + 1) / 8; ++k)
            xm[x].push_back(inner[k]);
    for (size_t k = 0; k < edge.size(); ++k) xe[k % 8].push_back(edge[k]);
    int rc = upload(pl.main, xm, Bm);
    if (rc) return rc;
    rc = upload(pl.edge, xe, Be);
    if (rc) return rc;
    pl.built = true;
    return MISOR_OK;
}

int configure_tb(misor_grid* g, int T, int variant, int rows) {
    if (T < 1 || T > kMaxT) return fail(MISOR_EINVAL, "iterations per pass must be 1..%d", kMaxT);
    if (variant < 0 || variant >= kNumTbVariants) return fail(MISOR_EINVAL, "bad tb variant");
    if (tb_max_t(variant) == 0)  // measured slower, then not built
        return fail(MISOR_EINVAL, "TB variant %d is retired (measured slower; not built)",
                    variant);
    if (variant == kHrTbVariant && !g->tb_persistent)
        return fail(MISOR_EINVAL, "TB variant %d runs persistent chained passes only", variant);
    if (T > tb_max_t(variant))
        return fail(MISOR_EINVAL, "TB variant %d runs at most %d iterations per pass", variant,
                    tb_max_t(variant));
    g->tsteps = T;
    g->tb_rows_req = rows;
    SweepParams& tp = g->tp;
    tp.variant = variant;
    tp.xcd_remap = g->sp.xcd_remap;
    const int Te = effective_tsteps(g);
    // every pass length a solve may launch (T, the last pass of a capped
    // solve, a pass recomputed after convergence) has its own geometry; the
    // partials hold the largest
    long long need = 1;
    for (int Tp = 1; Tp <= std::max(1, Te); ++Tp) {
        SweepParams q = tp;
        tb_geometry(g, Tp, q);
        // the steady march addresses a block's rows with 32-bit buffer offsets
        // and marks lanes that do not store with offset 2^30
        // (every block row is at most rows_per_block tall)
        if ((q.rows_per_block + 4LL * kMaxT + 8) * tp.pitch * 8 >= (1LL << 30))
            return fail(MISOR_EINVAL, "tb rows %d: a block of rows exceeds 1 GiB",
                        q.rows_per_block);
        need = std::max(need, (long long)Tp * tb_parts(q));
    }
    tb_geometry(g, std::max(2, Te), tp);
    g->tb_nparts = tb_parts(tp);
    // The short plan (solve_rb_from): a single-rank solve capped at few
    // iterations runs them in fewer, longer passes of the split-ring kernel
    // when that saves a pass; its geometries share the partials
    // Where (round 5, the chained split ring; profiles/r05_plan_ab*.txt, wall
    // ms per iteration of 20- and 100-iteration solves against the T = 8 plan):
    //  - blocks of [2^26, 2^28) cells, where the T = 8 passes are chained
    //    (the 8-GPU rank block 8192 x 16384: 0.106 vs 0.123, in the pipelined
    //    loop 0.122 vs 0.142): every solve of more than 8 iterations;
    //  - a single rank of >= 2^29 cells (the 32768^2 bench grid: 0.676 vs 0.682
    //    at 100 iterations, 20 iterations in 2 passes instead of 3): the same;
    //  - a single rank of 2^28 cells, and decomposed blocks of >= 2^28 (the
    //    two- and four-GPU splits of the bench grid): only where it saves
    //    passes, the rule in solve_rb_from (at 100 iterations the two plans are
    //    within 1-3%; the 4-GPU rank block through the pipelined loop of round
    //    5, 20 iterations: 0.2247-0.2250 vs 0.2317-0.2327 ms per iteration,
    //    profiles/r05_plan_ab_ranks.txt -- round 4's loop measured the opposite).
    const long long cells = (long long)g->loc.ni * g->loc.nj;
    const bool small_chain = cells >= kHrAllCells && cells < kTsteps8Cells &&
                             chain_on(g, variant);
    g->short_all = small_chain || (!g->dist && cells >= 2 * kTsteps8Cells);
    //  - round 6: blocks of >= 2^28 cells too, one rank or decomposed, while
    //    the residual lower bounds are on (MISOR_TUNE_RES_LITE: one FMA per
    //    update fewer on the 10-iteration passes) -- NS config 5, 16384^2 with
    //    100 iterations per solve: 20.63-20.66 ms per step against 21.85-22.57
    //    for the 13 T = 8 passes (profiles/r06_ns_plan_ab.txt); the 4-GPU rank
    //    block (sides L, B) at 100 iterations: 0.2072-0.2081 against
    //    0.2189-0.2224 ms per iteration (profiles/r06_plan_ab_rank100.txt)
    g->short_all_lite = cells >= kTsteps8Cells;
    g->short_plan = variant == kDefaultTbVariant && !g->tsteps_set &&
                    g->tb_persistent &&
                    (g->short_all ||
                     (!chain_on(g, variant) &&
                      cells >= (g->dist ? kShortDistCells : kTsteps8Cells)));
    if (g->short_plan) {
        for (int Tp = 1; Tp <= kShortT; ++Tp) {
            SweepParams q = tp;
            q.variant = kShortTbVariant;
            tb_geometry(g, Tp, q);
            if ((q.rows_per_block + 4LL * kMaxT + 8) * tp.pitch * 8 >= (1LL << 30)) {
                g->short_plan = false;
                break;
            }
            need = std::max(need, (long long)Tp * tb_parts(q));
        }
    }
    drop_chain_plans(g);  // geometry changed: rebuilt on first use
    const bool short_chain = g->short_plan && chain_on(g, kShortTbVariant);
    if (chain_on(g, variant) || short_chain) {
        for (int k = 0; k < 2; ++k) {  // the edge kernels' streams
            if (g->xstream[k]) continue;
            int lo = 0, hi = 0;
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            if (hipStreamCreateWithPriority(&g->xstream[k], hipStreamNonBlocking, hi) !=
                    hipSuccess ||
                hipEventCreateWithFlags(&g->ev_fork[k], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&g->ev_join[k], hipEventDisableTiming) != hipSuccess)
                return fail(MISOR_EHIP, "edge stream creation failed");
        }
        // work areas (parts 0 / 1, part 2): head, an initial list of at most
        // one segment per block, the dynamic slots; sized once for every pass
        // length (a launch may still be using them when a plan is built)
        long long most = 1;
        for (int Tp = 1; Tp <= std::max(2, Te); ++Tp) {
            SweepParams q = tp;
            tb_geometry(g, Tp, q);
            most = std::max(most, (long long)q.nblocks);
        }
        for (int Tp = 1; short_chain && Tp <= kShortT; ++Tp) {
            SweepParams q = tp;
            q.variant = kShortTbVariant;
            tb_geometry(g, Tp, q);
            most = std::max(most, (long long)q.nblocks);
        }
        const long long bytes = kChainHead * (long long)sizeof(int) +
                                (most + kChainSegCap) * (long long)sizeof(unsigned long long);
        const char* et = getenv("MISOR_CHAIN_TRACE");
        if (et && et[0] == '1' && most > g->chain_trace_blocks) {
            (void)hipDeviceSynchronize();
            (void)hipFree(g->chain_trace);
            g->chain_trace = nullptr;
            g->chain_trace_blocks = 0;
            if (hipMalloc(&g->chain_trace, 3 * most * sizeof(unsigned long long)) != hipSuccess)
                return fail(MISOR_ENOMEM, "chain trace allocation failed");
            g->chain_trace_blocks = most;
        }
        for (int k = 0; k < 4; ++k) {
            if (bytes <= g->tb_work_bytes[k]) continue;
            if (g->tb_work[k]) {
                (void)hipDeviceSynchronize();
                (void)hipFree(g->tb_work[k]);
            }
            g->tb_work[k] = nullptr;
            g->tb_work_bytes[k] = 0;
            if (hipMalloc(&g->tb_work[k], bytes) != hipSuccess)
                return fail(MISOR_ENOMEM, "chain work area allocation failed");
            g->tb_work_bytes[k] = bytes;
        }
    }
    return ensure_partials(g, (int)need);
}
