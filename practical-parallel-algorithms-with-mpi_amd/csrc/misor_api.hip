// misor_api.hip -- the C ABI of include/misor.h, part 1: errors, the 2D
// decomposition, grid lifecycle (create / destroy, streams), transfers
// (upload / download / gather / exchange / fill / Poisson init), tuning and
// statistics.  The solve loop is in misor_solve.hip, the NS step in
// misor_ns.hip, communication in misor_comm.hip, launch plans in
// misor_plan.hip; their shared state is struct misor_grid (misor_grid.h).

#include "misor_grid.h"

namespace {

thread_local std::string g_err;

// MPI_Dims_create(n, 2): the most balanced factorisation, larger factor first
void dims_create(int n, int dims[2]) {
    int best = 1;
    for (int d = 1; d * d <= n; ++d)
        if (n % d == 0) best = d;
    dims[0] = n / best;
    dims[1] = best;
}

// sizeOfRank (assignment-5/skeleton/src/solver.c:30-32)
int size_of_rank(int rank, int size, int n) { return n / size + ((n % size > rank) ? 1 : 0); }

std::mutex g_groups_mu;
std::map<std::string, std::shared_ptr<LocalGroup>> g_groups;
constexpr char kLocalPrefix[] = "LOCAL:";

}  // namespace

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

void misor::set_last_error(const char* msg) { g_err = msg; }

const char* misor_last_error(void) { return g_err.c_str(); }
const char* misor_version(void) { return "misor 0.1 (gfx950, fp64 red-black SOR)"; }

int misor_decompose(int nranks, int rank, int imax, int jmax, const int dims_in[2],
                    misor_local* out) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || imax < 2 || jmax < 2)
        return fail(MISOR_EINVAL, "misor_decompose: bad arguments");
    int dims[2] = {0, 0};
    if (dims_in && dims_in[0] > 0 && dims_in[1] > 0) {
        dims[0] = dims_in[0];
        dims[1] = dims_in[1];
        if (dims[0] * dims[1] != nranks)
            return fail(MISOR_EINVAL, "dims %dx%d != nranks %d", dims[0], dims[1], nranks);
    } else {
        dims_create(nranks, dims);
    }
    // MPI_Cart_create row-major rank order: coords = (rank / dims[1], rank % dims[1])
    const int cx = rank / dims[1], cy = rank % dims[1];
    misor_local L{};
    L.dims[0] = dims[0];
    L.dims[1] = dims[1];
    L.coords[0] = cx;
    L.coords[1] = cy;
    L.ni = size_of_rank(cx, dims[0], imax);
    L.nj = size_of_rank(cy, dims[1], jmax);
    int io = 0, jo = 0;
    for (int c = 0; c < cx; ++c) io += size_of_rank(c, dims[0], imax);
    for (int c = 0; c < cy; ++c) jo += size_of_rank(c, dims[1], jmax);
    L.ioff = io;
    L.joff = jo;
    auto rank_of = [&](int x, int y) { return x * dims[1] + y; };
    L.neighbours[0] = cx > 0 ? rank_of(cx - 1, cy) : -1;            // left
    L.neighbours[1] = cx < dims[0] - 1 ? rank_of(cx + 1, cy) : -1;  // right
    L.neighbours[2] = cy > 0 ? rank_of(cx, cy - 1) : -1;            // bottom
    L.neighbours[3] = cy < dims[1] - 1 ? rank_of(cx, cy + 1) : -1;  // top
    if (L.ni < 2 || L.nj < 2) return fail(MISOR_EINVAL, "local block smaller than 2x2");
    L.pitch = layout_pitch(L.ni);
    *out = L;
    return MISOR_OK;
}

int misor_comm_unique_id(void* id_out) {
    if (!id_out) return fail(MISOR_EINVAL, "null id");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == MISOR_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id_out, &id, sizeof id);
    return MISOR_OK;
}

void misor_destroy(misor_grid* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (auto& f : g->fld)
        if (f) (void)hipFree(f);
    (void)hipFree(g->partials);
    (void)hipFree(g->tb_queue);
    for (auto& v : g->chain_plan)
        for (auto& row : v)
            for (auto& pl : row) {
                (void)hipFree(pl.main.tmpl);
                (void)hipFree(pl.edge.tmpl);
            }
    for (int* w : g->tb_work) (void)hipFree(w);
    for (int k = 0; k < 2; ++k) {
        if (g->xstream[k]) {
            (void)hipStreamSynchronize(g->xstream[k]);
            (void)hipStreamDestroy(g->xstream[k]);
        }
        if (g->ev_fork[k]) (void)hipEventDestroy(g->ev_fork[k]);
        if (g->ev_join[k]) (void)hipEventDestroy(g->ev_join[k]);
    }
    (void)hipFree(g->chain_trace);
    (void)hipFree(g->st);
    (void)hipHostFree(g->st_host);
    (void)hipFree(g->red_partials);
    (void)hipFree(g->max_partials);
    (void)hipFree(g->red_out);
    (void)hipHostFree(g->red_host);
    (void)hipFree(g->sendbuf);
    (void)hipFree(g->recvbuf);
    (void)hipFree(g->gbuf);
    (void)hipFree(g->rsq);
    if (g->cstream) (void)hipStreamSynchronize(g->cstream);
    if (g->cstream) (void)hipStreamDestroy(g->cstream);
    for (int b = 0; b < 2; ++b) {
        if (g->ev_i[b]) (void)hipEventDestroy(g->ev_i[b]);
        if (g->ev_dk[b]) (void)hipEventDestroy(g->ev_dk[b]);
        if (g->ev_e2[b]) (void)hipEventDestroy(g->ev_e2[b]);
    }
    if (g->ev_s) (void)hipEventDestroy(g->ev_s);
    if (g->ev_x) (void)hipEventDestroy(g->ev_x);
    if (g->ev_d) (void)hipEventDestroy(g->ev_d);
    for (auto e : g->ev) (void)hipEventDestroy(e);
    for (auto& v : g->cev)
        for (auto e : v) (void)hipEventDestroy(e);
    for (auto& v : g->nev)
        for (auto e : v) (void)hipEventDestroy(e);
    for (hipEvent_t e : {g->lx_pk, g->lx_cp, g->la_val[0], g->la_val[1], g->la_rd[0], g->la_rd[1],
                         g->la_cmb[0], g->la_cmb[1]})
        if (e) (void)hipEventDestroy(e);
    (void)hipFree(g->la_stage);
    (void)hipFree(g->la_gather);
    if (g->comm) ncclCommDestroy(g->comm);
    if (g->own_stream && g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}


int misor_create(misor_grid** out, const misor_desc* d) {
    if (!out || !d) return fail(MISOR_EINVAL, "null argument");
    *out = nullptr;
    if (d->imax < 2 || d->jmax < 2) return fail(MISOR_EINVAL, "imax, jmax must be >= 2");
    if (!(d->dx > 0) || !(d->dy > 0)) return fail(MISOR_EINVAL, "dx, dy must be > 0");
    const int nranks = d->nranks < 1 ? 1 : d->nranks;
    misor_local L{};
    int rc = misor_decompose(nranks, nranks == 1 ? 0 : d->rank, d->imax, d->jmax, d->dims, &L);
    if (rc) return rc;
    // Measurement proxy, in an experiment build only (make ab B=build_proxy
    // L=lib_proxy XFLAGS=-DMISOR_PROXY; tools/scale_proxy.py --sides): one rank
    // on a one-rank communicator whose sides NOT named in MISOR_PROXY_SIDES (of
    // "LRBT") are treated as bordering another rank -- rank 0 itself: the
    // exchange sends each halo region to itself, sizes matching, contents
    // meaningless -- so the block runs the pass loop of a rank of a larger
    // decomposition (split launches, 2T-deep halo cones, exchanges, all-reduce)
    // on one GPU.  Timing only: the field it computes is not the reference's,
    // so misor_download / misor_gather refuse it (MISOR_ESTATE).
    bool proxy = false;
#ifdef MISOR_PROXY
    if (nranks == 1 && d->comm_id) {
        const char* ps = getenv("MISOR_PROXY_SIDES");
        if (ps) {
            proxy = true;
            const char* sides = "LRBT";
            for (int k = 0; k < 4; ++k)
                if (!strchr(ps, sides[k])) L.neighbours[k] = 0;
        }
    }
#endif

    misor_grid* g = new misor_grid();
#ifdef MISOR_PROXY
    g->proxy = proxy;
#endif
    g->desc = *d;
    g->desc.nranks = nranks;
    g->loc = L;
    // a comm id with nranks == 1 still runs the decomposed code path (one rank, no
    // neighbours): lets the RCCL / overlap machinery be exercised on one GPU
    g->dist = nranks > 1 || d->comm_id != nullptr;
    g->np = g->dist ? 3 : 2;
    if (d->device >= 0) {
        g->device = d->device;
        if (hipSetDevice(g->device) != hipSuccess) {
            delete g;
            return fail(MISOR_EHIP, "hipSetDevice(%d) failed", d->device);
        }
    } else {
        (void)hipGetDevice(&g->device);
    }
#define CREATE_FAIL(code, ...)          \
    do {                                \
        int c_ = fail(code, __VA_ARGS__); \
        misor_destroy(g);               \
        return c_;                      \
    } while (0)
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess)
        CREATE_FAIL(MISOR_EHIP, "hipStreamCreate failed");
    g->own_stream = true;

    g->pitch = layout_pitch(L.ni);
    g->rows = layout_rows(L.nj);
    g->elems = g->pitch * g->rows;
    for (int k = 0; k < kNumFields; ++k) {
        if (k == kP2 && g->np < 3) continue;
        if (hipMalloc(&g->fld[k], (size_t)g->elems * sizeof(double)) != hipSuccess)
            CREATE_FAIL(MISOR_ENOMEM, "hipMalloc of %lld doubles failed", g->elems);
        if (hipMemsetAsync(g->fld[k], 0, (size_t)g->elems * sizeof(double), g->stream) !=
            hipSuccess)
            CREATE_FAIL(MISOR_EHIP, "hipMemset failed");
    }

    // sweep configuration
    SweepParams& sp = g->sp;
    sp.pitch = g->pitch;
    sp.ni = L.ni;
    sp.nj = L.nj;
    sp.parity = (L.ioff + L.joff) & 1;
    sp.ghost_left = L.neighbours[0] < 0;
    sp.ghost_right = L.neighbours[1] < 0;
    sp.ghost_bottom = L.neighbours[2] < 0;
    sp.ghost_top = L.neighbours[3] < 0;
    sp.red_lo_i = sp.ghost_left ? 1 : 0;
    sp.red_hi_i = sp.ghost_right ? L.ni : L.ni + 1;
    sp.red_lo_j = sp.ghost_bottom ? 1 : 0;
    sp.red_hi_j = sp.ghost_top ? L.nj : L.nj + 1;
    const double dx2 = d->dx * d->dx, dy2 = d->dy * d->dy;
    sp.idx2 = 1.0 / dx2;
    sp.idy2 = 1.0 / dy2;
    {
        // power-of-two spacing (sor_tb.h resid<true>): 1/dx^2 == 1/dy^2 == 2^m, m >= 0
        int e = 0;
        const double mant = frexp(sp.idx2, &e);
        sp.pow2 = sp.idx2 == sp.idy2 && mant == 0.5 && e >= 1;
    }
    if (d->variant == MISOR_SOLVE_RBA) {
        const double factor = 0.5 * (dx2 * dy2) / (dx2 + dy2);  // solver.c:250
        sp.coef = d->omega * factor;                            // (omega*factor)*r, :273
    } else {
        sp.coef = d->omega * 0.5 * (dx2 * dy2) / (dx2 + dy2);  // solver.c:189
    }
    if (configure_sweep(g, kDefaultSweepVariant, 0, 1) != MISOR_OK) {
        misor_destroy(g);
        return MISOR_ENOMEM;
    }
    {
        // temporally blocked pass: same physics, its own geometry; every cell of
        // a neighbour's 2T-deep halo is updated (identical arithmetic), only the
        // physical sides are bounded
        constexpr int kBig = 1 << 29;
        SweepParams& tp = g->tp;
        tp = sp;
        tp.upd_lo_i = sp.ghost_left ? 1 : -kBig;
        tp.upd_hi_i = sp.ghost_right ? L.ni : kBig;
        tp.upd_lo_j = sp.ghost_bottom ? 1 : -kBig;
        tp.upd_hi_j = sp.ghost_top ? L.nj : kBig;
        // an interior block (overlapped pass) streams no halo cell of src
        tp.int_lo_i = sp.ghost_left ? -kBig : 1;
        tp.int_hi_i = sp.ghost_right ? kBig : L.ni;
        tp.int_lo_j = sp.ghost_bottom ? -kBig : 1;
        tp.int_hi_j = sp.ghost_top ? kBig : L.nj;
    }
    if (hipMalloc(&g->tb_queue, 16 * sizeof(int)) != hipSuccess ||
        hipMemsetAsync(g->tb_queue, 0, 16 * sizeof(int), g->stream) != hipSuccess ||
        hipMalloc(&g->st, sizeof(DevState)) != hipSuccess ||
        hipHostMalloc(&g->st_host, sizeof(DevState), hipHostMallocDefault) != hipSuccess)
        CREATE_FAIL(MISOR_ENOMEM, "state allocation failed");
    const int rb = reduce_blocks(L.ni, L.nj);
    if (hipMalloc(&g->red_partials, sizeof(double) * 2 * rb) != hipSuccess ||
        hipMalloc(&g->max_partials, sizeof(double) * 2 * rb) != hipSuccess ||
        hipMalloc(&g->red_out, sizeof(double) * 4) != hipSuccess ||
        hipHostMalloc(&g->red_host, sizeof(double) * 4, hipHostMallocDefault) != hipSuccess)
        CREATE_FAIL(MISOR_ENOMEM, "reduction allocation failed");

    if (g->dist) {
        if (!d->comm_id) CREATE_FAIL(MISOR_EINVAL, "nranks > 1 needs comm_id");
        const int cx = L.coords[0], cy = L.coords[1], dx_ = L.dims[0], dy_ = L.dims[1];
        auto at = [&](int x, int y) {
            return (x >= 0 && x < dx_ && y >= 0 && y < dy_) ? x * dy_ + y : -1;
        };
        const int nbrs[kDirs] = {at(cx - 1, cy),     at(cx + 1, cy),     at(cx, cy - 1),
                                 at(cx, cy + 1),     at(cx - 1, cy - 1), at(cx + 1, cy - 1),
                                 at(cx - 1, cy + 1), at(cx + 1, cy + 1)};
        for (int k = 0; k < kDirs; ++k) g->nbr[k] = nbrs[k];
        if (proxy) {  // (MISOR_PROXY_SIDES: every neighbour is rank 0; corners where both sides have one)
            const int* nb = L.neighbours;
            const int pn[kDirs] = {nb[0], nb[1], nb[2], nb[3],
                                   nb[0] >= 0 && nb[2] >= 0 ? 0 : -1,
                                   nb[1] >= 0 && nb[2] >= 0 ? 0 : -1,
                                   nb[0] >= 0 && nb[3] >= 0 ? 0 : -1,
                                   nb[1] >= 0 && nb[3] >= 0 ? 0 : -1};
            for (int k = 0; k < kDirs; ++k) g->nbr[k] = pn[k];
        }
        // halo plans up to depth 2*kMaxT + 1 (the skewed split ring's), as deep
        // as the smallest block allows
        const int minb = std::min(d->imax / L.dims[0], d->jmax / L.dims[1]);
        g->max_depth = std::max(2, std::min(2 * kMaxT + 1, minb));
        for (int dd = 1; dd <= g->max_depth; ++dd) build_plan(g, dd);
        // communication and edge blocks at high priority: their workgroups are
        // dispatched ahead of queued interior blocks as slots free up
        int prio_lo = 0, prio_hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
        bool ok = hipStreamCreateWithPriority(&g->cstream, hipStreamNonBlocking, prio_hi) ==
                  hipSuccess;
        for (hipEvent_t* e : {&g->ev_s, &g->ev_x, &g->ev_d, &g->ev_i[0], &g->ev_i[1],
                              &g->ev_e2[0], &g->ev_e2[1],
                              &g->ev_dk[0], &g->ev_dk[1]})
            ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
        if (!ok) CREATE_FAIL(MISOR_EHIP, "comm stream/event creation failed");
        // blocks whose footprint (rows j0-2..j1+1, columns c0-2..c_end+1) stays clear
        // of the halo on neighbour sides AND of the 2-deep send region can sweep
        // while the exchange is in flight
        sp.int_lo_i = L.neighbours[0] >= 0 ? 3 : -1000000000;
        sp.int_hi_i = L.neighbours[1] >= 0 ? L.ni - 2 : 2000000000;
        sp.int_lo_j = L.neighbours[2] >= 0 ? 3 : -1000000000;
        sp.int_hi_j = L.neighbours[3] >= 0 ? L.nj - 2 : 2000000000;
        long long maxtot = 1;
        for (int dd = 1; dd <= g->max_depth; ++dd) maxtot = std::max(maxtot, g->plan[dd].total);
        const size_t hb = (size_t)maxtot * sizeof(double);
        if (hipMalloc(&g->sendbuf, hb) != hipSuccess || hipMalloc(&g->recvbuf, hb) != hipSuccess)
            CREATE_FAIL(MISOR_ENOMEM, "halo buffer allocation failed");
        if (memcmp(d->comm_id, kLocalPrefix, sizeof kLocalPrefix - 1) == 0) {
            char name[MISOR_COMM_ID_BYTES + 1];
            memcpy(name, d->comm_id, MISOR_COMM_ID_BYTES);
            name[MISOR_COMM_ID_BYTES] = '\0';
            {
                std::lock_guard<std::mutex> lk(g_groups_mu);
                auto& G = g_groups[name];
                if (!G) {
                    G = std::make_shared<LocalGroup>();
                    G->n = nranks;
                    G->members.assign(nranks, nullptr);
                    G->vals.assign(kMaxT * (size_t)nranks, 0.0);
                }
                if (G->n != nranks || G->members[d->rank])
                    CREATE_FAIL(MISOR_EINVAL, "local group %s: bad rank/size", name);
                G->members[d->rank] = g;
                g->local = G;
                if (++G->joined == nranks) g_groups.erase(name);  // name reusable
            }
            bool lok = hipMalloc(&g->la_stage, sizeof(double) * 2 * kMaxT) == hipSuccess &&
                       hipMalloc(&g->la_gather, sizeof(double) * 2 * kMaxT * (size_t)nranks) ==
                           hipSuccess;
            for (hipEvent_t* e : {&g->lx_pk, &g->lx_cp, &g->la_val[0], &g->la_val[1],
                                  &g->la_rd[0], &g->la_rd[1], &g->la_cmb[0], &g->la_cmb[1]})
                lok = lok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
            g->local->barrier();  // every member registered before any exchange
            if (!lok) CREATE_FAIL(MISOR_EHIP, "in-process transport allocation failed");
        } else {
            ncclUniqueId id;
            memcpy(&id, d->comm_id, sizeof id);
            if (ncclCommInitRank(&g->comm, nranks, id, d->rank) != ncclSuccess)
                CREATE_FAIL(MISOR_ECOMM, "ncclCommInitRank failed");
        }
    }
    if (configure_tb(g, default_tsteps(g, kDefaultTbVariant), kDefaultTbVariant, 0) != MISOR_OK)
        CREATE_FAIL(MISOR_ENOMEM, "%s", g_err.c_str());
    if (hipStreamSynchronize(g->stream) != hipSuccess)
        CREATE_FAIL(MISOR_EHIP, "hipStreamSynchronize failed");
#undef CREATE_FAIL
    *out = g;
    return MISOR_OK;
}

int misor_local_info(const misor_grid* g, misor_local* out) {
    if (!g || !out) return fail(MISOR_EINVAL, "null argument");
    *out = g->loc;
    return MISOR_OK;
}

int misor_set_stream(misor_grid* g, void* s) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    HIPCHK(hipSetDevice(g->device));
    HIPCHK(hipStreamSynchronize(g->stream));
    if (g->own_stream) HIPCHK(hipStreamDestroy(g->stream));
    if (s) {
        g->stream = (hipStream_t)s;
        g->own_stream = false;
    } else {
        HIPCHK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
        g->own_stream = true;
    }
    g->nl.s = g->stream;
    return MISOR_OK;
}

int misor_synchronize(misor_grid* g) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    return MISOR_OK;
}

static double* field_ptr(misor_grid* g, int field) {
    switch (field) {
    case MISOR_P: return pbuf(g, g->cur);
    case MISOR_RHS: return g->fld[kRhs];
    case MISOR_U: return g->fld[kU];
    case MISOR_V: return g->fld[kV];
    case MISOR_F: return g->fld[kF];
    case MISOR_G: return g->fld[kG];
    default: return nullptr;
    }
}

static double* origin(misor_grid* g, double* base) {
    return base + (long long)kYOff * g->pitch + kXOff;  // cell (0,0)
}

int misor_upload(misor_grid* g, int field, const double* host) {
    if (!g || !host || !field_ptr(g, field)) return fail(MISOR_EINVAL, "bad upload");
    HIPCHK(hipSetDevice(g->device));
    const size_t w = (size_t)(g->loc.ni + 2) * sizeof(double);
    const size_t h = (size_t)(g->loc.nj + 2);
    if (field == MISOR_RHS) g->rhs_halo = 0;
    if (field == MISOR_U || field == MISOR_V) ++g->uv_ver;
    if (field == MISOR_F || field == MISOR_G || field == MISOR_RHS) ++g->fgr_ver;
    if (field == MISOR_P) {  // every pressure buffer: corners and ghosts must agree
        g->cur = 0;
        g->p_stale = false;  // (the caller's halo)
        for (int b = 0; b < g->np; ++b)
            HIPCHK(hipMemcpy2DAsync(origin(g, pbuf(g, b)), g->pitch * sizeof(double), host,
                                    w, w, h, hipMemcpyHostToDevice, g->stream));
    } else {
        HIPCHK(hipMemcpy2DAsync(origin(g, field_ptr(g, field)), g->pitch * sizeof(double), host,
                                w, w, h, hipMemcpyHostToDevice, g->stream));
    }
    HIPCHK(hipStreamSynchronize(g->stream));
    return MISOR_OK;
}

#ifdef MISOR_PROXY
#define PROXYCHK(g)                                                                        \
    do {                                                                                   \
        if ((g)->proxy)                                                                    \
            return fail(MISOR_ESTATE, "a MISOR_PROXY_SIDES grid holds no meaningful field"); \
    } while (0)
#else
#define PROXYCHK(g) \
    do {            \
    } while (0)
#endif

int misor_download(misor_grid* g, int field, double* host) {
    if (!g || !host || !field_ptr(g, field)) return fail(MISOR_EINVAL, "bad download");
    PROXYCHK(g);
    HIPCHK(hipSetDevice(g->device));
    if (field == MISOR_P) {  // the local block with a consistent halo
        int rc = p_halo(g);
        if (rc) return rc;
    }
    const size_t w = (size_t)(g->loc.ni + 2) * sizeof(double);
    const size_t h = (size_t)(g->loc.nj + 2);
    HIPCHK(hipMemcpy2DAsync(host, w, origin(g, field_ptr(g, field)), g->pitch * sizeof(double), w,
                            h, hipMemcpyDeviceToHost, g->stream));
    HIPCHK(hipStreamSynchronize(g->stream));
    return MISOR_OK;
}

// The block a rank contributes to the assembled global field: its interior
// plus the ghost layer on its physical sides (assembleResult,
// assignment-5/skeleton/src/solver.c:234-300), in local indices.
struct OwnedBlock {
    int i0, j0, w, h;    // first local cell and extent
    int gi0, gj0;        // first global cell
};
static OwnedBlock owned_block(const misor_local& L) {
    OwnedBlock b{};
    b.i0 = L.neighbours[0] < 0 ? 0 : 1;
    b.j0 = L.neighbours[2] < 0 ? 0 : 1;
    const int i1 = L.neighbours[1] < 0 ? L.ni + 1 : L.ni;
    const int j1 = L.neighbours[3] < 0 ? L.nj + 1 : L.nj;
    b.w = i1 - b.i0 + 1;
    b.h = j1 - b.j0 + 1;
    b.gi0 = L.ioff + b.i0;
    b.gj0 = L.joff + b.j0;
    return b;
}

int misor_gather(misor_grid* g, int field, double* host) {
    if (!g || !field_ptr(g, field)) return fail(MISOR_EINVAL, "bad gather");
    PROXYCHK(g);
    const int rank = g->dist ? g->desc.rank : 0;
    if (rank == 0 && !host) return fail(MISOR_EINVAL, "gather: rank 0 needs the global array");
    if (g->desc.nranks == 1) return misor_download(g, field, host);
    HIPCHK(hipSetDevice(g->device));
    const size_t gw = (size_t)(g->desc.imax + 2);  // global row length (doubles)
    const OwnedBlock mine = owned_block(g->loc);
    // every rank packs its block contiguously (a strided 2D copy on the device)
    long long need = (long long)(g->loc.ni + 2) * (g->loc.nj + 2);
    if (rank == 0) {
        for (int r = 0; r < g->desc.nranks; ++r) {
            misor_local L{};
            int rc = misor_decompose(g->desc.nranks, r, g->desc.imax, g->desc.jmax,
                                     g->loc.dims, &L);
            if (rc) return rc;
            need = std::max(need, (long long)(L.ni + 2) * (L.nj + 2));
        }
    }
    // every rank allocates its packing buffer (rank 0: large enough for any
    // rank's block -- it is also the receive stage); all ranks agree on the
    // outcome before any send / receive is posted, so a failed allocation is
    // an error on every rank instead of a rank blocked in a send
    int alloc_ok = 1;
    if (need > g->gbuf_cap) {
        (void)hipFree(g->gbuf);
        g->gbuf = nullptr;
        g->gbuf_cap = 0;
        if (hipMalloc(&g->gbuf, sizeof(double) * (size_t)need) == hipSuccess)
            g->gbuf_cap = need;
        else
            alloc_ok = 0;
    }
    {
        g->red_host[3] = alloc_ok ? 0.0 : 1.0;
        HIPCHK(hipMemcpyAsync(g->red_out + 3, g->red_host + 3, sizeof(double),
                              hipMemcpyHostToDevice, g->stream));
        int rc = allreduce(g, g->red_out + 3, 1, 1);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(g->red_host + 3, g->red_out + 3, sizeof(double),
                              hipMemcpyDeviceToHost, g->stream));
        {
            int rc_ = wait_stream(g, g->stream);
            if (rc_) return rc_;
        }
        if (g->red_host[3] != 0.0)
            return fail(MISOR_ENOMEM, "gather: a rank could not allocate its %s buffer",
                        alloc_ok ? "peer's" : "own");
    }
    const double* f = field_ptr(g, field);
    const double* src = origin(g, const_cast<double*>(f)) + (long long)mine.j0 * g->pitch + mine.i0;
    HIPCHK(hipMemcpy2DAsync(g->gbuf, sizeof(double) * mine.w, src, sizeof(double) * g->pitch,
                            sizeof(double) * mine.w, mine.h, hipMemcpyDeviceToDevice, g->stream));
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    auto to_host = [&](const double* dev, const OwnedBlock& b) -> int {
        HIPCHK(hipMemcpy2DAsync(host + (size_t)b.gj0 * gw + b.gi0, sizeof(double) * gw, dev,
                                sizeof(double) * b.w, sizeof(double) * b.w, b.h,
                                hipMemcpyDeviceToHost, g->stream));
        {
            int rc_ = wait_stream(g, g->stream);
            if (rc_) return rc_;
        }
        return MISOR_OK;
    };
    if (g->local) {
        g->local->barrier();  // every block packed
        if (rank == 0) {
            for (int r = 0; r < g->desc.nranks; ++r) {
                const misor_grid* q = g->local->members[r];
                const OwnedBlock b = owned_block(q->loc);
                int rc = to_host(q->gbuf, b);  // unified addressing: any member's device
                if (rc) return rc;
            }
        }
        g->local->barrier();  // nobody repacks before rank 0 has read
        return MISOR_OK;
    }
    // RCCL: rank r sends its packed block to rank 0, one peer at a time; rank
    // 0 receives into its own packing buffer once its block is on the host
    double* const stage = g->gbuf;
    if (rank == 0) {
        int rc = to_host(g->gbuf, mine);
        if (rc) return rc;
    }
    int rc = MISOR_OK;
    for (int r = 1; r < g->desc.nranks && rc == MISOR_OK; ++r) {
        misor_local L{};
        rc = misor_decompose(g->desc.nranks, r, g->desc.imax, g->desc.jmax, g->loc.dims, &L);
        if (rc) break;
        const OwnedBlock b = owned_block(L);
        const size_t count = (size_t)b.w * b.h;
        if (rank == r) {
            if (ncclSend(g->gbuf, count, ncclDouble, 0, g->comm, g->stream) != ncclSuccess)
                rc = fail(MISOR_ECOMM, "gather: ncclSend failed");
        } else if (rank == 0) {
            if (ncclRecv(stage, count, ncclDouble, r, g->comm, g->stream) != ncclSuccess)
                rc = fail(MISOR_ECOMM, "gather: ncclRecv failed");
            else
                rc = to_host(stage, b);
        }
    }
    if (rc) return rc;
    {
        int rc_ = wait_stream(g, g->stream);
        if (rc_) return rc_;
    }
    return MISOR_OK;
}

int misor_exchange(misor_grid* g, int field, int depth) {
    if (!g || !field_ptr(g, field)) return fail(MISOR_EINVAL, "bad exchange");
    if (!g->dist) return MISOR_OK;
    if (depth < 1 || depth > g->max_depth)
        return fail(MISOR_EINVAL, "exchange depth %d outside 1..%d", depth, g->max_depth);
    HIPCHK(hipSetDevice(g->device));
    int rc = exchange(g, field_ptr(g, field), depth);
    if (rc) return rc;
    if (field == MISOR_RHS) g->rhs_halo = std::max(g->rhs_halo, depth);  // now fresh to depth
    if (field == MISOR_P && depth >= 2) g->p_stale = false;
    return wait_stream(g, g->stream);
}

int misor_device_count(int* n) {
    if (!n) return fail(MISOR_EINVAL, "null argument");
    HIPCHK(hipGetDeviceCount(n));
    return MISOR_OK;
}

int misor_comm_ranks(const misor_grid* g, int* n) {
    if (!g || !n) return fail(MISOR_EINVAL, "null argument");
    if (g->comm) {
        NCCLCHK(ncclCommCount(g->comm, n));
    } else if (g->local) {
        *n = g->local->n;
    } else if (g->comm_dead) {
        return fail(MISOR_ECOMM, "the communicator was aborted by an earlier error");
    } else {
        *n = 1;
    }
    return MISOR_OK;
}

int misor_fill(misor_grid* g, int field, double value) {
    if (!g || !field_ptr(g, field)) return fail(MISOR_EINVAL, "bad fill");
    HIPCHK(hipSetDevice(g->device));
    // whole padded array: ghosts included, pads too (pads never feed results)
    if (field == MISOR_RHS) g->rhs_halo = 0;
    if (field == MISOR_U || field == MISOR_V) ++g->uv_ver;
    if (field == MISOR_F || field == MISOR_G || field == MISOR_RHS) ++g->fgr_ver;
    if (field == MISOR_P) {
        g->cur = 0;
        g->p_stale = false;
        for (int b = 0; b < g->np; ++b) launch_fill(g->stream, pbuf(g, b), g->elems, value);
    } else {
        launch_fill(g->stream, field_ptr(g, field), g->elems, value);
    }
    HIPCHK(hipGetLastError());
    return MISOR_OK;
}

int misor_poisson_init(misor_grid* g, double xlength, double ylength, int problem) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    HIPCHK(hipSetDevice(g->device));
    const int ni = g->loc.ni, nj = g->loc.nj;
    const double PI = 3.14159265358979323846;  // assignment-4/src/solver.c:15
    const double dx = xlength / g->desc.imax, dy = ylength / g->desc.jmax;
    // host tables with the reference's exact expressions (solver.c:107,114)
    std::vector<double> sx(ni + 2), sy(nj + 2), rx(ni + 2);
    for (int i = 0; i < ni + 2; ++i) {
        const int gi = g->loc.ioff + i;
        sx[i] = sin(2.0 * PI * gi * dx * 2.0);
        rx[i] = sin(2.0 * PI * gi * dx);
    }
    for (int j = 0; j < nj + 2; ++j) sy[j] = sin(2.0 * PI * (g->loc.joff + j) * dy * 2.0);
    double* tab = nullptr;
    const size_t n = (size_t)(2 * (ni + 2) + (nj + 2));
    HIPCHK(hipMalloc(&tab, n * sizeof(double)));
    HIPCHK(hipMemcpyAsync(tab, sx.data(), (ni + 2) * sizeof(double), hipMemcpyHostToDevice,
                          g->stream));
    HIPCHK(hipMemcpyAsync(tab + (ni + 2), rx.data(), (ni + 2) * sizeof(double),
                          hipMemcpyHostToDevice, g->stream));
    HIPCHK(hipMemcpyAsync(tab + 2 * (ni + 2), sy.data(), (nj + 2) * sizeof(double),
                          hipMemcpyHostToDevice, g->stream));
    g->cur = 0;
    g->p_stale = false;
    g->rhs_halo = 0;
    ++g->fgr_ver;
    for (int b = 0; b < g->np; ++b)
        launch_poisson_init(g->stream, pbuf(g, b), g->fld[kRhs], tab, tab + 2 * (ni + 2),
                            tab + (ni + 2), ni, nj, g->pitch, problem);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(g->stream));
    HIPCHK(hipFree(tab));
    return MISOR_OK;
}


int misor_enable_timing(misor_grid* g, int on) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    g->timing = on != 0;
    return MISOR_OK;
}

int misor_get_stats(const misor_grid* g, misor_stats* out) {
    if (!g || !out) return fail(MISOR_EINVAL, "null argument");
    {
        misor_grid* gm = const_cast<misor_grid*>(g);  // (pending NS kernel timings)
        HIPCHK(hipSetDevice(gm->device));
        int rc = collect_ns_times(gm);
        if (rc) return rc;
    }
    *out = g->stats;
    return MISOR_OK;
}

int misor_set_tuning(misor_grid* g, int key, int value) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    switch (key) {
    case MISOR_TUNE_SWEEP_VARIANT:
        return configure_sweep(g, value, g->sp.rows_per_block, g->sp.xcd_remap);
    case MISOR_TUNE_ROWS_PER_BLOCK:
        return configure_sweep(g, g->sp.variant, value, g->sp.xcd_remap);
    case MISOR_TUNE_XCD_REMAP:
        return configure_sweep(g, g->sp.variant, g->sp.rows_per_block, value != 0);
    case MISOR_TUNE_SMALL_SOLVE: g->small_solve = value != 0; return MISOR_OK;
    case MISOR_TUNE_OVERLAP: g->overlap = value != 0; return MISOR_OK;
    case MISOR_TUNE_TSTEPS: {
        // an explicit request binds: every pass runs T = value iterations (no
        // short plan, no re-pick by MISOR_TUNE_TB_CHAIN); value <= 0 returns
        // to the default rule.  A rejected request changes nothing.
        const bool prev = g->tsteps_set;
        g->tsteps_set = value > 0;
        const int rc = configure_tb(g, value > 0 ? value : default_tsteps(g, g->tp.variant),
                                    g->tp.variant, g->tb_rows_req);
        if (rc) g->tsteps_set = prev;
        return rc;
    }
    case MISOR_TUNE_TB_VARIANT: return configure_tb(g, g->tsteps, value, g->tb_rows_req);
    case MISOR_TUNE_TB_ROWS: return configure_tb(g, g->tsteps, g->tp.variant, value);
    case MISOR_TUNE_TB_PERSISTENT: {
        const bool prev = g->tb_persistent;  // (a rejected request changes nothing)
        g->tb_persistent = value != 0;
        const int rc = configure_tb(g, g->tsteps, g->tp.variant, g->tb_rows_req);
        if (rc) g->tb_persistent = prev;
        return rc;
    }
    case MISOR_TUNE_TB_CHAIN:
        // without an explicit T request the default rule re-picks T (chained
        // small blocks run T = 8, unchained ones T = 7)
        g->tb_chain = value < 0 ? -1 : value != 0;
        return configure_tb(g, g->tsteps_set ? g->tsteps : default_tsteps(g, g->tp.variant),
                            g->tp.variant, g->tb_rows_req);
    case MISOR_TUNE_NS_FUSE: g->ns_fuse = value != 0; return MISOR_OK;
    case MISOR_TUNE_FINISH2: g->finish2 = value != 0; return MISOR_OK;
    case MISOR_TUNE_TB_RESERVE:
        if (value < 0) return fail(MISOR_EINVAL, "reserve must be >= 0");
        g->tb_reserve = value;
        drop_chain_plans(g);  // (the one-list plans count the workgroups left)
        return MISOR_OK;
    case MISOR_TUNE_NEAR_BAND:
        g->near_exp = value;
        g->near_rel = value >= 300 ? 0.0 : pow(10.0, -(double)value);
        return MISOR_OK;
    case MISOR_TUNE_RES_LITE:
        if (value != 0 && value != 1) return fail(MISOR_EINVAL, "RES_LITE is 0 or 1");
        g->res_lite = value != 0;
        return MISOR_OK;
    default: return fail(MISOR_EINVAL, "unknown tuning key %d", key);
    }
}

int misor_get_tuning(const misor_grid* g, int key, int* value) {
    if (!g || !value) return fail(MISOR_EINVAL, "null argument");
    switch (key) {
    case MISOR_TUNE_SWEEP_VARIANT: *value = g->sp.variant; return MISOR_OK;
    case MISOR_TUNE_ROWS_PER_BLOCK: *value = g->sp.rows_per_block; return MISOR_OK;
    case MISOR_TUNE_XCD_REMAP: *value = g->sp.xcd_remap; return MISOR_OK;
    case MISOR_TUNE_SMALL_SOLVE: *value = g->small_solve; return MISOR_OK;
    case MISOR_TUNE_OVERLAP: *value = g->overlap; return MISOR_OK;
    case MISOR_TUNE_TSTEPS: *value = g->tsteps; return MISOR_OK;
    case MISOR_TUNE_TB_VARIANT: *value = g->tp.variant; return MISOR_OK;
    case MISOR_TUNE_TB_ROWS: *value = g->tp.rows_per_block; return MISOR_OK;
    case MISOR_TUNE_TB_PERSISTENT: *value = g->tb_persistent; return MISOR_OK;
    case MISOR_TUNE_TB_CHAIN: *value = chain_on(g, g->tp.variant); return MISOR_OK;
    case MISOR_TUNE_NEAR_BAND: *value = g->near_exp; return MISOR_OK;
    case MISOR_TUNE_RES_LITE: *value = g->res_lite; return MISOR_OK;
    case MISOR_TUNE_NS_FUSE: *value = g->ns_fuse; return MISOR_OK;
    case MISOR_TUNE_FINISH2: *value = g->finish2; return MISOR_OK;
    case MISOR_TUNE_TB_RESERVE: *value = g->tb_reserve; return MISOR_OK;
    default: return fail(MISOR_EINVAL, "unknown tuning key %d", key);
    }
}

int misor_chain_trace(misor_grid* g, unsigned long long* out, long long cap, long long* n) {
    if (!g || !n) return fail(MISOR_EINVAL, "null argument");
    *n = 0;
    if (!g->chain_trace) return MISOR_OK;
    HIPCHK(hipSetDevice(g->device));
    HIPCHK(hipDeviceSynchronize());
    const long long m = std::min(cap, 3 * g->chain_trace_last);
    if (out && m > 0)
        HIPCHK(hipMemcpy(out, g->chain_trace, m * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost));
    *n = 3 * g->chain_trace_last;
    return MISOR_OK;
}

int misor_reset_stats(misor_grid* g) {
    if (!g) return fail(MISOR_EINVAL, "null grid");
    for (auto& u : g->nev_used) u = 0;  // (pending NS kernel timings dropped)
    g->stats = misor_stats{};
    return MISOR_OK;
}
