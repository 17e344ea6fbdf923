// misor3d_api.hip -- the C ABI of the 3D path (include/misor.h, misor3_*):
// assignment-6's 3D Navier-Stokes solver (assignment-6/src/solver.c).  The
// entry points mirror the reference's solver.h one to one; fields are
// device-resident in the reference layout.
//
// Decomposition: slabs of planes along k, one rank per GPU (or per host
// thread with the in-process transport).  The reference splits the box over a
// 3D Cartesian process grid (assignment-6/src/comm.c:24-101, 476-513); on one
// MI355X node a 1D split of at most 8 slabs keeps every halo a run of whole
// planes -- contiguous in this layout, so halos move by ncclSend/ncclRecv
// straight from the field, no packing -- and each GPU still owns >= 16 planes
// at the reference's 128^3.  Colours are global (i+j+k with global k), so the
// fields are bit-identical to the single-domain solve for every slab count.
//
// Storage per field: planes -1 .. K+2 of the rank's slab (K = its plane count),
// i.e. the reference's local array (planes 0 .. K+1) plus one more plane on
// each side for the 2-deep halo the fused sweep reads.

#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "misor_internal.h"

using namespace misor;

namespace {

int fail3(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail3(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    set_last_error(buf);
    return code;
}

#define HIPCHK3(x)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess)                                                              \
            return fail3(MISOR_EHIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                        \
    } while (0)

#define NCCLCHK3(x)                                                                        \
    do {                                                                                   \
        ncclResult_t r_ = (x);                                                             \
        if (r_ != ncclSuccess)                                                             \
            return fail3(MISOR_ECOMM, "%s: %s (%s:%d)", #x, ncclGetErrorString(r_),       \
                         __FILE__, __LINE__);                                              \
    } while (0)

constexpr int kHalo = 2;          // halo planes per side in storage
constexpr int kSlack = 2;         // spare doubles before / after every buffer: the sweep's
                                  // 16-byte column-pair loads reach one past a row end
constexpr int kBufs = 9;          // the 8 fields + the ping-pong partner of P
constexpr int kAlt = 8;
constexpr char kLocalPrefix3[] = "LOCAL:";

int size_of_rank3(int rank, int size, int n) { return n / size + ((n % size > rank) ? 1 : 0); }

struct LocalGroup3;

}  // namespace

struct misor_grid3 {
    int device = 0;
    hipStream_t stream = nullptr;
    misor3_desc desc{};
    G3 g{};                    // this rank's slab: g.K planes, g.koff, physical flags
    long long n = 0;           // cells of the reference's local array (planes 0 .. K+1)
    long long nalloc = 0;      // cells allocated per field (planes -1 .. K+2)
    double* alloc[kBufs] = {}; // allocations: nalloc + 2*kSlack doubles
    double* mem[kBufs] = {};   // plane -1 of each buffer (alloc + kSlack)
    double* fld[kBufs] = {};   // plane-0 origins: MISOR3_P .. MISOR3_H, kAlt = P's partner
    bool alt_stale = true;     // the partner's edge/corner ghosts may differ from P's
    int sweep = 1;             // MISOR3_TUNE_SWEEP
    int rows = 8;              // MISOR3_TUNE_ROWS
    int kchunk = 0;            // MISOR3_TUNE_KCHUNK (0: automatic)
    int fold = 1;              // MISOR3_TUNE_FOLD: single rank, loop test inside the sweep
    int resident = -1;         // MISOR3_TUNE_RESIDENT: whole solve in one launch when it fits
    void* rbar = nullptr;      // its grid-barrier state and partials, uncached memory
    double* rmbox = nullptr;   // its exchange mailboxes (2 x p's layout), uncached memory
    int rhs_ahead = 0;         // MISOR3_TUNE_RHS_AHEAD: fused sweep's rhs loads 1 or 2 steps
                               // ahead; 0: 2 on marches of >= 16 planes, else 1
    double dx = 0, dy = 0, dz = 0, dt = 0, dt_bound = 0;
    double* partials = nullptr;  // per-block partial sums / maxima
    long long partials_cap = 0;
    double* out = nullptr;      // 4 doubles on the device (maxima / sum)
    double* out_host = nullptr; // pinned
    DevState* st = nullptr;
    DevState* st2 = nullptr;  // the folded loop test's second state buffer
    DevState* st_host = nullptr;
    int last_iters = 0;
    bool timing = false;          // misor3_enable_timing
    hipEvent_t ev[2] = {};        // around each solve, on the grid's stream
    double solve_ms = 0;          // accumulated device time of timed solves
    long long solve_iters = 0;    // iterations of the timed solves
    // decomposition
    int nranks = 1, rank = 0, prev = -1, next = -1;
    ncclComm_t comm = nullptr;
    std::shared_ptr<LocalGroup3> local;
    double* gstage = nullptr;     // rank 0: receive staging of misor3_gather (RCCL)
};

namespace {

// In-process transport (as in 2D, misor_api.hip): the ranks are grids driven
// by host threads of one process; collectives are a host barrier plus
// device-to-device copies, sums combined in rank order.
struct LocalGroup3 {
    int n = 0;
    std::vector<misor_grid3*> members;
    std::vector<double> vals;  // n * 4 scratch for all-reduce
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0, joined = 0;
    long long generation = 0;
    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        const long long gen = generation;
        if (++arrived == n) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};
std::mutex g_groups3_mu;
std::map<std::string, std::shared_ptr<LocalGroup3>> g_groups3;

bool dist(const misor_grid3* g) { return g->nranks > 1; }

// plane kk of buffer b
double* plane_ptr(misor_grid3* g, int b, int kk) { return g->fld[b] + (long long)kk * g->g.sxy; }

// d-deep halo of buffer b: planes K-d+1..K to the next rank's 1-d..0, planes
// 1..d to the previous rank's K+1..K+d
int exchange3(misor_grid3* g, int b, int d) {
    if (!dist(g)) return MISOR_OK;
    const size_t cnt = (size_t)d * (size_t)g->g.sxy;
    const int K = g->g.K;
    if (g->local) {
        LocalGroup3& G = *g->local;
        HIPCHK3(hipStreamSynchronize(g->stream));
        G.barrier();  // every rank's sent planes are final
        if (g->prev >= 0) {
            misor_grid3* q = G.members[g->prev];
            HIPCHK3(hipMemcpyAsync(plane_ptr(g, b, 1 - d), plane_ptr(q, b, q->g.K - d + 1),
                                   cnt * sizeof(double), hipMemcpyDeviceToDevice, g->stream));
        }
        if (g->next >= 0) {
            misor_grid3* q = G.members[g->next];
            HIPCHK3(hipMemcpyAsync(plane_ptr(g, b, K + 1), plane_ptr(q, b, 1),
                                   cnt * sizeof(double), hipMemcpyDeviceToDevice, g->stream));
        }
        HIPCHK3(hipStreamSynchronize(g->stream));
        G.barrier();  // nobody overwrites a sent plane before every copy is done
        return MISOR_OK;
    }
    NCCLCHK3(ncclGroupStart());
    if (g->next >= 0) {
        NCCLCHK3(ncclSend(plane_ptr(g, b, K - d + 1), cnt, ncclDouble, g->next, g->comm,
                          g->stream));
        NCCLCHK3(ncclRecv(plane_ptr(g, b, K + 1), cnt, ncclDouble, g->next, g->comm, g->stream));
    }
    if (g->prev >= 0) {
        NCCLCHK3(ncclSend(plane_ptr(g, b, 1), cnt, ncclDouble, g->prev, g->comm, g->stream));
        NCCLCHK3(ncclRecv(plane_ptr(g, b, 1 - d), cnt, ncclDouble, g->prev, g->comm, g->stream));
    }
    NCCLCHK3(ncclGroupEnd());
    return MISOR_OK;
}

// all-reduce of n <= 4 device doubles (sum or max)
int allreduce3(misor_grid3* g, double* dev, int n, bool is_max) {
    if (!dist(g)) return MISOR_OK;
    if (g->local) {
        LocalGroup3& G = *g->local;
        double v[4];
        HIPCHK3(hipMemcpyAsync(v, dev, sizeof(double) * n, hipMemcpyDeviceToHost, g->stream));
        HIPCHK3(hipStreamSynchronize(g->stream));
        for (int k = 0; k < n; ++k) G.vals[4 * g->rank + k] = v[k];
        G.barrier();
        for (int k = 0; k < n; ++k) {
            double a = G.vals[k];
            for (int q = 1; q < G.n; ++q) {
                const double c = G.vals[4 * q + k];
                a = is_max ? ((a > c) ? a : c) : a + c;
            }
            v[k] = a;
        }
        G.barrier();
        HIPCHK3(hipMemcpyAsync(dev, v, sizeof(double) * n, hipMemcpyHostToDevice, g->stream));
        HIPCHK3(hipStreamSynchronize(g->stream));
        return MISOR_OK;
    }
    NCCLCHK3(ncclAllReduce(dev, dev, n, ncclDouble, is_max ? ncclMax : ncclSum, g->comm,
                           g->stream));
    return MISOR_OK;
}

}  // namespace

extern "C" {

void misor3_destroy(misor_grid3* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (auto& f : g->alloc)
        if (f) (void)hipFree(f);
    (void)hipFree(g->partials);
    (void)hipFree(g->rbar);
    (void)hipFree(g->rmbox);
    (void)hipFree(g->out);
    (void)hipHostFree(g->out_host);
    (void)hipFree(g->st);
    (void)hipFree(g->st2);
    (void)hipHostFree(g->st_host);
    (void)hipFree(g->gstage);
    for (auto& e : g->ev)
        if (e) (void)hipEventDestroy(e);
    if (g->comm) ncclCommDestroy(g->comm);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

int misor3_decompose(int nranks, int rank, int kmax, int* kloc, int* koff) {
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return fail3(MISOR_EINVAL, "bad rank %d of %d", rank, nranks);
    if (kmax / nranks < kHalo)
        return fail3(MISOR_EINVAL, "%d planes over %d ranks: fewer than %d per rank", kmax,
                     nranks, kHalo);
    int off = 0;
    for (int r = 0; r < rank; ++r) off += size_of_rank3(r, nranks, kmax);
    if (kloc) *kloc = size_of_rank3(rank, nranks, kmax);
    if (koff) *koff = off;
    return MISOR_OK;
}

int misor3_create(misor_grid3** out, const misor3_desc* d) {
    if (!out || !d) return fail3(MISOR_EINVAL, "null argument");
    *out = nullptr;
    if (d->imax < 2 || d->jmax < 2 || d->kmax < 2)
        return fail3(MISOR_EINVAL, "imax, jmax, kmax must be >= 2");
    const int nranks = d->nranks > 0 ? d->nranks : 1;
    int kloc = d->kmax, koff = 0;
    if (nranks > 1) {
        if (!d->comm_id) return fail3(MISOR_EINVAL, "nranks > 1 needs a comm_id");
        const int rc = misor3_decompose(nranks, d->rank, d->kmax, &kloc, &koff);
        if (rc != MISOR_OK) return rc;
    }
    misor_grid3* g = new misor_grid3();
    g->desc = *d;
    g->device = d->device;
    g->nranks = nranks;
    g->rank = nranks > 1 ? d->rank : 0;
    g->prev = g->rank > 0 ? g->rank - 1 : -1;
    g->next = g->rank < nranks - 1 ? g->rank + 1 : -1;
    if (d->device >= 0) {
        if (hipSetDevice(d->device) != hipSuccess) {
            delete g;
            return fail3(MISOR_EHIP, "hipSetDevice(%d) failed", d->device);
        }
    } else {
        (void)hipGetDevice(&g->device);
    }
#define CF(code, ...)                        \
    do {                                     \
        int c_ = fail3(code, __VA_ARGS__);   \
        misor3_destroy(g);                   \
        return c_;                           \
    } while (0)
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess)
        CF(MISOR_EHIP, "hipStreamCreate failed");
    g->g.I = d->imax;
    g->g.J = d->jmax;
    g->g.K = kloc;
    g->g.sx = d->imax + 2;
    g->g.sxy = (long long)(d->imax + 2) * (d->jmax + 2);
    g->g.Kg = d->kmax;
    g->g.koff = koff;
    g->g.lo_phys = g->prev < 0;
    g->g.hi_phys = g->next < 0;
    g->n = g->g.sxy * (kloc + 2);
    g->nalloc = g->g.sxy * (kloc + 2 * kHalo);
    // initSolver, solver.c:86-95
    g->dx = d->xlength / d->imax;
    g->dy = d->ylength / d->jmax;
    g->dz = d->zlength / d->kmax;
    {
        const double inv = 1.0 / (g->dx * g->dx) + 1.0 / (g->dy * g->dy) + 1.0 / (g->dz * g->dz);
        g->dt_bound = 0.5 * d->re * 1.0 / inv;  // solver.c:136-139
    }
    for (int b = 0; b < kBufs; ++b) {
        const size_t bytes = sizeof(double) * (size_t)(g->nalloc + 2 * kSlack);
        if (hipMalloc(&g->alloc[b], bytes) != hipSuccess)
            CF(MISOR_ENOMEM, "hipMalloc of %lld doubles failed", g->nalloc);
        if (hipMemsetAsync(g->alloc[b], 0, bytes, g->stream) != hipSuccess)
            CF(MISOR_EHIP, "hipMemset failed");
        g->mem[b] = g->alloc[b] + kSlack;
        g->fld[b] = g->mem[b] + (long long)(kHalo - 1) * g->g.sxy;
    }
    g->partials_cap = 2LL * ns3_partials(g->g);
    if (g->partials_cap < 3LL * absmax3_blocks()) g->partials_cap = 3LL * absmax3_blocks();
    // the fused sweep's partials: the smallest rows / kchunk settings
    // (two sets: the folded loop test reads the previous sweep's partials)
    if (g->partials_cap < 2LL * sweep3_blocks(g->g, 4, 4))
        g->partials_cap = 2LL * sweep3_blocks(g->g, 4, 4);
    if (hipMalloc(&g->partials, sizeof(double) * (size_t)g->partials_cap) != hipSuccess ||
        hipMalloc(&g->out, sizeof(double) * 4) != hipSuccess ||
        hipHostMalloc(&g->out_host, sizeof(double) * 4, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&g->st, sizeof(DevState)) != hipSuccess ||
        hipMalloc(&g->st2, sizeof(DevState)) != hipSuccess ||
        hipHostMalloc(&g->st_host, sizeof(DevState), hipHostMallocDefault) != hipSuccess)
        CF(MISOR_ENOMEM, "allocation failed");
    if (nranks > 1) {
        if (memcmp(d->comm_id, kLocalPrefix3, sizeof kLocalPrefix3 - 1) == 0) {
            char name[MISOR_COMM_ID_BYTES + 1];
            memcpy(name, d->comm_id, MISOR_COMM_ID_BYTES);
            name[MISOR_COMM_ID_BYTES] = '\0';
            {
                std::lock_guard<std::mutex> lk(g_groups3_mu);
                auto& G = g_groups3[name];
                if (!G) {
                    G = std::make_shared<LocalGroup3>();
                    G->n = nranks;
                    G->members.assign(nranks, nullptr);
                    G->vals.assign(4 * (size_t)nranks, 0.0);
                }
                if (G->n != nranks || G->members[g->rank])
                    CF(MISOR_EINVAL, "local group %s: bad rank/size", name);
                G->members[g->rank] = g;
                g->local = G;
                if (++G->joined == nranks) g_groups3.erase(name);  // name reusable
            }
            g->local->barrier();  // every member registered before any exchange
        } else {
            ncclUniqueId id;
            memcpy(&id, d->comm_id, sizeof id);
            if (ncclCommInitRank(&g->comm, nranks, id, g->rank) != ncclSuccess)
                CF(MISOR_ECOMM, "ncclCommInitRank failed");
        }
    }
    if (hipStreamSynchronize(g->stream) != hipSuccess) CF(MISOR_EHIP, "sync failed");
#undef CF
    *out = g;
    return MISOR_OK;
}

int misor3_local_info(const misor_grid3* g, int* kloc, int* koff) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    if (kloc) *kloc = g->g.K;
    if (koff) *koff = g->g.koff;
    return MISOR_OK;
}

static double* fld3(misor_grid3* g, int field) {
    return (field >= 0 && field < 8) ? g->fld[field] : nullptr;
}

int misor3_upload(misor_grid3* g, int field, const double* host) {
    if (!g || !host || !fld3(g, field)) return fail3(MISOR_EINVAL, "bad upload");
    HIPCHK3(hipSetDevice(g->device));
    HIPCHK3(hipMemcpyAsync(fld3(g, field), host, sizeof(double) * (size_t)g->n,
                           hipMemcpyHostToDevice, g->stream));
    HIPCHK3(hipStreamSynchronize(g->stream));
    if (field == MISOR3_P) g->alt_stale = true;
    return MISOR_OK;
}

int misor3_download(misor_grid3* g, int field, double* host) {
    if (!g || !host || !fld3(g, field)) return fail3(MISOR_EINVAL, "bad download");
    HIPCHK3(hipSetDevice(g->device));
    HIPCHK3(hipMemcpyAsync(host, fld3(g, field), sizeof(double) * (size_t)g->n,
                           hipMemcpyDeviceToHost, g->stream));
    HIPCHK3(hipStreamSynchronize(g->stream));
    return MISOR_OK;
}

// commCollectResult's gather (assignment-6/src/comm.c:246-384) of one whole
// field: rank 0 receives (imax+2)(jmax+2)(kmax+2) doubles; rank r sends its
// planes 1..K, plus plane 0 / K+1 where they are the physical ghost planes
int misor3_gather(misor_grid3* g, int field, double* host_global) {
    if (!g || !fld3(g, field)) return fail3(MISOR_EINVAL, "bad gather");
    if (g->rank == 0 && !host_global) return fail3(MISOR_EINVAL, "rank 0 needs a buffer");
    HIPCHK3(hipSetDevice(g->device));
    if (!dist(g)) return misor3_download(g, field, host_global);
    const long long sxy = g->g.sxy;
    auto range = [&](int r, int& k_first, int& k_count, long long& goff) {
        int kl = 0, ko = 0;
        misor3_decompose(g->nranks, r, g->desc.kmax, &kl, &ko);
        k_first = (r == 0) ? 0 : 1;
        const int k_last = (r == g->nranks - 1) ? kl + 1 : kl;
        k_count = k_last - k_first + 1;
        goff = (long long)(ko + k_first) * sxy;  // global plane of local plane k_first
    };
    if (g->local) {
        LocalGroup3& G = *g->local;
        HIPCHK3(hipStreamSynchronize(g->stream));
        G.barrier();
        if (g->rank == 0) {
            for (int r = 0; r < g->nranks; ++r) {
                int kf, kc;
                long long goff;
                range(r, kf, kc, goff);
                misor_grid3* q = G.members[r];
                HIPCHK3(hipSetDevice(q->device));
                HIPCHK3(hipMemcpy(host_global + goff, plane_ptr(q, field, kf),
                                  sizeof(double) * (size_t)kc * sxy, hipMemcpyDeviceToHost));
            }
            HIPCHK3(hipSetDevice(g->device));
        }
        G.barrier();
        return MISOR_OK;
    }
    int kf, kc;
    long long goff;
    range(g->rank, kf, kc, goff);
    if (g->rank != 0) {
        NCCLCHK3(ncclSend(plane_ptr(g, field, kf), (size_t)kc * sxy, ncclDouble, 0, g->comm,
                          g->stream));
        HIPCHK3(hipStreamSynchronize(g->stream));
        return MISOR_OK;
    }
    HIPCHK3(hipMemcpyAsync(host_global + goff, plane_ptr(g, field, kf),
                           sizeof(double) * (size_t)kc * sxy, hipMemcpyDeviceToHost, g->stream));
    if (!g->gstage) {
        int kmaxloc = 0;
        misor3_decompose(g->nranks, 0, g->desc.kmax, &kmaxloc, nullptr);  // rank 0 is largest
        HIPCHK3(hipMalloc(&g->gstage, sizeof(double) * (size_t)(kmaxloc + 2) * sxy));
    }
    for (int r = 1; r < g->nranks; ++r) {
        range(r, kf, kc, goff);
        NCCLCHK3(ncclRecv(g->gstage, (size_t)kc * sxy, ncclDouble, r, g->comm, g->stream));
        HIPCHK3(hipMemcpyAsync(host_global + goff, g->gstage, sizeof(double) * (size_t)kc * sxy,
                               hipMemcpyDeviceToHost, g->stream));
    }
    HIPCHK3(hipStreamSynchronize(g->stream));
    return MISOR_OK;
}

int misor3_fill(misor_grid3* g, int field, double value) {
    if (!g || !fld3(g, field)) return fail3(MISOR_EINVAL, "bad fill");
    HIPCHK3(hipSetDevice(g->device));
    launch_fill(g->stream, g->mem[field], g->nalloc, value);
    HIPCHK3(hipGetLastError());
    if (field == MISOR3_P) g->alt_stale = true;
    return MISOR_OK;
}

int misor3_set_dt(misor_grid3* g, double dt) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    g->dt = dt;
    return MISOR_OK;
}

// max |u|, |v|, |w| over every cell of the global array incl. ghosts: this
// rank's planes plus the physical ghost planes, then a max all-reduce
static int absmax_uvw(misor_grid3* g) {
    const int k_first = g->g.lo_phys ? 0 : 1, k_last = g->g.hi_phys ? g->g.K + 1 : g->g.K;
    const long long off = (long long)k_first * g->g.sxy;
    launch3_absmax(g->stream, g->fld[MISOR3_U] + off, g->fld[MISOR3_V] + off,
                   g->fld[MISOR3_W] + off, (long long)(k_last - k_first + 1) * g->g.sxy,
                   g->partials, g->out);
    HIPCHK3(hipGetLastError());
    int rc = allreduce3(g, g->out, 3, true);
    if (rc != MISOR_OK) return rc;
    HIPCHK3(hipMemcpyAsync(g->out_host, g->out, 3 * sizeof(double), hipMemcpyDeviceToHost,
                           g->stream));
    HIPCHK3(hipStreamSynchronize(g->stream));
    return MISOR_OK;
}

// computeTimestep, solver.c:340-362 (maxElement over all cells incl. ghosts)
int misor3_compute_timestep(misor_grid3* g, double* dt_out) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    int rc = absmax_uvw(g);
    if (rc != MISOR_OK) return rc;
    const double umax = g->out_host[0], vmax = g->out_host[1], wmax = g->out_host[2];
    double dt = g->dt_bound;
    if (umax > 0) dt = (dt > g->dx / umax) ? g->dx / umax : dt;
    if (vmax > 0) dt = (dt > g->dy / vmax) ? g->dy / vmax : dt;
    if (wmax > 0) dt = (dt > g->dz / wmax) ? g->dz / wmax : dt;
    g->dt = dt * g->desc.tau;
    if (dt_out) *dt_out = g->dt;
    return MISOR_OK;
}

int misor3_max_uvw(misor_grid3* g, double* mx /* 3 */) {
    if (!g || !mx) return fail3(MISOR_EINVAL, "null argument");
    HIPCHK3(hipSetDevice(g->device));
    int rc = absmax_uvw(g);
    if (rc != MISOR_OK) return rc;
    for (int q = 0; q < 3; ++q) mx[q] = g->out_host[q];
    return MISOR_OK;
}

// setBoundaryConditions, solver.c:364-577: top, bottom, left, right, front,
// back, in that order (a later wall reads cells an earlier one wrote); the
// front / back walls belong to the ranks holding the first / last plane
int misor3_set_boundary_conditions(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    const int I = g->g.I, J = g->g.J, K = g->g.K;
    double *u = g->fld[MISOR3_U], *v = g->fld[MISOR3_V], *w = g->fld[MISOR3_W];
    const misor3_desc& d = g->desc;
    launch3_wall(g->stream, g->g, v, u, w, 1, J + 1, J, J, J - 1, d.bcTop);
    launch3_wall(g->stream, g->g, v, u, w, 1, 0, 1, 0, 1, d.bcBottom);
    launch3_wall(g->stream, g->g, u, v, w, 0, 0, 1, 0, 1, d.bcLeft);
    launch3_wall(g->stream, g->g, u, v, w, 0, I + 1, I, I, I - 1, d.bcRight);
    if (g->g.lo_phys) launch3_wall(g->stream, g->g, w, u, v, 2, 0, 1, 0, 1, d.bcFront);
    if (g->g.hi_phys) launch3_wall(g->stream, g->g, w, u, v, 2, K + 1, K, K, K - 1, d.bcBack);
    HIPCHK3(hipGetLastError());
    return MISOR_OK;
}

int misor3_set_special_boundary_condition(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    launch3_special(g->stream, g->g, g->fld[MISOR3_U], g->desc.problem);
    HIPCHK3(hipGetLastError());
    return MISOR_OK;
}

// computeFG reads u, v, w one plane beyond the slab: the reference's
// commExchange of u, v, w before it (assignment-6/src/solver.c:606-610)
int misor3_compute_fg(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    for (int b : {MISOR3_U, MISOR3_V, MISOR3_W}) {
        int rc = exchange3(g, b, 1);
        if (rc != MISOR_OK) return rc;
    }
    const misor3_desc& d = g->desc;
    Fg3 c;
    c.gamma = d.gamma;
    c.iRe = 1.0 / d.re;
    c.ix = 1.0 / g->dx;
    c.iy = 1.0 / g->dy;
    c.iz = 1.0 / g->dz;
    c.dt = g->dt;
    c.gx = d.gx;
    c.gy = d.gy;
    c.gz = d.gz;
    launch3_fg(g->stream, g->g, g->fld[MISOR3_U], g->fld[MISOR3_V], g->fld[MISOR3_W],
               g->fld[MISOR3_F], g->fld[MISOR3_G], g->fld[MISOR3_H], c);
    HIPCHK3(hipGetLastError());
    return MISOR_OK;
}

// computeRHS reads h one plane below the slab (the reference's commShift)
int misor3_compute_rhs(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    int rc = exchange3(g, MISOR3_H, 1);
    if (rc != MISOR_OK) return rc;
    launch3_rhs(g->stream, g->g, g->fld[MISOR3_F], g->fld[MISOR3_G], g->fld[MISOR3_H],
                g->fld[MISOR3_RHS], 1.0 / g->dx, 1.0 / g->dy, 1.0 / g->dz, 1.0 / g->dt);
    HIPCHK3(hipGetLastError());
    return MISOR_OK;
}

int misor3_adapt_uvw(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    launch3_adapt(g->stream, g->g, g->fld[MISOR3_F], g->fld[MISOR3_G], g->fld[MISOR3_H],
                  g->fld[MISOR3_P], g->fld[MISOR3_U], g->fld[MISOR3_V], g->fld[MISOR3_W],
                  g->dt / g->dx, g->dt / g->dy, g->dt / g->dz);
    HIPCHK3(hipGetLastError());
    return MISOR_OK;
}

int misor3_normalize_pressure(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    const double cells = (double)((long long)g->g.I * g->g.J * g->desc.kmax);
    if (!dist(g)) {
        launch3_normalize(g->stream, g->g, g->fld[MISOR3_P], g->partials, g->out, cells);
    } else {
        launch3_interior_sum(g->stream, g->g, g->fld[MISOR3_P], g->partials, g->out);
        int rc = allreduce3(g, g->out, 1, false);
        if (rc != MISOR_OK) return rc;
        launch3_sub_mean(g->stream, g->g, g->fld[MISOR3_P], g->out, cells);
    }
    HIPCHK3(hipGetLastError());
    return MISOR_OK;
}

static int auto_kchunk(const G3& g, int rows) {
    // enough workgroups to fill 256 CUs twice over, chunks of at least 8 planes
    int kc = 64;
    while (kc > 8 && sweep3_blocks(g, rows, kc) < 2048) kc /= 2;
    return kc;
}

// solve, solver.c:175-297: red-black SOR with the reference's residual
// (carried over between iterations); batches of iterations are enqueued and
// the device-resident state is read once per batch.  Default: the fused
// sweep, one launch per iteration, ping-ponging between fld[P] and its
// partner (launches after the loop test fails are no-ops, so the result is in
// the buffer of parity `it`; the pointers are swapped so fld[P] holds it).
// The edge and corner ghosts are never written by a sweep, so the partner
// gets a copy of fld[P] whenever P was set from outside.
//
// Decomposed: the sweep writes its slab's sum of r^2, an all-reduce adds the
// ranks' sums and the decide kernel applies the loop test on every rank (so
// every rank stops after the same iteration); after each sweep the new
// buffer's 2-deep halo is exchanged.  The loop is the single-domain one, so
// p and the iteration count do not depend on the slab count (only the order
// of the residual's sum does).  After the loop test fails, the remaining
// launches of a batch are no-ops and their exchanges move final planes
// between buffers of the same parity on every rank.
int misor3_solve(misor_grid3* g, int* iters, double* res) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    const misor3_desc& d = g->desc;
    const double dx2 = g->dx * g->dx, dy2 = g->dy * g->dy, dz2 = g->dz * g->dz;
    const double factor = d.omega * 0.5 * (dx2 * dy2 * dz2) / (dy2 * dz2 + dx2 * dz2 + dx2 * dy2);
    const double cells = (double)((long long)g->g.I * g->g.J * d.kmax);
    DevState s0{};
    s0.res = 1.0;
    s0.epssq = d.eps * d.eps;
    s0.itermax = d.itermax;
    s0.done = !((s0.res >= s0.epssq) && (0 < d.itermax));
    if (s0.done) {
        if (iters) *iters = 0;
        if (res) *res = 1.0;
        return MISOR_OK;
    }
    // p resident in LDS, one cooperative launch for the whole solve (ns3d_resident.hip)
    if (!dist(g) && g->resident != 0 && resident3_boxes(g->g) > 0) {
        // barrier state + 2 x 256 partials, and a mailbox of p's layout for the
        // box-surface cells, in uncached memory: coherent across the XCDs' L2s
        // without cache write-backs / invalidations at every barrier
        if (!g->rbar)
            HIPCHK3(hipExtMallocWithFlags(&g->rbar, resident3_bar_bytes() + 2 * 256 * sizeof(double),
                                          hipDeviceMallocUncached));
        if (!g->rmbox)
            HIPCHK3(hipExtMallocWithFlags(reinterpret_cast<void**>(&g->rmbox),
                                          2 * sizeof(double) * (size_t)g->nalloc,
                                          hipDeviceMallocUncached));
        double* const rpart =
            reinterpret_cast<double*>(static_cast<char*>(g->rbar) + resident3_bar_bytes());
        double* const mbox0 = g->rmbox + (g->fld[MISOR3_P] - g->mem[MISOR3_P]);
        *g->st_host = s0;
        if (g->timing) HIPCHK3(hipEventRecord(g->ev[0], g->stream));
        HIPCHK3(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice,
                               g->stream));
        const int lr = launch3_resident(g->stream, g->g, g->fld[MISOR3_P], g->fld[MISOR3_RHS],
                                        1.0 / dx2, 1.0 / dy2, 1.0 / dz2, factor, cells,
                                        rpart, g->st, g->rbar, mbox0);
        if (lr < 0) return fail3(MISOR_EHIP, "resident solve: launch failed");
        if (lr == 0) {
            if (g->timing) HIPCHK3(hipEventRecord(g->ev[1], g->stream));
            HIPCHK3(hipMemcpyAsync(g->st_host, g->st, sizeof(DevState), hipMemcpyDeviceToHost,
                                   g->stream));
            int aborted = 0;
            if (resident3_aborted(g->rbar, g->stream, &aborted) != 0)
                return fail3(MISOR_EHIP, "resident solve: state readback failed");
            if (aborted)
                return fail3(MISOR_EHIP, "resident solve: a grid barrier timed out (p undefined)");
            g->alt_stale = true;  // the fused sweep's partner buffer no longer matches p
            g->last_iters = g->st_host->it;
            if (g->timing) {
                float ms = 0.f;
                HIPCHK3(hipEventElapsedTime(&ms, g->ev[0], g->ev[1]));
                g->solve_ms += ms;
                g->solve_iters += g->st_host->it;
            }
            if (iters) *iters = g->st_host->it;
            if (res) *res = g->st_host->res;
            return MISOR_OK;
        }
        // lr == 1: the device refused the cooperative grid -- the streaming sweep below
    }
    const bool fused = g->sweep != 0;
    if (!fused && dist(g)) return fail3(MISOR_ESTATE, "the two-pass solve is single-rank only");
    const int kc = g->kchunk > 0 ? g->kchunk : auto_kchunk(g->g, g->rows);
    // rhs two plane steps ahead pays on long marches (384^3, 32 planes: 0.384 ->
    // 0.376 ms per iteration) and costs on short ones (128^3, 8 planes: 27.4 ->
    // 28.1 us; profiles/r02_tune3d_ra2.txt)
    const bool ra2 = g->rhs_ahead ? g->rhs_ahead == 2 : kc >= 16;
    // single rank: the loop test of sweep m runs inside sweep m+1 (k3_sweep,
    // Fold3); the state alternates between st and st2, the partials between
    // the two halves of g->partials
    const bool fold = fused && !dist(g) && g->fold;
    DevState* const stb[2] = {g->st, g->st2};
    const long long half = g->partials_cap / 2;
    double* const part[2] = {g->partials, g->partials + half};
    int sx = 0;  // the state buffer that holds the current state
    *g->st_host = s0;
    if (g->timing) HIPCHK3(hipEventRecord(g->ev[0], g->stream));
    HIPCHK3(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice,
                           g->stream));
    int rc;
    if (fused && g->alt_stale) {
        HIPCHK3(hipMemcpyAsync(g->mem[kAlt], g->mem[MISOR3_P], sizeof(double) * (size_t)g->nalloc,
                               hipMemcpyDeviceToDevice, g->stream));
        g->alt_stale = false;
    }
    if (dist(g)) {  // halos of p (2 deep) and rhs (1 deep, red on halo planes)
        if ((rc = exchange3(g, MISOR3_P, kHalo)) != MISOR_OK) return rc;
        if ((rc = exchange3(g, MISOR3_RHS, 1)) != MISOR_OK) return rc;
    }
    const int bufs[2] = {MISOR3_P, kAlt};
    double* buf[2] = {g->fld[MISOR3_P], g->fld[kAlt]};
    long long launched = 0;
    int batch = g->last_iters > 8 ? g->last_iters : 8;
    if (dist(g) && g->local) batch = 1;  // host-synchronised transport: no batching gain
    for (;;) {
        if (batch > d.itermax - launched) batch = (int)(d.itermax - launched);
        if (batch < 1) batch = 1;
        for (int b = 0; b < batch; ++b) {
            const long long m = launched + b;
            if (fold) {
                launch3_sweep_folded(g->stream, g->g, buf[m & 1], buf[(m + 1) & 1],
                                     g->fld[MISOR3_RHS], 1.0 / dx2, 1.0 / dy2, 1.0 / dz2, factor,
                                     g->rows, kc, part[m & 1], b == 0 ? nullptr : part[(m - 1) & 1],
                                     stb[sx], stb[sx ^ 1], cells, ra2);
                sx ^= 1;
                continue;
            }
            if (!fused) {
                launch3_rb_iteration(g->stream, g->g, g->fld[MISOR3_P], g->fld[MISOR3_RHS],
                                     1.0 / dx2, 1.0 / dy2, 1.0 / dz2, factor, g->partials,
                                     g->st, cells);
                continue;
            }
            launch3_sweep(g->stream, g->g, buf[m & 1], buf[(m + 1) & 1], g->fld[MISOR3_RHS],
                          1.0 / dx2, 1.0 / dy2, 1.0 / dz2, factor, g->rows, kc, g->partials,
                          g->st, cells, dist(g), ra2);
            if (dist(g)) {
                if ((rc = allreduce3(g, &g->st->sum[0], 1, false)) != MISOR_OK) return rc;
                launch3_decide(g->stream, g->st, cells);
                // the halo of the new buffer: by index, so the LOCAL transport finds
                // the same buffer on the neighbour (every rank swaps alike)
                const int nb = bufs[(m + 1) & 1];
                if ((rc = exchange3(g, nb, kHalo)) != MISOR_OK) return rc;
            }
        }
        if (fold) {  // the loop test of the batch's last sweep
            launch3_fold_decide(g->stream, g->g, g->rows, kc, part[(launched + batch - 1) & 1],
                                stb[sx], stb[sx ^ 1], cells);
            sx ^= 1;
        }
        HIPCHK3(hipGetLastError());
        launched += batch;
        if (g->timing) HIPCHK3(hipEventRecord(g->ev[1], g->stream));
        HIPCHK3(hipMemcpyAsync(g->st_host, stb[sx], sizeof(DevState), hipMemcpyDeviceToHost,
                               g->stream));
        HIPCHK3(hipStreamSynchronize(g->stream));
        if (g->st_host->done || launched >= d.itermax) break;
        batch = (dist(g) && g->local) ? 1 : (batch < 512 ? 2 * batch : 1024);
    }
    g->last_iters = g->st_host->it;
    if (fused && (g->st_host->it & 1)) {
        std::swap(g->fld[MISOR3_P], g->fld[kAlt]);
        std::swap(g->mem[MISOR3_P], g->mem[kAlt]);
        std::swap(g->alloc[MISOR3_P], g->alloc[kAlt]);
    }
    if (g->timing) {
        float ms = 0.f;
        HIPCHK3(hipEventElapsedTime(&ms, g->ev[0], g->ev[1]));
        g->solve_ms += ms;
        g->solve_iters += g->st_host->it;
    }
    if (iters) *iters = g->st_host->it;
    if (res) *res = g->st_host->res;
    return MISOR_OK;
}

int misor3_set_tuning(misor_grid3* g, int key, int value) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    switch (key) {
    case MISOR3_TUNE_SWEEP:
        if (value != 0 && value != 1) return fail3(MISOR_EINVAL, "sweep must be 0 or 1");
        if (value == 0 && dist(g))
            return fail3(MISOR_EINVAL, "the two-pass solve is single-rank only");
        g->sweep = value;
        return MISOR_OK;
    case MISOR3_TUNE_ROWS:
        if (value != 4 && value != 8 && value != 12)
            return fail3(MISOR_EINVAL, "rows must be 4, 8 or 12");
        g->rows = value;
        return MISOR_OK;
    case MISOR3_TUNE_KCHUNK:
        if (value != 0 && value < 4) return fail3(MISOR_EINVAL, "kchunk must be 0 or >= 4");
        g->kchunk = value;
        return MISOR_OK;
    case MISOR3_TUNE_FOLD: g->fold = value != 0; return MISOR_OK;
    case MISOR3_TUNE_RHS_AHEAD:
        if (value < 0 || value > 2) return fail3(MISOR_EINVAL, "rhs_ahead must be 0, 1 or 2");
        g->rhs_ahead = value;
        return MISOR_OK;
    case MISOR3_TUNE_RESIDENT:
        if (value < -1 || value > 1) return fail3(MISOR_EINVAL, "resident must be -1, 0 or 1");
        g->resident = value;
        return MISOR_OK;
    }
    return fail3(MISOR_EINVAL, "unknown tuning key %d", key);
}

int misor3_get_tuning(const misor_grid3* g, int key, int* value) {
    if (!g || !value) return fail3(MISOR_EINVAL, "null argument");
    switch (key) {
    case MISOR3_TUNE_SWEEP: *value = g->sweep; return MISOR_OK;
    case MISOR3_TUNE_ROWS: *value = g->rows; return MISOR_OK;
    case MISOR3_TUNE_KCHUNK:
        *value = g->kchunk > 0 ? g->kchunk : auto_kchunk(g->g, g->rows);
        return MISOR_OK;
    case MISOR3_TUNE_FOLD: *value = g->fold; return MISOR_OK;
    case MISOR3_TUNE_RHS_AHEAD: *value = g->rhs_ahead; return MISOR_OK;
    case MISOR3_TUNE_RESIDENT:
        *value = !dist(g) && g->resident != 0 && resident3_boxes(g->g) > 0;
        return MISOR_OK;
    }
    return fail3(MISOR_EINVAL, "unknown tuning key %d", key);
}

int misor3_enable_timing(misor_grid3* g, int on) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    if (on && !g->ev[0])
        for (auto& e : g->ev) HIPCHK3(hipEventCreate(&e));
    g->timing = on != 0;
    g->solve_ms = 0;
    g->solve_iters = 0;
    return MISOR_OK;
}

int misor3_get_solve_time(const misor_grid3* g, double* ms, long long* iters) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    if (ms) *ms = g->solve_ms;
    if (iters) *iters = g->solve_iters;
    return MISOR_OK;
}

int misor3_synchronize(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipStreamSynchronize(g->stream));
    return MISOR_OK;
}

}  // extern "C"
