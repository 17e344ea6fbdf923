// misor3d_api.hip -- the C ABI of the 3D path (include/misor.h, misor3_*):
// assignment-6's 3D Navier-Stokes solver (assignment-6/src/solver.c) on one
// GPU.  The entry points mirror the reference's solver.h one to one; fields
// are device-resident in the reference layout.

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>

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

}  // namespace

struct misor_grid3 {
    int device = 0;
    hipStream_t stream = nullptr;
    misor3_desc desc{};
    G3 g{};
    long long n = 0;           // cells incl. ghosts
    double* fld[8] = {};       // MISOR3_P .. MISOR3_H
    double* p_alt = nullptr;   // ping-pong partner of fld[P] for the fused sweep
    bool alt_stale = true;     // p_alt's edge/corner ghosts may differ from fld[P]'s
    int sweep = 1;             // MISOR3_TUNE_SWEEP
    int rows = 8;              // MISOR3_TUNE_ROWS
    int kchunk = 0;            // MISOR3_TUNE_KCHUNK (0: automatic)
    double dx = 0, dy = 0, dz = 0, dt = 0, dt_bound = 0;
    double* partials = nullptr;  // 2 * ns3_partials (solve), also reductions
    long long partials_cap = 0;
    double* out = nullptr;      // 4 doubles on the device (maxima / sum)
    double* out_host = nullptr; // pinned
    DevState* st = nullptr;
    DevState* st_host = nullptr;
    int last_iters = 0;
    bool timing = false;          // misor3_enable_timing
    hipEvent_t ev[2] = {};        // around each solve, on the grid's stream
    double solve_ms = 0;          // accumulated device time of timed solves
    long long solve_iters = 0;    // iterations of the timed solves
};

extern "C" {

void misor3_destroy(misor_grid3* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (auto& f : g->fld)
        if (f) (void)hipFree(f);
    (void)hipFree(g->p_alt);
    (void)hipFree(g->partials);
    (void)hipFree(g->out);
    (void)hipHostFree(g->out_host);
    (void)hipFree(g->st);
    (void)hipHostFree(g->st_host);
    for (auto& e : g->ev)
        if (e) (void)hipEventDestroy(e);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

int misor3_create(misor_grid3** out, const misor3_desc* d) {
    if (!out || !d) return fail3(MISOR_EINVAL, "null argument");
    *out = nullptr;
    if (d->imax < 2 || d->jmax < 2 || d->kmax < 2)
        return fail3(MISOR_EINVAL, "imax, jmax, kmax must be >= 2");
    misor_grid3* g = new misor_grid3();
    g->desc = *d;
    g->device = d->device;
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
    g->g.K = d->kmax;
    g->g.sx = d->imax + 2;
    g->g.sxy = (long long)(d->imax + 2) * (d->jmax + 2);
    g->n = g->g.sxy * (d->kmax + 2);
    // initSolver, solver.c:86-95
    g->dx = d->xlength / d->imax;
    g->dy = d->ylength / d->jmax;
    g->dz = d->zlength / d->kmax;
    {
        const double inv = 1.0 / (g->dx * g->dx) + 1.0 / (g->dy * g->dy) + 1.0 / (g->dz * g->dz);
        g->dt_bound = 0.5 * d->re * 1.0 / inv;  // solver.c:136-139
    }
    for (auto& f : g->fld) {
        if (hipMalloc(&f, sizeof(double) * (size_t)g->n) != hipSuccess)
            CF(MISOR_ENOMEM, "hipMalloc of %lld doubles failed", g->n);
        if (hipMemsetAsync(f, 0, sizeof(double) * (size_t)g->n, g->stream) != hipSuccess)
            CF(MISOR_EHIP, "hipMemset failed");
    }
    if (hipMalloc(&g->p_alt, sizeof(double) * (size_t)g->n) != hipSuccess)
        CF(MISOR_ENOMEM, "hipMalloc of %lld doubles failed", g->n);
    g->partials_cap = 2LL * ns3_partials(g->g);
    if (g->partials_cap < 3LL * absmax3_blocks()) g->partials_cap = 3LL * absmax3_blocks();
    // the fused sweep's partials: the smallest rows / kchunk settings
    if (g->partials_cap < sweep3_blocks(g->g, 4, 4)) g->partials_cap = sweep3_blocks(g->g, 4, 4);
    if (hipMalloc(&g->partials, sizeof(double) * (size_t)g->partials_cap) != hipSuccess ||
        hipMalloc(&g->out, sizeof(double) * 4) != hipSuccess ||
        hipHostMalloc(&g->out_host, sizeof(double) * 4, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&g->st, sizeof(DevState)) != hipSuccess ||
        hipHostMalloc(&g->st_host, sizeof(DevState), hipHostMallocDefault) != hipSuccess)
        CF(MISOR_ENOMEM, "allocation failed");
    if (hipStreamSynchronize(g->stream) != hipSuccess) CF(MISOR_EHIP, "sync failed");
#undef CF
    *out = g;
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

int misor3_fill(misor_grid3* g, int field, double value) {
    if (!g || !fld3(g, field)) return fail3(MISOR_EINVAL, "bad fill");
    HIPCHK3(hipSetDevice(g->device));
    launch_fill(g->stream, fld3(g, field), g->n, value);
    HIPCHK3(hipGetLastError());
    if (field == MISOR3_P) g->alt_stale = true;
    return MISOR_OK;
}

int misor3_set_dt(misor_grid3* g, double dt) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    g->dt = dt;
    return MISOR_OK;
}

// computeTimestep, solver.c:340-362 (maxElement over all cells incl. ghosts)
int misor3_compute_timestep(misor_grid3* g, double* dt_out) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    launch3_absmax(g->stream, g->fld[MISOR3_U], g->fld[MISOR3_V], g->fld[MISOR3_W], g->n,
                   g->partials, g->out);
    HIPCHK3(hipGetLastError());
    HIPCHK3(hipMemcpyAsync(g->out_host, g->out, 3 * sizeof(double), hipMemcpyDeviceToHost,
                           g->stream));
    HIPCHK3(hipStreamSynchronize(g->stream));
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
    launch3_absmax(g->stream, g->fld[MISOR3_U], g->fld[MISOR3_V], g->fld[MISOR3_W], g->n,
                   g->partials, g->out);
    HIPCHK3(hipMemcpyAsync(g->out_host, g->out, 3 * sizeof(double), hipMemcpyDeviceToHost,
                           g->stream));
    HIPCHK3(hipStreamSynchronize(g->stream));
    for (int q = 0; q < 3; ++q) mx[q] = g->out_host[q];
    return MISOR_OK;
}

// setBoundaryConditions, solver.c:364-577: top, bottom, left, right, front,
// back, in that order (a later wall reads cells an earlier one wrote)
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
    launch3_wall(g->stream, g->g, w, u, v, 2, 0, 1, 0, 1, d.bcFront);
    launch3_wall(g->stream, g->g, w, u, v, 2, K + 1, K, K, K - 1, d.bcBack);
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

int misor3_compute_fg(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
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

int misor3_compute_rhs(misor_grid3* g) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
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
    launch3_normalize(g->stream, g->g, g->fld[MISOR3_P], g->partials, g->out,
                      (double)((long long)g->g.I * g->g.J * g->g.K));
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
// sweep, one launch per iteration, ping-ponging between fld[P] and p_alt
// (launches after the loop test fails are no-ops, so the result is in the
// buffer of parity `it`; the pointers are swapped so fld[P] holds it).  The
// edge and corner ghosts are never written by a sweep, so p_alt gets a copy
// of fld[P] whenever P was set from outside.
int misor3_solve(misor_grid3* g, int* iters, double* res) {
    if (!g) return fail3(MISOR_EINVAL, "null grid");
    HIPCHK3(hipSetDevice(g->device));
    const misor3_desc& d = g->desc;
    const double dx2 = g->dx * g->dx, dy2 = g->dy * g->dy, dz2 = g->dz * g->dz;
    const double factor = d.omega * 0.5 * (dx2 * dy2 * dz2) / (dy2 * dz2 + dx2 * dz2 + dx2 * dy2);
    const double cells = (double)((long long)g->g.I * g->g.J * g->g.K);
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
    *g->st_host = s0;
    if (g->timing) HIPCHK3(hipEventRecord(g->ev[0], g->stream));
    HIPCHK3(hipMemcpyAsync(g->st, g->st_host, sizeof(DevState), hipMemcpyHostToDevice,
                           g->stream));
    const bool fused = g->sweep != 0;
    const int kc = g->kchunk > 0 ? g->kchunk : auto_kchunk(g->g, g->rows);
    if (fused && g->alt_stale) {
        HIPCHK3(hipMemcpyAsync(g->p_alt, g->fld[MISOR3_P], sizeof(double) * (size_t)g->n,
                               hipMemcpyDeviceToDevice, g->stream));
        g->alt_stale = false;
    }
    double* buf[2] = {g->fld[MISOR3_P], g->p_alt};
    long long launched = 0;
    int batch = g->last_iters > 8 ? g->last_iters : 8;
    for (;;) {
        if (batch > d.itermax - launched) batch = (int)(d.itermax - launched);
        if (batch < 1) batch = 1;
        for (int b = 0; b < batch; ++b) {
            if (fused) {
                const long long m = launched + b;
                launch3_sweep(g->stream, g->g, buf[m & 1], buf[(m + 1) & 1], g->fld[MISOR3_RHS],
                              1.0 / dx2, 1.0 / dy2, 1.0 / dz2, factor, g->rows, kc, g->partials,
                              g->st, cells);
            } else {
                launch3_rb_iteration(g->stream, g->g, g->fld[MISOR3_P], g->fld[MISOR3_RHS],
                                     1.0 / dx2, 1.0 / dy2, 1.0 / dz2, factor, g->partials,
                                     g->st, cells);
            }
        }
        HIPCHK3(hipGetLastError());
        launched += batch;
        if (g->timing) HIPCHK3(hipEventRecord(g->ev[1], g->stream));
        HIPCHK3(hipMemcpyAsync(g->st_host, g->st, sizeof(DevState), hipMemcpyDeviceToHost,
                               g->stream));
        HIPCHK3(hipStreamSynchronize(g->stream));
        if (g->st_host->done || launched >= d.itermax) break;
        batch = batch < 512 ? 2 * batch : 1024;
    }
    g->last_iters = g->st_host->it;
    if (fused && (g->st_host->it & 1)) {
        g->fld[MISOR3_P] = buf[1];
        g->p_alt = buf[0];
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
