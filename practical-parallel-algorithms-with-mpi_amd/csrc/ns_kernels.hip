// ns_kernels.hip -- the 2D Navier-Stokes step around the pressure solve,
// assignment-5/sequential/src/solver.c, on the padded HBM layout of
// misor_internal.h.  All kernels are HBM-bandwidth bound FP64 stencils or
// O(perimeter) boundary updates; expression order follows the reference and
// the file is compiled with -ffp-contract=off, so every per-cell value is
// bit-identical to the CPU.  Only the two reductions whose result depends on
// summation order (normalizePressure's mean) differ from the CPU in rounding.

#include "misor_internal.h"

namespace misor {

namespace {

struct Lay {
    double* a;
    long long pitch;
    __device__ __forceinline__ double& operator()(int i, int j) const {
        return a[(long long)(j + kYOff) * pitch + (i + kXOff)];
    }
};
struct CLay {
    const double* a;
    long long pitch;
    __device__ __forceinline__ double operator()(int i, int j) const {
        return a[(long long)(j + kYOff) * pitch + (i + kXOff)];
    }
};

// a store the kernel never reads back (NT: nontemporal, streamed past the
// caches).  fg_rhs / adapt_absmax store NT by default (MISOR_NS_NT=0: plain
// stores): config 5's fg_rhs 1.93 vs 1.97 ms, adapt_absmax unchanged, the step
// 22.26 vs 22.36 ms over three alternated pairs (profiles/r05_ns_nt_ab.txt)
template <bool NT, class V>
__device__ __forceinline__ void put(V* p, V v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else    *p = v;
}

constexpr int kTx = 64, kTy = 4;

}  // namespace

// ---- setBoundaryConditions, :236-337.  The reference applies left, right,
// bottom, top in that order and bottom/top read cells that left/right wrote
// (U(imax,1), ...), so the walls run as two dependent launches:
// phase 0 = left + right (loop over j), phase 1 = bottom + top (loop over i).
__global__ void bc_lr_kernel(Lay u, Lay v, int ni, int nj, int bcl, int bcr, int wl, int wr) {
    const int j = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    if (j > nj) return;
    if (wl) {
        switch (bcl) {
        case MISOR_NOSLIP: u(0, j) = 0.0; v(0, j) = -v(1, j); break;
        case MISOR_SLIP: u(0, j) = 0.0; v(0, j) = v(1, j); break;
        case MISOR_OUTFLOW: u(0, j) = u(1, j); v(0, j) = v(1, j); break;
        default: break;
        }
    }
    if (wr) {
        switch (bcr) {
        case MISOR_NOSLIP: u(ni, j) = 0.0; v(ni + 1, j) = -v(ni, j); break;
        case MISOR_SLIP: u(ni, j) = 0.0; v(ni + 1, j) = v(ni, j); break;
        case MISOR_OUTFLOW: u(ni, j) = u(ni - 1, j); v(ni + 1, j) = v(ni, j); break;
        default: break;
        }
    }
}

__global__ void bc_bt_kernel(Lay u, Lay v, int ni, int nj, int bcb, int bct, int wb, int wt) {
    const int i = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i > ni) return;
    if (wb) {
        switch (bcb) {
        case MISOR_NOSLIP: v(i, 0) = 0.0; u(i, 0) = -u(i, 1); break;
        case MISOR_SLIP: v(i, 0) = 0.0; u(i, 0) = u(i, 1); break;
        case MISOR_OUTFLOW: u(i, 0) = u(i, 1); v(i, 0) = v(i, 1); break;
        default: break;
        }
    }
    if (wt) {
        switch (bct) {
        case MISOR_NOSLIP: v(i, nj) = 0.0; u(i, nj + 1) = -u(i, nj); break;
        case MISOR_SLIP: v(i, nj) = 0.0; u(i, nj + 1) = u(i, nj); break;
        case MISOR_OUTFLOW: u(i, nj + 1) = u(i, nj); v(i, nj) = v(i, nj - 1); break;
        default: break;
        }
    }
}

void launch_set_bc(const NsLaunch& L, double* u, double* v) {
    Lay U{u, L.pitch}, V{v, L.pitch};
    hipLaunchKernelGGL(bc_lr_kernel, dim3((L.nj + 255) / 256), dim3(256), 0, L.s, U, V, L.ni,
                       L.nj, L.prm.bc_left, L.prm.bc_right, L.wall_left, L.wall_right);
    hipLaunchKernelGGL(bc_bt_kernel, dim3((L.ni + 255) / 256), dim3(256), 0, L.s, U, V, L.ni,
                       L.nj, L.prm.bc_bottom, L.prm.bc_top, L.wall_bottom, L.wall_top);
}

// ---- setSpecialBoundaryCondition, :339-358
// dcavity: U(i, jmax+1) = 2 - U(i, jmax) for GLOBAL i = 1 .. imax-1 (not imax)
// canal:   U(0, j) = y (ylength - y) 4 / ylength^2,  y = dy (j - 1/2)
__global__ void special_bc_kernel(Lay u, int ni, int nj, int problem, int wt, int wl, int ioff,
                                  int joff, int imax_global, double dy, double ylength) {
    const int k = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    if (problem == MISOR_PROBLEM_DCAVITY) {
        if (wt && k <= ni && ioff + k < imax_global) u(k, nj + 1) = 2.0 - u(k, nj);
    } else if (problem == MISOR_PROBLEM_CANAL) {
        if (wl && k <= nj) {
            const int jg = joff + k;
            const double y = dy * (jg - 0.5);
            u(0, k) = y * (ylength - y) * 4.0 / (ylength * ylength);
        }
    }
}

void launch_special_bc(const NsLaunch& L, double* u) {
    const int n = L.ni > L.nj ? L.ni : L.nj;
    hipLaunchKernelGGL(special_bc_kernel, dim3((n + 255) / 256), dim3(256), 0, L.s,
                       Lay{u, L.pitch}, L.ni, L.nj, L.prm.problem, L.wall_top, L.wall_left,
                       L.ioff, L.joff, L.imax_g, L.prm.dy, L.prm.ylength);
}

// ---- computeFG, :360-436 (+ its F/G boundary lines :426-435 on wall ranks)
//
// Column march: a thread owns column i and walks up a band of kFgBand rows,
// keeping rows j-1, j, j+1 of u and v (each at i-1, i, i+1) in registers, so
// each row of u and v is loaded once per band (its x-neighbours hit in L1)
// instead of once per stencil use; consecutive lanes are consecutive columns
// (coalesced).  Per-cell arithmetic is the reference's, term by term.
constexpr int kFgBand = 32;

struct Uv3 {  // u and v at i-1, i, i+1 of one row
    double um, uc, up, vm, vc, vp;
};

__device__ __forceinline__ Uv3 load_uv3(const CLay& u, const CLay& v, int i, int j) {
    Uv3 r;
    r.um = u(i - 1, j);
    r.uc = u(i, j);
    r.up = u(i + 1, j);
    r.vm = v(i - 1, j);
    r.vc = v(i, j);
    r.vp = v(i + 1, j);
    return r;
}

__global__ __launch_bounds__(kTx* kTy) void fg_kernel(CLay u, CLay v, Lay f, Lay g, int ni,
                                                      int nj, double dt, double inverseRe,
                                                      double inverseDx, double inverseDy,
                                                      double gamma, double gx, double gy,
                                                      int wl, int wr, int wb, int wt) {
    const int i = 1 + blockIdx.x * kTx + threadIdx.x;
    const int j0 = 1 + (blockIdx.y * kTy + threadIdx.y) * kFgBand;
    if (i > ni || j0 > nj) return;
    const int j1 = min(nj, j0 + kFgBand - 1);
    Uv3 S = load_uv3(u, v, i, j0 - 1), C = load_uv3(u, v, i, j0), N = load_uv3(u, v, i, j0 + 1);
    for (int j = j0; j <= j1; ++j) {
        Uv3 NN;
        if (j + 2 <= nj + 1) NN = load_uv3(u, v, i, j + 2);  // next row, one step ahead
        const double uc = C.uc, ue = C.up, uw = C.um;
        const double un = N.uc, us = S.uc, unw = N.um;
        const double vc = C.vc, ve = C.vp, vw = C.vm;
        const double vn = N.vc, vs = S.vc, vse = S.vp;

        const double du2dx = inverseDx * 0.25 * ((uc + ue) * (uc + ue) - (uc + uw) * (uc + uw)) +
                             gamma * inverseDx * 0.25 *
                                 (fabs(uc + ue) * (uc - ue) + fabs(uc + uw) * (uc - uw));
        const double duvdy = inverseDy * 0.25 * ((vc + ve) * (uc + un) - (vs + vse) * (uc + us)) +
                             gamma * inverseDy * 0.25 *
                                 (fabs(vc + ve) * (uc - un) + fabs(vs + vse) * (uc - us));
        const double du2dx2 = inverseDx * inverseDx * (ue - 2.0 * uc + uw);
        const double du2dy2 = inverseDy * inverseDy * (un - 2.0 * uc + us);
        double fv = uc + dt * (inverseRe * (du2dx2 + du2dy2) - du2dx - duvdy + gx);

        const double duvdx = inverseDx * 0.25 * ((uc + un) * (vc + ve) - (uw + unw) * (vc + vw)) +
                             gamma * inverseDx * 0.25 *
                                 (fabs(uc + un) * (vc - ve) + fabs(uw + unw) * (vc - vw));
        const double dv2dy = inverseDy * 0.25 * ((vc + vn) * (vc + vn) - (vc + vs) * (vc + vs)) +
                             gamma * inverseDy * 0.25 *
                                 (fabs(vc + vn) * (vc - vn) + fabs(vc + vs) * (vc - vs));
        const double dv2dx2 = inverseDx * inverseDx * (ve - 2.0 * vc + vw);
        const double dv2dy2 = inverseDy * inverseDy * (vn - 2.0 * vc + vs);
        double gv = vc + dt * (inverseRe * (dv2dx2 + dv2dy2) - duvdx - dv2dy + gy);

        // boundary of F / G (:426-435) overrides the interior value at i = imax / j = jmax
        if (wr && i == ni) fv = uc;
        if (wt && j == nj) gv = vc;
        f(i, j) = fv;
        g(i, j) = gv;
        if (wl && i == 1) f(0, j) = uw;
        if (wb && j == 1) g(i, 0) = vs;
        S = C;
        C = N;
        N = NN;
    }
}

void launch_compute_fg(const NsLaunch& L, const double* u, const double* v, double* f,
                       double* g) {
    const int bands = (L.nj + kFgBand - 1) / kFgBand;
    dim3 grid((L.ni + kTx - 1) / kTx, (bands + kTy - 1) / kTy);
    const NsParams& P = L.prm;
    hipLaunchKernelGGL(fg_kernel, grid, dim3(kTx, kTy), 0, L.s, CLay{u, L.pitch},
                       CLay{v, L.pitch}, Lay{f, L.pitch}, Lay{g, L.pitch}, L.ni, L.nj, P.dt,
                       1.0 / P.re, 1.0 / P.dx, 1.0 / P.dy, P.gamma, P.gx, P.gy, L.wall_left,
                       L.wall_right, L.wall_bottom, L.wall_top);
}

// ---- computeFG fused with computeRHS (:122-138).  The reference's main loop
// (main.c:43-60) calls computeRHS right after computeFG, and RHS needs only
// F(i-1..i, j) and G(i, j-1..j): the column march has both at hand.  The lanes
// keep fg_kernel's aligned columns (lane = column i, a wave's row segment on
// whole 128-B lines); F(i-1, j) is recomputed in the lane from the same
// registers plus u(i-2, j) (the kernel is bound by HBM, not by its FP64 work,
// so the second F costs no time), and G(i, j-1) is carried in a register (the
// band's first row gets it from one extra row of the march).  One pass reads
// u, v and writes f, g, rhs: 40 B per cell instead of 32 + 24.  Every value is
// the same expression on the same operands as fg_kernel / rhs_kernel, so the
// bits are identical.  RHS cells whose F(0, j) / G(i, 0) belong to a neighbour
// rank (column 1 with a left neighbour, row 1 with a bottom one) are left to
// rhs_edge_kernel after the f, g exchange (the skeleton's shift()).
struct FgArgs {
    double dt, inverseRe, inverseDx, inverseDy, gamma, gx, gy, idx, idy, idt;
};

// F of one cell (:384-398, :415-416), operands named as in fg_kernel
__device__ __forceinline__ double f_val(const FgArgs& a, double uc, double ue, double uw,
                                        double un, double us, double vc, double ve, double vs,
                                        double vse) {
    const double inverseDx = a.inverseDx, inverseDy = a.inverseDy, gamma = a.gamma;
    const double du2dx = inverseDx * 0.25 * ((uc + ue) * (uc + ue) - (uc + uw) * (uc + uw)) +
                         gamma * inverseDx * 0.25 *
                             (fabs(uc + ue) * (uc - ue) + fabs(uc + uw) * (uc - uw));
    const double duvdy = inverseDy * 0.25 * ((vc + ve) * (uc + un) - (vs + vse) * (uc + us)) +
                         gamma * inverseDy * 0.25 *
                             (fabs(vc + ve) * (uc - un) + fabs(vs + vse) * (uc - us));
    const double du2dx2 = inverseDx * inverseDx * (ue - 2.0 * uc + uw);
    const double du2dy2 = inverseDy * inverseDy * (un - 2.0 * uc + us);
    return uc + a.dt * (a.inverseRe * (du2dx2 + du2dy2) - du2dx - duvdy + a.gx);
}

// G of one cell (:400-413, :417-418)
__device__ __forceinline__ double g_val(const FgArgs& a, const Uv3& S, const Uv3& C,
                                        const Uv3& N) {
    const double uc = C.uc, uw = C.um, un = N.uc, unw = N.um;
    const double vc = C.vc, ve = C.vp, vw = C.vm, vn = N.vc, vs = S.vc;
    const double inverseDx = a.inverseDx, inverseDy = a.inverseDy, gamma = a.gamma;
    const double duvdx = inverseDx * 0.25 * ((uc + un) * (vc + ve) - (uw + unw) * (vc + vw)) +
                         gamma * inverseDx * 0.25 *
                             (fabs(uc + un) * (vc - ve) + fabs(uw + unw) * (vc - vw));
    const double dv2dy = inverseDy * 0.25 * ((vc + vn) * (vc + vn) - (vc + vs) * (vc + vs)) +
                         gamma * inverseDy * 0.25 *
                             (fabs(vc + vn) * (vc - vn) + fabs(vc + vs) * (vc - vs));
    const double dv2dx2 = inverseDx * inverseDx * (ve - 2.0 * vc + vw);
    const double dv2dy2 = inverseDy * inverseDy * (vn - 2.0 * vc + vs);
    return vc + a.dt * (a.inverseRe * (dv2dx2 + dv2dy2) - duvdx - dv2dy + a.gy);
}

// Workgroups of kFgW columns (4 waves side by side) x one band of kFgRows
// rows, dealt to the XCDs in contiguous runs of the row-major block order:
// the workgroups an XCD runs at once are horizontal neighbours, so the lines
// at a wave's column edges (u(i-2..i-1), u(i+1), v(i+-1)) and the band's 4
// overlap rows come from its L2.  (Round 2's 64 x 4-band workgroups, dealt
// round-robin, fetched those neighbour lines from HBM: reads 1.68x the
// algorithmic 16 B/cell, profiles/r03_pmc_ns16384_base.json.)
constexpr int kFgW = 256, kFgRows = 64;

// nontemporal stores of f, g, rhs, u, v (fg_rhs 1.93 vs 1.97 ms at 16384^2,
// the NS step 22.26 vs 22.36 ms, profiles/r05_ns_nt_ab.txt); the plain-store
// instantiation is kept for A/B builds (make ab XFLAGS=-DMISOR_NS_PLAIN_STORES)
#ifdef MISOR_NS_PLAIN_STORES
static constexpr bool kNsNt = false;
#else
static constexpr bool kNsNt = true;
#endif

template <bool NT>
__global__ __launch_bounds__(kFgW) void fg_rhs_kernel(CLay u, CLay v, Lay f, Lay g, Lay rhs,
                                                      int ni, int nj, FgArgs a, int wl, int wr,
                                                      int wb, int wt, int nbx, int nblocks) {
    // XCD-aware block order: workgroup w runs on XCD w % 8; XCD x takes the
    // blocks [x nblocks / 8, (x + 1) nblocks / 8) in order
    const int w = blockIdx.x, x = w & 7, k = w >> 3;
    const int L = (int)((long long)nblocks * x / 8) + k;
    if (L >= (int)((long long)nblocks * (x + 1) / 8)) return;
    const int i = 1 + (L % nbx) * kFgW + threadIdx.x;
    const int j0 = 1 + (L / nbx) * kFgRows;
    if (i > ni || j0 > nj) return;
    const int j1 = min(nj, j0 + kFgRows - 1);
    const bool has_fl = i > 1 || wl;  // F(i-1, j) is local (F(0, j) = U(0, j) on a left wall)
    Uv3 S, C, N;
    double gprev;
    bool has_gp;
    if (j0 > 1) {  // G(i, j0-1) from one extra row of the march
        S = load_uv3(u, v, i, j0 - 2);
        C = load_uv3(u, v, i, j0 - 1);
        N = load_uv3(u, v, i, j0);
        gprev = g_val(a, S, C, N);
        has_gp = true;
        S = C;
        C = N;
        N = load_uv3(u, v, i, j0 + 1);
    } else {
        S = load_uv3(u, v, i, 0);
        C = load_uv3(u, v, i, 1);
        N = load_uv3(u, v, i, 2);
        gprev = S.vc;  // G(i, 0) = V(i, 0) on a bottom wall (:434)
        has_gp = wb != 0;
    }
    double uww = i >= 2 ? u(i - 2, j0) : 0.0;  // u(i-2, j) of the current row
    for (int j = j0; j <= j1; ++j) {
        Uv3 NN;
        if (j + 2 <= nj + 1) NN = load_uv3(u, v, i, j + 2);
        const double uww_n = (i >= 2 && j < j1) ? u(i - 2, j + 1) : 0.0;
        double fv = f_val(a, C.uc, C.up, C.um, N.uc, S.uc, C.vc, C.vp, S.vc, S.vp);
        double gv = g_val(a, S, C, N);
        // boundary of F / G (:426-435) overrides the interior value
        if (wr && i == ni) fv = C.uc;
        if (wt && j == nj) gv = C.vc;
        put<NT>(&f(i, j), fv);
        put<NT>(&g(i, j), gv);
        if (wl && i == 1) f(0, j) = C.um;
        if (wb && j == 1) g(i, 0) = S.vc;
        if (has_fl && has_gp) {
            // F(i-1, j): the same expression lane i-1 evaluates (F(0, j) = U(0, j))
            const double fl = i == 1 ? C.um
                                     : f_val(a, C.um, C.uc, uww, N.um, S.um, C.vm, C.vc, S.vm,
                                             S.vc);
            put<NT>(&rhs(i, j), a.idt * ((fv - fl) * a.idx + (gv - gprev) * a.idy));  // :131-133
        }
        gprev = gv;
        has_gp = true;
        uww = uww_n;
        S = C;
        C = N;
        N = NN;
    }
}

void launch_compute_fg_rhs(const NsLaunch& L, const double* u, const double* v, double* f,
                           double* g, double* rhs) {
    const int nbx = (L.ni + kFgW - 1) / kFgW, nby = (L.nj + kFgRows - 1) / kFgRows;
    const int nblocks = nbx * nby;
    // every XCD run has at most ceil(nblocks / 8) blocks: 8 x that many workgroups
    const int grid = 8 * ((nblocks + 7) / 8);
    const NsParams& P = L.prm;
    FgArgs a{P.dt, 1.0 / P.re, 1.0 / P.dx, 1.0 / P.dy, P.gamma, P.gx, P.gy,
             1.0 / P.dx, 1.0 / P.dy, 1.0 / P.dt};
    hipLaunchKernelGGL(fg_rhs_kernel<kNsNt>, dim3(grid), dim3(kFgW), 0, L.s, CLay{u, L.pitch},
                       CLay{v, L.pitch}, Lay{f, L.pitch}, Lay{g, L.pitch}, Lay{rhs, L.pitch},
                       L.ni, L.nj, a, L.wall_left, L.wall_right, L.wall_bottom, L.wall_top, nbx,
                       nblocks);
}

// the RHS cells fg_rhs_kernel leaves to after the f, g exchange: column 1
// (left neighbour) and row 1 (bottom neighbour); same expression as rhs_kernel
__global__ void rhs_edge_kernel(CLay f, CLay g, Lay rhs, int ni, int nj, double idx, double idy,
                                double idt, int wl, int wb) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    int i, j;
    if (k < nj) {
        if (wl) return;
        i = 1;
        j = 1 + k;
    } else if (k < nj + ni) {
        if (wb) return;
        i = 1 + (k - nj);
        j = 1;
    } else {
        return;
    }
    rhs(i, j) = idt * ((f(i, j) - f(i - 1, j)) * idx + (g(i, j) - g(i, j - 1)) * idy);
}

void launch_rhs_edges(const NsLaunch& L, const double* f, const double* g, double* rhs) {
    const int n = L.ni + L.nj;
    hipLaunchKernelGGL(rhs_edge_kernel, dim3((n + 255) / 256), dim3(256), 0, L.s,
                       CLay{f, L.pitch}, CLay{g, L.pitch}, Lay{rhs, L.pitch}, L.ni, L.nj,
                       1.0 / L.prm.dx, 1.0 / L.prm.dy, 1.0 / L.prm.dt, L.wall_left,
                       L.wall_bottom);
}

// ---- computeRHS, :122-138
__global__ void rhs_kernel(CLay f, CLay g, Lay rhs, int ni, int nj, double idx, double idy,
                           double idt) {
    const int i = 1 + blockIdx.x * kTx + threadIdx.x;
    const int j = 1 + blockIdx.y * kTy + threadIdx.y;
    if (i > ni || j > nj) return;
    rhs(i, j) = idt * ((f(i, j) - f(i - 1, j)) * idx + (g(i, j) - g(i, j - 1)) * idy);
}

void launch_compute_rhs(const NsLaunch& L, const double* f, const double* g, double* rhs) {
    dim3 grid((L.ni + kTx - 1) / kTx, (L.nj + kTy - 1) / kTy);
    hipLaunchKernelGGL(rhs_kernel, grid, dim3(kTx, kTy), 0, L.s, CLay{f, L.pitch},
                       CLay{g, L.pitch}, Lay{rhs, L.pitch}, L.ni, L.nj, 1.0 / L.prm.dx,
                       1.0 / L.prm.dy, 1.0 / L.prm.dt);
}

// ---- adaptUV, :438-455
__global__ void adapt_kernel(CLay f, CLay g, CLay p, Lay u, Lay v, int ni, int nj, double fx,
                             double fy) {
    const int i = 1 + blockIdx.x * kTx + threadIdx.x;
    const int j = 1 + blockIdx.y * kTy + threadIdx.y;
    if (i > ni || j > nj) return;
    const double pc = p(i, j);
    u(i, j) = f(i, j) - (p(i + 1, j) - pc) * fx;
    v(i, j) = g(i, j) - (p(i, j + 1) - pc) * fy;
}

void launch_adapt_uv(const NsLaunch& L, const double* f, const double* g, const double* p,
                     double* u, double* v) {
    dim3 grid((L.ni + kTx - 1) / kTx, (L.nj + kTy - 1) / kTy);
    hipLaunchKernelGGL(adapt_kernel, grid, dim3(kTx, kTy), 0, L.s, CLay{f, L.pitch},
                       CLay{g, L.pitch}, CLay{p, L.pitch}, Lay{u, L.pitch}, Lay{v, L.pitch},
                       L.ni, L.nj, L.prm.dt / L.prm.dx, L.prm.dt / L.prm.dy);
}

// ---- reductions over the cells the reference visits (all (imax+2)(jmax+2),
// ghosts included).  On a decomposed grid a rank covers its interior plus the
// ghost rows/columns that lie on the physical boundary, so every global cell is
// visited exactly once.  Block partials, then one fixed-order finish.
constexpr int kRedBlocks = 1024;
constexpr int kRedThreads = 256;

int reduce_blocks(int ni, int nj) {
    const int cap = kRedBlocks;
    long long cells = (long long)(ni + 2) * (nj + 2);
    long long b = (cells + kRedThreads - 1) / kRedThreads;
    return (int)(b < cap ? (b < 1 ? 1 : b) : cap);
}

namespace {
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double w = __shfl_xor(v, o, 64);
        v = (v > w) ? v : w;
    }
    return v;
}
struct Region {
    int ilo, jlo, w, h;  // first cell and extent
};
__host__ Region region_of(const NsLaunch& L) {
    Region R;
    R.ilo = L.wall_left ? 0 : 1;
    R.jlo = L.wall_bottom ? 0 : 1;
    R.w = (L.wall_right ? L.ni + 1 : L.ni) - R.ilo + 1;
    R.h = (L.wall_top ? L.nj + 1 : L.nj) - R.jlo + 1;
    return R;
}
}  // namespace

// maxElement (:193-202) for u and v at once: max |x| seeded with DBL_MIN
__global__ __launch_bounds__(kRedThreads) void absmax2_kernel(CLay u, CLay v, Region R,
                                                              double* partials) {
    __shared__ double su[kRedThreads / 64], sv[kRedThreads / 64];
    double mu = 2.2250738585072014e-308, mv = 2.2250738585072014e-308;  // DBL_MIN
    // rows over blocks, columns over threads (coalesced; max is order-free)
    for (int jj = blockIdx.x; jj < R.h; jj += gridDim.x) {
        const int j = R.jlo + jj;
        for (int ii = threadIdx.x; ii < R.w; ii += kRedThreads) {
            const int i = R.ilo + ii;
            const double a = fabs(u(i, j)), b = fabs(v(i, j));
            mu = (mu > a) ? mu : a;
            mv = (mv > b) ? mv : b;
        }
    }
    mu = wmax(mu);
    mv = wmax(mv);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { su[w] = mu; sv[w] = mv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kRedThreads / 64; ++k) {
            mu = (mu > su[k]) ? mu : su[k];
            mv = (mv > sv[k]) ? mv : sv[k];
        }
        mu = (su[0] > mu) ? su[0] : mu;
        mv = (sv[0] > mv) ? sv[0] : mv;
        partials[2 * blockIdx.x] = mu;
        partials[2 * blockIdx.x + 1] = mv;
    }
}

void launch_absmax2(const NsLaunch& L, const double* u, const double* v, double* partials) {
    hipLaunchKernelGGL(absmax2_kernel, dim3(reduce_blocks(L.ni, L.nj)), dim3(kRedThreads), 0,
                       L.s, CLay{u, L.pitch}, CLay{v, L.pitch}, region_of(L), partials);
}

// adaptUV (:438-455) fused with the maxElement partials of the NEXT step's
// computeTimestep (:193-234): the reference's main loop changes no u, v
// between adaptUV and computeTimestep (main.c:43-60), so the maxima of the
// fields adaptUV leaves are the ones computeTimestep needs.  One pass over
// f, g, p -> u, v instead of that pass plus a 16-B/cell re-read of u, v
// (misor_api.hip misor_adapt_uv / misor_max_uv).
//
// Walk: tiles of 2 kRedThreads columns (two per lane: 16-byte loads and
// stores of the column pairs (odd, even), whose first column starts a
// 16-byte word in the padded layout) x kAR rows, row-major; a workgroup takes
// every gridDim-th tile, so the workgroups running at any time cover one
// compact stretch of rows.  Tiles inside [1, ni] x [1, nj] run without lane
// masks or branches; p(i+1) of a pair's first column is its second column,
// of the second one an 8-byte load (the same lines), p(j+1) the next row's
// p (one extra row per tile).  The cells of the reduction region outside the
// interior (the physical ghost cells) contribute their unchanged value in a
// separate walk; max is order-free and idempotent, so a cell counted twice
// changes nothing.  One partial per workgroup.

typedef double ad2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ ad2 ld2(const double* q) { return *reinterpret_cast<const ad2*>(q); }

template <int kAR, bool NT>
__global__ __launch_bounds__(kRedThreads) void adapt_absmax_kernel(CLay f, CLay g, CLay p, Lay u,
                                                                   Lay v, int ni, int nj,
                                                                   double fx, double fy, Region R,
                                                                   double* partials) {
    __shared__ double su[kRedThreads / 64], sv[kRedThreads / 64];
    double mu = 2.2250738585072014e-308, mv = 2.2250738585072014e-308;  // DBL_MIN
    constexpr int TW = 2 * kRedThreads;
    const int ntx = (ni + TW - 1) / TW, nty = (nj + kAR - 1) / kAR;
    const long long pitch = p.pitch;
    auto at = [&](int i, int j) { return (long long)(j + kYOff) * pitch + (i + kXOff); };
    for (int t = blockIdx.x; t < ntx * nty; t += gridDim.x) {
        const int tx = t % ntx, ty = t / ntx;
        const int ia = 1 + tx * TW + 2 * (int)threadIdx.x;
        const int j0 = 1 + ty * kAR;
        if ((tx + 1) * TW <= ni && j0 + kAR - 1 <= nj) {  // interior tile (workgroup-uniform)
            ad2 pc[kAR + 1], fv[kAR], gv[kAR];
            double pe[kAR];
#pragma unroll
            for (int q = 0; q < kAR; ++q) {
                const long long o = at(ia, j0 + q);
                fv[q] = ld2(f.a + o);
                gv[q] = ld2(g.a + o);
                pc[q] = ld2(p.a + o);
                pe[q] = p.a[o + 2];  // p(ib + 1, j)
            }
            pc[kAR] = ld2(p.a + at(ia, j0 + kAR));  // p(., j + 1) of the tile's last row
#pragma unroll
            for (int q = 0; q < kAR; ++q) {
                const long long o = at(ia, j0 + q);
                // :447-452, per column
                const double a0 = fv[q].x - (pc[q].y - pc[q].x) * fx;
                const double a1 = fv[q].y - (pe[q] - pc[q].y) * fx;
                const double b0 = gv[q].x - (pc[q + 1].x - pc[q].x) * fy;
                const double b1 = gv[q].y - (pc[q + 1].y - pc[q].y) * fy;
                put<NT>(reinterpret_cast<ad2*>(u.a + o), ad2{a0, a1});
                put<NT>(reinterpret_cast<ad2*>(v.a + o), ad2{b0, b1});
                mu = fmax(mu, fmax(fabs(a0), fabs(a1)));
                mv = fmax(mv, fmax(fabs(b0), fabs(b1)));
            }
        } else {  // a tile at the right / top end: per cell
            for (int q = 0; q < kAR; ++q) {
                const int j = j0 + q;
                if (j > nj) break;
                for (int c = 0; c < 2; ++c) {
                    const int i = ia + c;
                    if (i > ni) break;
                    const double pc0 = p(i, j);
                    const double a = f(i, j) - (p(i + 1, j) - pc0) * fx;
                    const double b = g(i, j) - (p(i, j + 1) - pc0) * fy;
                    u(i, j) = a;
                    v(i, j) = b;
                    mu = fmax(mu, fabs(a));
                    mv = fmax(mv, fabs(b));
                }
            }
        }
    }
    // the region's cells outside the interior: physical ghost columns and rows
    // (R covers [ilo, ilo + w) x [jlo, jlo + h); the interior is [1, ni] x [1, nj])
    {
        const int nl = R.ilo == 0 ? R.h : 0;                      // column 0
        const int nr = R.ilo + R.w - 1 == ni + 1 ? R.h : 0;      // column ni + 1
        const int nb = R.jlo == 0 ? R.w : 0;                      // row 0
        const int nt = R.jlo + R.h - 1 == nj + 1 ? R.w : 0;      // row nj + 1
        const int n = nl + nr + nb + nt;
        for (int k = blockIdx.x * kRedThreads + threadIdx.x; k < n; k += gridDim.x * kRedThreads) {
            int i, j;
            if (k < nl) {
                i = 0;
                j = R.jlo + k;
            } else if (k < nl + nr) {
                i = ni + 1;
                j = R.jlo + (k - nl);
            } else if (k < nl + nr + nb) {
                i = R.ilo + (k - nl - nr);
                j = 0;
            } else {
                i = R.ilo + (k - nl - nr - nb);
                j = nj + 1;
            }
            mu = fmax(mu, fabs(u(i, j)));
            mv = fmax(mv, fabs(v(i, j)));
        }
    }
    mu = wmax(mu);
    mv = wmax(mv);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { su[w] = mu; sv[w] = mv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kRedThreads / 64; ++k) {
            mu = (mu > su[k]) ? mu : su[k];
            mv = (mv > sv[k]) ? mv : sv[k];
        }
        mu = (su[0] > mu) ? su[0] : mu;
        mv = (sv[0] > mv) ? sv[0] : mv;
        partials[2 * blockIdx.x] = mu;
        partials[2 * blockIdx.x + 1] = mv;
    }
}

void launch_adapt_absmax(const NsLaunch& L, const double* f, const double* g, const double* p,
                         double* u, double* v, double* partials) {
    // rows per tile: 8 (16384^2: 2.06 ms against 2.12 for 4 and 2.14 for 2,
    // profiles/r03_ns_adapt_rows.txt)
    auto k = adapt_absmax_kernel<8, kNsNt>;
    hipLaunchKernelGGL(k, dim3(reduce_blocks(L.ni, L.nj)), dim3(kRedThreads), 0,
                       L.s, CLay{f, L.pitch}, CLay{g, L.pitch}, CLay{p, L.pitch},
                       Lay{u, L.pitch}, Lay{v, L.pitch}, L.ni, L.nj, L.prm.dt / L.prm.dx,
                       L.prm.dt / L.prm.dy, region_of(L), partials);
}

// ---- normalizePressure's sum (:208-212), exact: independent of the
// summation order, so of the block / rank decomposition.  Every cell
// x = m * 2^(ex-53) (|m| < 2^53 an integer) becomes the fixed-point integer
// trunc(x * 2^(kSumFrac - E)) with E the exponent of the largest |x| of the
// whole (global) field, so |term| < 2^(kSumFrac+1); terms and their sums are
// 128-bit integers, added exactly in any order.  The total is rounded to a
// double once, on the host (exact_sum_value).  The truncation of each term is
// a function of the cell alone: < 2^(E - kSumFrac) per cell, 2^17 times below
// the rounding of one double addition at the field's scale.
namespace {
struct U128 {
    unsigned long long lo, hi;
};
__device__ __forceinline__ U128 add128(U128 a, U128 b) {
    U128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1ull : 0ull);
    return r;
}
__device__ __forceinline__ U128 term128(double x, int E) {
    U128 r{0ull, 0ull};
    if (x == 0.0) return r;
    int ex;
    const double f = frexp(fabs(x), &ex);                     // |x| = f 2^ex, f in [0.5, 1)
    const unsigned long long m = (unsigned long long)ldexp(f, 53);  // exact
    const int sh = ex - 53 - E + kSumFrac;                    // <= kSumFrac - 53
    if (sh >= 0) {
        r.lo = m << sh;
        r.hi = sh == 0 ? 0ull : (m >> (64 - sh));
    } else if (sh > -64) {
        r.lo = m >> (-sh);
    }
    if (x < 0.0) {  // two's complement
        r.lo = ~r.lo;
        r.hi = ~r.hi;
        r = add128(r, U128{1ull, 0ull});
    }
    return r;
}
}  // namespace

__global__ __launch_bounds__(kRedThreads) void exact_sum_kernel(CLay p, Region R, int E,
                                                                unsigned long long* partials) {
    __shared__ U128 sh[kRedThreads];
    U128 s{0ull, 0ull};
    // rows over blocks, columns over threads (coalesced; the sum is exact)
    for (int jj = blockIdx.x; jj < R.h; jj += gridDim.x) {
        const int j = R.jlo + jj;
        for (int ii = threadIdx.x; ii < R.w; ii += kRedThreads)
            s = add128(s, term128(p(R.ilo + ii, j), E));
    }
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = kRedThreads / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] = add128(sh[threadIdx.x], sh[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = sh[0].lo;
        partials[2 * blockIdx.x + 1] = sh[0].hi;
    }
}

// the block sums added (one thread: exact, so any order), written as three
// limbs of 44 bits (the top one signed) as doubles: integers below 2^53, which
// a floating-point all-reduce over the ranks adds exactly
__global__ void exact_finish_kernel(const unsigned long long* partials, int n, double* limbs) {
    U128 s{0ull, 0ull};
    for (int k = 0; k < n; ++k) s = add128(s, U128{partials[2 * k], partials[2 * k + 1]});
    const unsigned long long m44 = (1ull << 44) - 1;
    limbs[0] = (double)(s.lo & m44);
    limbs[1] = (double)(((s.lo >> 44) | (s.hi << 20)) & m44);
    limbs[2] = (double)((long long)s.hi >> 24);  // bits 88..127, arithmetic shift
}

void launch_exact_sum(const NsLaunch& L, const double* p, int E, double* partials,
                      double* limbs) {
    const int nb = reduce_blocks(L.ni, L.nj);
    hipLaunchKernelGGL(exact_sum_kernel, dim3(nb), dim3(kRedThreads), 0, L.s, CLay{p, L.pitch},
                       region_of(L), E, reinterpret_cast<unsigned long long*>(partials));
    hipLaunchKernelGGL(exact_finish_kernel, dim3(1), dim3(1), 0, L.s,
                       reinterpret_cast<const unsigned long long*>(partials), nb, limbs);
}

double exact_sum_value(const double limbs[3], int E) {
    // V = l2 2^88 + l1 2^44 + l0, rounded to a double once (gcc's conversion of
    // a 128-bit integer rounds to nearest even), then scaled exactly
    const __int128 v = (__int128)(long long)limbs[2] * ((__int128)1 << 88) +
                       (__int128)(long long)limbs[1] * ((__int128)1 << 44) +
                       (__int128)(long long)limbs[0];
    return ldexp((double)v, E - kSumFrac);
}

// fixed-order combination of `n` partial records of `width` doubles
__global__ __launch_bounds__(256) void finish_reduce_kernel(const double* partials, int n,
                                                            int op, int width, double* out) {
    __shared__ double sh[2][256];
    const int t = threadIdx.x;
    for (int c = 0; c < width; ++c) {
        double acc = (op == kReduceSum) ? 0.0 : 2.2250738585072014e-308;
        for (int k = t; k < n; k += 256) {
            const double x = partials[(long long)k * width + c];
            acc = (op == kReduceSum) ? acc + x : ((acc > x) ? acc : x);
        }
        sh[c][t] = acc;
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (t < s) {
            for (int c = 0; c < width; ++c) {
                const double a = sh[c][t], b = sh[c][t + s];
                sh[c][t] = (op == kReduceSum) ? a + b : ((a > b) ? a : b);
            }
        }
        __syncthreads();
    }
    if (t < width) out[t] = sh[t][0];
}

void launch_finish_reduce(hipStream_t s, const double* partials, int n, int op, int width,
                          double* out) {
    hipLaunchKernelGGL(finish_reduce_kernel, dim3(1), dim3(256), 0, s, partials, n, op, width,
                       out);
}

// normalizePressure's second loop (:214-216): p -= avg over every cell
__global__ void sub_mean_kernel(Lay p, int ni, int nj, double avg) {
    const long long n = (long long)(ni + 2) * (nj + 2);
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const int i = (int)(k % (ni + 2)), j = (int)(k / (ni + 2));
        p(i, j) = p(i, j) - avg;
    }
}

void launch_sub_mean(const NsLaunch& L, double* p, double avg) {
    hipLaunchKernelGGL(sub_mean_kernel, dim3(reduce_blocks(L.ni, L.nj)), dim3(256), 0, L.s,
                       Lay{p, L.pitch}, L.ni, L.nj, avg);
}

}  // namespace misor
