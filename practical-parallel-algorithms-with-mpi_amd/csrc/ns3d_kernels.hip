// ns3d_kernels.hip -- assignment-6's 3D Navier-Stokes step and its red-black
// pressure solve (assignment-6/src/solver.c) for gfx950, single domain.
//
// Fields use the reference layout (imax+2)(jmax+2)(kmax+2), i fastest
// (solver.c:19-34); one thread per cell, consecutive threads on consecutive
// i (coalesced rows).  Every per-cell expression follows the reference term
// by term and the file is compiled with -ffp-contract=off, so each value is
// bit-identical to the reference's; only the order in which the residual is
// summed differs (fixed-order tree, deterministic).  These are 7-point / 19-
// point FP64 stencils: HBM-bound, no MFMA.

#include <cfloat>

#include "misor_internal.h"

namespace misor {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double w = __shfl_xor(v, o, 64);
        v = (v > w) ? v : w;
    }
    return v;
}

constexpr int kBx = 64, kBy = 4;  // 256-thread blocks: 64 along i, 4 along j

// ih*0.25*(ap*bp - am*bm) + gamma*ih*0.25*(|ap|*dp + |am|*dm): the donor-cell /
// gamma-upwind convective term of computeFG (solver.c:636-764)
__device__ __forceinline__ double conv(double ih, double gamma, double ap, double bp, double dp,
                                       double am, double bm, double dm) {
    return ih * 0.25 * (ap * bp - am * bm) + gamma * ih * 0.25 * (fabs(ap) * dp + fabs(am) * dm);
}

__device__ __forceinline__ double diff2(double ih, double ap, double c, double am) {
    return ih * ih * (ap - 2.0 * c + am);
}

// block-wide fixed-order sum of a 256-thread block (wave tree, then waves in order)
__device__ __forceinline__ double block_sum256(double v, double* sh) {
    const int t = threadIdx.y * kBx + threadIdx.x;
    v = wave_sum(v);
    if ((t & 63) == 0) sh[t >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (t == 0) s = ((sh[0] + sh[1]) + sh[2]) + sh[3];
    return s;
}

}  // namespace

// computeRHS, solver.c:145-173
__global__ __launch_bounds__(256) void k3_rhs(G3 g, const double* __restrict__ f,
                                              const double* __restrict__ gg,
                                              const double* __restrict__ h,
                                              double* __restrict__ rhs, double idx, double idy,
                                              double idz, double idt) {
    const int i = 1 + blockIdx.x * kBx + threadIdx.x;
    const int j = 1 + blockIdx.y * kBy + threadIdx.y;
    const int k = 1 + blockIdx.z;
    if (i > g.I || j > g.J) return;
    const long long c = g.ix(i, j, k);
    rhs[c] = ((f[c] - f[c - 1]) * idx + (gg[c] - gg[c - g.sx]) * idy +
              (h[c] - h[c - g.sxy]) * idz) *
             idt;
}

// one colour pass of solve (solver.c:203-231): pass 0 updates the cells with
// i+j+k odd, pass 1 the even ones; r^2 of the block into partials[block].
//
// The Neumann ghost copy that ends each iteration (solver.c:237-278: faces
// only, interior index ranges) is fused into the update: a face ghost is read
// only by the interior cell next to it, and that cell is updated in exactly
// one of the two passes and never again in the iteration, so the thread that
// updates it writes its mirror(s) right away -- the same values the separate
// copy would write, after the neighbour has read the old ghost.
__global__ __launch_bounds__(256) void k3_rb_pass(G3 g, double* __restrict__ p,
                                                  const double* __restrict__ rhs, int pass,
                                                  double idx2, double idy2, double idz2,
                                                  double factor, double* __restrict__ partials,
                                                  const DevState* __restrict__ st) {
    __shared__ double sh[4];
    if (st->done) return;
    const int j = 1 + blockIdx.y * kBy + threadIdx.y;
    const int k = 1 + blockIdx.z;
    const int i = 2 * (blockIdx.x * kBx + threadIdx.x) + (((1 + j + k + pass) & 1) ? 1 : 2);
    double acc = 0.0;
    if (i <= g.I && j <= g.J) {
        const long long q = g.ix(i, j, k);
        const double c = p[q];
        const double tx = (p[q + 1] - 2.0 * c) + p[q - 1];
        const double ty = (p[q + g.sx] - 2.0 * c) + p[q - g.sx];
        const double tz = (p[q + g.sxy] - 2.0 * c) + p[q - g.sxy];
        const double r = rhs[q] - ((tx * idx2 + ty * idy2) + tz * idz2);
        const double np = c - (factor * r);
        p[q] = np;
        acc = r * r;
        if (i == 1) p[q - 1] = np;
        if (i == g.I) p[q + 1] = np;
        if (j == 1) p[q - g.sx] = np;
        if (j == g.J) p[q + g.sx] = np;
        if (k == 1) p[q - g.sxy] = np;
        if (k == g.K) p[q + g.sxy] = np;
    }
    const double s = block_sum256(acc, sh);
    if (threadIdx.x == 0 && threadIdx.y == 0)
        partials[((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = s;
}

// end of one solve iteration: the reference never resets `res` (it is 1.0
// before the first iteration only, solver.c:196), so
//   res = (res + sum r^2 of pass 0 + sum r^2 of pass 1) / (imax*jmax*kmax)
// then it++ and the loop test (solver.c:199, 280-282, 291)
__global__ __launch_bounds__(1024) void k3_finish(const double* __restrict__ partials, int nb,
                                                  DevState* st, double cells) {
    __shared__ double sh[1024];
    __shared__ double tot[2];
    if (st->done) return;
    const int t = threadIdx.x;
    for (int ps = 0; ps < 2; ++ps) {
        double s = 0.0;
        for (int q = t; q < nb; q += 1024) s += partials[(long long)ps * nb + q];
        sh[t] = s;
        __syncthreads();
        for (int w = 512; w >= 64; w >>= 1) {
            if (t < w) sh[t] += sh[t + w];
            __syncthreads();
        }
        if (t < 64) {
            const double v = wave_sum(sh[t]);
            if (t == 0) tot[ps] = v;
        }
        __syncthreads();
    }
    if (t == 0) {
        const double res = ((st->res + tot[0]) + tot[1]) / cells;
        const int it = st->it + 1;
        st->res = res;
        st->it = it;
        st->done = !((res >= st->epssq) && (it < st->itermax));
    }
}

// computeFG, solver.c:606-772 (interior cells)
__global__ __launch_bounds__(256) void k3_fg(G3 g, const double* __restrict__ u,
                                             const double* __restrict__ v,
                                             const double* __restrict__ w, double* __restrict__ f,
                                             double* __restrict__ gg, double* __restrict__ h,
                                             Fg3 c) {
    const int i = 1 + blockIdx.x * kBx + threadIdx.x;
    const int j = 1 + blockIdx.y * kBy + threadIdx.y;
    const int k = 1 + blockIdx.z;
    if (i > g.I || j > g.J) return;
    const long long q = g.ix(i, j, k);
    const long long X = 1, Y = g.sx, Z = g.sxy;
    const double gm = c.gamma, ix = c.ix, iy = c.iy, iz = c.iz;
    const double Uc = u[q], Vc = v[q], Wc = w[q];

    const double du2dx = conv(ix, gm, Uc + u[q + X], Uc + u[q + X], Uc - u[q + X], Uc + u[q - X],
                              Uc + u[q - X], Uc - u[q - X]);
    const double duvdy = conv(iy, gm, Vc + v[q + X], Uc + u[q + Y], Uc - u[q + Y],
                              v[q - Y] + v[q + X - Y], Uc + u[q - Y], Uc - u[q - Y]);
    const double duwdz = conv(iz, gm, Wc + w[q + X], Uc + u[q + Z], Uc - u[q + Z],
                              w[q - Z] + w[q + X - Z], Uc + u[q - Z], Uc - u[q - Z]);
    const double lu = diff2(ix, u[q + X], Uc, u[q - X]) + diff2(iy, u[q + Y], Uc, u[q - Y]) +
                      diff2(iz, u[q + Z], Uc, u[q - Z]);
    f[q] = Uc + c.dt * (c.iRe * lu - du2dx - duvdy - duwdz + c.gx);

    const double duvdx = conv(ix, gm, Uc + u[q + Y], Vc + v[q + X], Vc - v[q + X],
                              u[q - X] + u[q - X + Y], Vc + v[q - X], Vc - v[q - X]);
    const double dv2dy = conv(iy, gm, Vc + v[q + Y], Vc + v[q + Y], Vc - v[q + Y], Vc + v[q - Y],
                              Vc + v[q - Y], Vc - v[q - Y]);
    // as the reference (solver.c:719-727): the - side reuses V(i,j,k+1)
    const double dvwdz = conv(iz, gm, Wc + w[q + Y], Vc + v[q + Z], Vc - v[q + Z],
                              w[q - Z] + w[q + Y - Z], Vc + v[q + Z], Vc - v[q + Z]);
    const double lv = diff2(ix, v[q + X], Vc, v[q - X]) + diff2(iy, v[q + Y], Vc, v[q - Y]) +
                      diff2(iz, v[q + Z], Vc, v[q - Z]);
    gg[q] = Vc + c.dt * (c.iRe * lv - duvdx - dv2dy - dvwdz + c.gy);

    const double duwdx = conv(ix, gm, Uc + u[q + Z], Wc + w[q + X], Wc - w[q + X],
                              u[q - X] + u[q - X + Z], Wc + w[q - X], Wc - w[q - X]);
    const double dvwdy = conv(iy, gm, Vc + v[q + Z], Wc + w[q + Y], Wc - w[q + Y],
                              v[q - Y + Z] + v[q - Y], Wc + w[q - Y], Wc - w[q - Y]);
    const double dw2dz = conv(iz, gm, Wc + w[q + Z], Wc + w[q + Z], Wc - w[q + Z], Wc + w[q - Z],
                              Wc + w[q - Z], Wc - w[q - Z]);
    const double lw = diff2(ix, w[q + X], Wc, w[q - X]) + diff2(iy, w[q + Y], Wc, w[q - Y]) +
                      diff2(iz, w[q + Z], Wc, w[q - Z]);
    h[q] = Wc + c.dt * (c.iRe * lw - duwdx - dvwdy - dw2dz + c.gz);
}

// boundary values of F, G, H (solver.c:774-823), after k3_fg: z = 0 the
// x walls (j, k), z = 1 the y walls (i, k), z = 2 the z walls (i, j)
__global__ void k3_fg_boundary(G3 g, const double* __restrict__ u, const double* __restrict__ v,
                               const double* __restrict__ w, double* __restrict__ f,
                               double* __restrict__ gg, double* __restrict__ h) {
    const int a = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    const int b = 1 + blockIdx.y;
    if (blockIdx.z == 0) {
        if (a > g.J || b > g.K) return;
        f[g.ix(0, a, b)] = u[g.ix(0, a, b)];
        f[g.ix(g.I, a, b)] = u[g.ix(g.I, a, b)];
    } else if (blockIdx.z == 1) {
        if (a > g.I || b > g.K) return;
        gg[g.ix(a, 0, b)] = v[g.ix(a, 0, b)];
        gg[g.ix(a, g.J, b)] = v[g.ix(a, g.J, b)];
    } else {
        if (a > g.I || b > g.J) return;
        h[g.ix(a, b, 0)] = w[g.ix(a, b, 0)];
        h[g.ix(a, b, g.K)] = w[g.ix(a, b, g.K)];
    }
}

// adaptUV, solver.c:826-853
__global__ __launch_bounds__(256) void k3_adapt(G3 g, const double* __restrict__ f,
                                                const double* __restrict__ gg,
                                                const double* __restrict__ h,
                                                const double* __restrict__ p, double* __restrict__ u,
                                                double* __restrict__ v, double* __restrict__ w,
                                                double fx, double fy, double fz) {
    const int i = 1 + blockIdx.x * kBx + threadIdx.x;
    const int j = 1 + blockIdx.y * kBy + threadIdx.y;
    const int k = 1 + blockIdx.z;
    if (i > g.I || j > g.J) return;
    const long long q = g.ix(i, j, k);
    const double pc = p[q];
    u[q] = f[q] - (p[q + 1] - pc) * fx;
    v[q] = gg[q] - (p[q + g.sx] - pc) * fy;
    w[q] = h[q] - (p[q + g.sxy] - pc) * fz;
}

// one wall of setBoundaryConditions (solver.c:364-577).  n: the velocity
// normal to the wall, set ON the wall (layer `on`); t1, t2: the tangential
// ones in the ghost layer `gh`, from the first interior layer `in`.
__global__ void k3_wall(G3 g, double* __restrict__ n, double* __restrict__ t1,
                        double* __restrict__ t2, int axis, int gh, int in, int on, int onin,
                        int bc) {
    const int a = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    const int b = 1 + blockIdx.y;
    const int na = axis == 0 ? g.J : g.I;
    const int nb = axis == 2 ? g.J : g.K;
    if (a > na || b > nb) return;
    long long G, I, O, OI;
    if (axis == 0) {
        G = g.ix(gh, a, b); I = g.ix(in, a, b); O = g.ix(on, a, b); OI = g.ix(onin, a, b);
    } else if (axis == 1) {
        G = g.ix(a, gh, b); I = g.ix(a, in, b); O = g.ix(a, on, b); OI = g.ix(a, onin, b);
    } else {
        G = g.ix(a, b, gh); I = g.ix(a, b, in); O = g.ix(a, b, on); OI = g.ix(a, b, onin);
    }
    switch (bc) {
    case MISOR_NOSLIP: n[O] = 0.0; t1[G] = -t1[I]; t2[G] = -t2[I]; break;
    case MISOR_SLIP: n[O] = 0.0; t1[G] = t1[I]; t2[G] = t2[I]; break;
    case MISOR_OUTFLOW: n[O] = n[OI]; t1[G] = t1[I]; t2[G] = t2[I]; break;
    default: break;  // PERIODIC: nothing (as the reference)
    }
}

// setSpecialBoundaryCondition, solver.c:579-604
__global__ void k3_special(G3 g, double* __restrict__ u, int problem) {
    const int a = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    const int b = 1 + blockIdx.y;
    if (problem == MISOR_PROBLEM_DCAVITY) {  // i = 1..imax-1, k = 1..kmax-1
        if (a < g.I && b < g.K) u[g.ix(a, g.J + 1, b)] = 2.0 - u[g.ix(a, g.J, b)];
    } else if (problem == MISOR_PROBLEM_CANAL) {  // U(0,j,k) = 2.0
        if (a <= g.J && b <= g.K) u[g.ix(0, a, b)] = 2.0;
    }
}

// maxElement (solver.c:299-310) of u, v, w over every cell incl. ghosts:
// per-block maxima (order-free: exact)
__global__ __launch_bounds__(256) void k3_absmax3(const double* __restrict__ u,
                                                  const double* __restrict__ v,
                                                  const double* __restrict__ w, long long n,
                                                  double* __restrict__ partials) {
    __shared__ double sh[3][4];
    double mu = DBL_MIN, mv = DBL_MIN, mw = DBL_MIN;  // seeds of maxElement
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n; q += stride) {
        const double a = fabs(u[q]), b = fabs(v[q]), c = fabs(w[q]);
        mu = (mu > a) ? mu : a;
        mv = (mv > b) ? mv : b;
        mw = (mw > c) ? mw : c;
    }
    mu = wave_max(mu);
    mv = wave_max(mv);
    mw = wave_max(mw);
    const int t = threadIdx.x;
    if ((t & 63) == 0) {
        sh[0][t >> 6] = mu;
        sh[1][t >> 6] = mv;
        sh[2][t >> 6] = mw;
    }
    __syncthreads();
    if (t < 3) {
        double m = sh[t][0];
        for (int x = 1; x < 4; ++x) m = (m > sh[t][x]) ? m : sh[t][x];
        partials[3 * blockIdx.x + t] = m;
    }
}

__global__ __launch_bounds__(256) void k3_max_finish(const double* __restrict__ partials, int nb,
                                                     double* out) {
    __shared__ double sh[3][4];
    const int t = threadIdx.x;
    double m[3] = {DBL_MIN, DBL_MIN, DBL_MIN};
    for (int q = t; q < nb; q += 256)
        for (int c = 0; c < 3; ++c) m[c] = (m[c] > partials[3 * q + c]) ? m[c] : partials[3 * q + c];
    for (int c = 0; c < 3; ++c) {
        m[c] = wave_max(m[c]);
        if ((t & 63) == 0) sh[c][t >> 6] = m[c];
    }
    __syncthreads();
    if (t < 3) {
        double v = sh[t][0];
        for (int x = 1; x < 4; ++x) v = (v > sh[t][x]) ? v : sh[t][x];
        out[t] = v;
    }
}

// normalizePressure (solver.c:312-338): interior sum (fixed order), then subtract
__global__ __launch_bounds__(256) void k3_sum_interior(G3 g, const double* __restrict__ p,
                                                       double* __restrict__ partials) {
    __shared__ double sh[4];
    const int i = 1 + blockIdx.x * kBx + threadIdx.x;
    const int j = 1 + blockIdx.y * kBy + threadIdx.y;
    const int k = 1 + blockIdx.z;
    const double v = (i <= g.I && j <= g.J) ? p[g.ix(i, j, k)] : 0.0;
    const double s = block_sum256(v, sh);
    if (threadIdx.x == 0 && threadIdx.y == 0)
        partials[((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void k3_sum_finish(const double* __restrict__ partials, int nb,
                                                      double* out) {
    __shared__ double sh[1024];
    const int t = threadIdx.x;
    double s = 0.0;
    for (int q = t; q < nb; q += 1024) s += partials[q];
    sh[t] = s;
    __syncthreads();
    for (int w = 512; w >= 64; w >>= 1) {
        if (t < w) sh[t] += sh[t + w];
        __syncthreads();
    }
    if (t < 64) {
        const double v = wave_sum(sh[t]);
        if (t == 0) out[0] = v;
    }
}

__global__ __launch_bounds__(256) void k3_sub_mean(G3 g, double* __restrict__ p,
                                                   const double* __restrict__ sum, double cells) {
    const int i = 1 + blockIdx.x * kBx + threadIdx.x;
    const int j = 1 + blockIdx.y * kBy + threadIdx.y;
    const int k = 1 + blockIdx.z;
    if (i > g.I || j > g.J) return;
    const double avg = sum[0] / cells;
    const long long q = g.ix(i, j, k);
    p[q] = p[q] - avg;
}

// ---------------------------------------------------------------- launchers
static dim3 cells_grid(const G3& g, int nx) {
    return dim3((unsigned)((nx + kBx - 1) / kBx), (unsigned)((g.J + kBy - 1) / kBy),
                (unsigned)g.K);
}

int ns3_partials(const G3& g) {
    const dim3 a = cells_grid(g, (g.I + 1) / 2);
    const dim3 b = cells_grid(g, g.I);
    const long long na = (long long)a.x * a.y * a.z, nb = (long long)b.x * b.y * b.z;
    return (int)(na > nb ? na : nb);
}

void launch3_rhs(hipStream_t s, const G3& g, const double* f, const double* gg, const double* h,
                 double* rhs, double idx, double idy, double idz, double idt) {
    hipLaunchKernelGGL(k3_rhs, cells_grid(g, g.I), dim3(kBx, kBy), 0, s, g, f, gg, h, rhs, idx,
                       idy, idz, idt);
}

int launch3_rb_iteration(hipStream_t s, const G3& g, double* p, const double* rhs, double idx2,
                         double idy2, double idz2, double factor, double* partials, DevState* st,
                         double cells) {
    const dim3 grid = cells_grid(g, (g.I + 1) / 2);
    const int nb = (int)(grid.x * grid.y * grid.z);
    for (int pass = 0; pass < 2; ++pass)
        hipLaunchKernelGGL(k3_rb_pass, grid, dim3(kBx, kBy), 0, s, g, p, rhs, pass, idx2, idy2,
                           idz2, factor, partials + (long long)pass * nb, st);
    hipLaunchKernelGGL(k3_finish, dim3(1), dim3(1024), 0, s, partials, nb, st, cells);
    return nb;
}

void launch3_fg(hipStream_t s, const G3& g, const double* u, const double* v, const double* w,
                double* f, double* gg, double* h, const Fg3& c) {
    hipLaunchKernelGGL(k3_fg, cells_grid(g, g.I), dim3(kBx, kBy), 0, s, g, u, v, w, f, gg, h, c);
    const int mx = g.I > g.J ? g.I : g.J;
    const int my = g.J > g.K ? g.J : g.K;
    hipLaunchKernelGGL(k3_fg_boundary, dim3((unsigned)((mx + 127) / 128), (unsigned)my, 3),
                       dim3(128), 0, s, g, u, v, w, f, gg, h);
}

void launch3_adapt(hipStream_t s, const G3& g, const double* f, const double* gg,
                   const double* h, const double* p, double* u, double* v, double* w, double fx,
                   double fy, double fz) {
    hipLaunchKernelGGL(k3_adapt, cells_grid(g, g.I), dim3(kBx, kBy), 0, s, g, f, gg, h, p, u, v,
                       w, fx, fy, fz);
}

void launch3_wall(hipStream_t s, const G3& g, double* n, double* t1, double* t2, int axis,
                  int gh, int in, int on, int onin, int bc) {
    const int na = axis == 0 ? g.J : g.I;
    const int nb = axis == 2 ? g.J : g.K;
    hipLaunchKernelGGL(k3_wall, dim3((unsigned)((na + 127) / 128), (unsigned)nb), dim3(128), 0,
                       s, g, n, t1, t2, axis, gh, in, on, onin, bc);
}

void launch3_special(hipStream_t s, const G3& g, double* u, int problem) {
    const int na = g.I > g.J ? g.I : g.J;
    hipLaunchKernelGGL(k3_special, dim3((unsigned)((na + 127) / 128), (unsigned)g.K), dim3(128),
                       0, s, g, u, problem);
}

int absmax3_blocks() { return 1024; }

void launch3_absmax(hipStream_t s, const double* u, const double* v, const double* w,
                    long long n, double* partials, double* out) {
    hipLaunchKernelGGL(k3_absmax3, dim3(absmax3_blocks()), dim3(256), 0, s, u, v, w, n,
                       partials);
    hipLaunchKernelGGL(k3_max_finish, dim3(1), dim3(256), 0, s, partials, absmax3_blocks(), out);
}

void launch3_normalize(hipStream_t s, const G3& g, double* p, double* partials, double* sum,
                       double cells) {
    const dim3 grid = cells_grid(g, g.I);
    hipLaunchKernelGGL(k3_sum_interior, grid, dim3(kBx, kBy), 0, s, g, p, partials);
    hipLaunchKernelGGL(k3_sum_finish, dim3(1), dim3(1024), 0, s, partials,
                       (int)(grid.x * grid.y * grid.z), sum);
    hipLaunchKernelGGL(k3_sub_mean, grid, dim3(kBx, kBy), 0, s, g, p, sum, cells);
}

}  // namespace misor
