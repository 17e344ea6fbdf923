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
//   res = (res + sum r^2 of pass 0 [+ sum r^2 of pass 1]) / (imax*jmax*kmax)
// then it++ and the loop test (solver.c:199, 280-282, 291).  npass = 2 for
// the two colour-pass form, 1 for the fused sweep (one partial per block).
__global__ __launch_bounds__(1024) void k3_finish(const double* __restrict__ partials, int nb,
                                                  int npass, DevState* st, double cells,
                                                  int sum_only) {
    __shared__ double sh[1024];
    __shared__ double tot[2];
    if (st->done) return;
    const int t = threadIdx.x;
    for (int ps = 0; ps < npass; ++ps) {
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
    if (t == 0 && sum_only) st->sum[0] = tot[0];  // decomposed: all-reduce, then decide
    if (t == 0 && !sum_only) {
        double res = st->res + tot[0];
        if (npass > 1) res = res + tot[1];
        res = res / cells;
        const int it = st->it + 1;
        st->res = res;
        st->it = it;
        st->done = !((res >= st->epssq) && (it < st->itermax));
    }
}

// decomposed solve: res = (res + all-reduced sum r^2) / (imax*jmax*kmax)
__global__ void k3_decide(DevState* st, double cells) {
    if (threadIdx.x != 0 || st->done) return;
    const double res = (st->res + st->sum[0]) / cells;
    const int it = st->it + 1;
    st->res = res;
    st->it = it;
    st->done = !((res >= st->epssq) && (it < st->itermax));
}

// Folded loop test (single rank).  Instead of a k3_finish launch after every
// sweep, sweep launch b of a batch first completes the loop test of sweep
// b-1 from its per-workgroup partials -- every workgroup redundantly, in
// k3_finish's exact order (1024 strided sums, then the same tree), so all
// agree bit for bit -- and returns at once if the loop is over.  The state is
// double-buffered (launch b reads in, workgroup 0 writes out; the next launch
// swaps them) so no workgroup reads a state another one of the same launch is
// writing.  k3_fold_decide applies the last test of a batch.  One launch per
// iteration instead of two.
struct Fold3 {
    const double* prev;   // partials of the previous sweep (nullptr: no test, copy the state)
    int prev_nb;
    const DevState* in;
    DevState* out;
    double cells;
};

// the loop test of one sweep; scratch: 1025 doubles of LDS; every thread of
// the (256-thread) workgroup returns the new state's done flag.  The state is
// handled field by field (a whole-struct copy lands in scratch memory).
__device__ __forceinline__ int fold_test(const Fold3& F, double* scratch) {
    const int t = threadIdx.y * blockDim.x + threadIdx.x;
    int it = F.in->it, done = F.in->done;
    double res = F.in->res;
    if (!done && F.prev) {
        // k3_finish's order with 1024 virtual threads v = t + 256 m
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int vt = t + 256 * m;
            double x = 0.0;
            for (int q = vt; q < F.prev_nb; q += 1024) x += F.prev[q];
            scratch[vt] = x;
        }
        __syncthreads();
        scratch[t] += scratch[t + 512];  // w = 512: virtual threads t and t + 256
        scratch[t + 256] += scratch[t + 768];
        __syncthreads();
        for (int w = 256; w >= 64; w >>= 1) {
            if (t < w) scratch[t] += scratch[t + w];
            __syncthreads();
        }
        if (t < 64) {
            const double v = wave_sum(scratch[t]);
            if (t == 0) scratch[1024] = v;
        }
        __syncthreads();
        res = (res + scratch[1024]) / F.cells;
        it = it + 1;
        done = !((res >= F.in->epssq) && (it < F.in->itermax));
    }
    if (blockIdx.x == 0 && t == 0) {
        F.out->it = it;
        F.out->done = done;
        F.out->res = res;
        F.out->itermax = F.in->itermax;
        F.out->epssq = F.in->epssq;
    }
    return done;
}

__global__ __launch_bounds__(256) void k3_fold_decide(Fold3 F) {
    __shared__ double scratch[1025];
    (void)fold_test(F, scratch);
}

// ------------------------------------------------- fused red-black sweep
// One launch = one whole solve iteration (red of every cell, then black),
// read from `src`, written to `dst` (ping-pong: blocks never see another
// block's new values).  A workgroup owns a tile of kSwOwn columns x R rows and
// a chunk of planes, and marches up k: at step k it updates the red cells of
// plane k and then the black cells of plane k-1, whose red neighbours
// (planes k-2, k-1, k) are all new by then -- exactly the values the
// reference's two passes use.
//
// * Planes live in an LDS ring of 5 slots of (R+4) x 128 doubles: the tile
//   plus a 2-cell ring, on which red is computed redundantly (black on the
//   tile's edge needs red one cell outside).  Within a row the columns are
//   stored split by parity (even columns, then odd ones), so the cells of one
//   colour -- and each of their x-neighbours -- are 64 consecutive doubles:
//   every LDS access of a wave is contiguous.
// * Loads: lane l reads the column pair (2l, 2l+1) of a row with one 16-byte
//   load (the fields carry one spare double at each end of the allocation,
//   so the pair of the first strip's column -1 stays inside it).  p rows go
//   to LDS, split by parity.  rhs rows are read once for both colours: the
//   pair of row t of plane k arrives during step k-1; step k uses its red
//   element and keeps the black one for step k+1.  Red and black cells of a
//   row are handled by the same lane, so nothing is exchanged.
// * Software pipeline: step k issues the loads of plane k+3 and the rhs pairs
//   of plane k+1, and writes plane k+2 (issued one step earlier) to LDS at its
//   end; the k loop is unrolled by two so the register sets alternate with
//   compile-time indices.  Loads are unconditional (addresses clamped into the
//   array), so the compiler waits for each with a counted vmcnt.
// * Everything per-thread that does not change along k (LDS positions,
//   in-plane offsets, validity and boundary flags, for the two parities of k)
//   is computed once; a step adds scalar plane offsets.
// * Finished planes go from LDS to dst in whole rows (one write per 128-B
//   line) with the Neumann face mirrors of k3_rb_pass.  Per-cell arithmetic
//   is the reference's, term by term; the residual of the owned cells is
//   summed per workgroup in a fixed order.
constexpr int kSwCols = 128;           // loaded columns per strip
constexpr int kSwOwn = kSwCols - 4;    // owned columns per strip
constexpr int kSwSlots = 5;
constexpr int kSwOdd = 80;             // LDS position of odd column 1 in a row: the odd half
                                       // starts 32 banks after the even half
constexpr int kSwRow = kSwOdd + 64;    // doubles per LDS row

namespace {
struct SwCell {
    int lds;    // row offset + position of the cell in the split row
    int nb;     // row offset + position of its left x-neighbour (right = nb + 1)
    int sel;    // which element of the lane's column pair the cell is (0 / 1)
    int flags;  // 1 red valid, 2 red owned, 4 black valid (owned)
};

// the red cell (i+j+k odd) of LDS row t for planes of parity q, and whether
// this lane's black cell of the same row is owned
__device__ __forceinline__ SwCell sw_cell(const G3& g, int c_ld, int j_ld, int t, int lane, int q,
                                          int R) {
    const int j = j_ld + t;
    const int sel = ((c_ld + j + q) & 1) ^ 1;  // LDS column parity of the red cell
    const int x = 2 * lane + sel, i = c_ld + x;
    const int xb = 2 * lane + (sel ^ 1), ib = c_ld + xb;  // the black cell of the pair
    SwCell c;
    c.lds = t * kSwRow + sel * kSwOdd + lane;
    c.nb = t * kSwRow + (1 - sel) * kSwOdd + lane + sel - 1;
    c.sel = sel;
    const bool row_in = j >= 1 && j <= g.J && t <= R + 2;
    const bool red_valid = row_in && i >= 1 && i <= g.I && x >= 1 && x <= kSwCols - 2;
    const bool red_owned = red_valid && t >= 2 && t <= R + 1 && x >= 2 && x <= kSwCols - 3;
    const bool blk_owned = row_in && t >= 2 && t <= R + 1 && ib >= 1 && ib <= g.I && xb >= 2 &&
                           xb <= kSwCols - 3;
    c.flags = (red_valid ? 1 : 0) | (red_owned ? 2 : 0) | (blk_owned ? 4 : 0);
    return c;
}

struct alignas(8) D2 {
    double v[2];
};
}  // namespace

template <int R, bool RA2 = false>
__global__ __launch_bounds__(256) void k3_sweep(G3 g, const double* __restrict__ src,
                                                double* __restrict__ dst,
                                                const double* __restrict__ rhs, double idx2,
                                                double idy2, double idz2, double factor,
                                                int nstrips, int nrowb, int kc,
                                                double* __restrict__ partials,
                                                const DevState* __restrict__ st, Fold3 F) {
    constexpr int NR = R + 4;  // rows per plane in LDS
    static_assert(R % 4 == 0, "R must be a multiple of 4");
    constexpr int LR = NR / 4;           // rows each wave loads
    constexpr int RR = (R + 2 + 3) / 4;  // update rows per wave (LDS rows 1..R+2)
    constexpr int PL = NR * kSwRow;      // doubles per LDS plane
    static_assert(kSwSlots * PL >= 1025, "the folded loop test uses the plane ring as scratch");
    __shared__ double L[kSwSlots * PL];
    __shared__ double sh[4];
    if (!F.in && st->done) return;

    // XCD-aware order: the hardware deals workgroups round-robin to the 8 XCDs
    // (each with its own L2); give XCD x a contiguous run of tiles so that
    // neighbouring tiles -- which re-read each other's halo rows -- share an L2
    int b;
    {
        const int nb = (int)gridDim.x, x = (int)blockIdx.x % 8, q = nb / 8, rem = nb % 8;
        b = x * q + min(x, rem) + (int)blockIdx.x / 8;
    }
    const int strip = b % nstrips;
    b /= nstrips;
    const int rb = b % nrowb;
    const int kb = b / nrowb;
    const int c_ld = strip * kSwOwn - 1;  // global column of LDS column 0
    const int j_ld = rb * R - 1;          // global row of LDS row 0 (owned rows j_ld+2 ..)
    const int k0 = 1 + kb * kc;           // owned planes k0 .. kend
    const int kend = min(g.K, k0 + kc - 1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long sxy = g.sxy;
    const int sx = (int)g.sx;
    // the pair of lane l starts at column c_ld + 2l: >= -1 and, clamped, <=
    // I+1, so it reaches at most one double before / after a row -- inside the
    // allocation, which has a spare double at each end; lanes past the last
    // column re-read the last pair (their LDS columns are never used)
    const int pc = min(c_ld + 2 * lane, g.I + 1);

    // p loads: in-plane offsets (rows clamped) and LDS positions (parity split)
    int lo[LR], ls[LR];
#pragma unroll
    for (int m = 0; m < LR; ++m) {
        const int t = w + 4 * m;
        lo[m] = min(max(j_ld + t, 0), g.J + 1) * sx + pc;
        ls[m] = t * kSwRow + lane;  // even column 2l at lane, odd 2l+1 at kSwOdd + lane
    }
    // update rows t = 1 + w + 4m: rhs pair offsets and the cells for the two
    // parities of k (A = parity of the first step, k0-1)
    const int qa = (k0 - 1 + g.koff) & 1;  // colours are global: i + j + (koff + k)
    int ro[RR];
    SwCell cA[RR], cB[RR];
#pragma unroll
    for (int m = 0; m < RR; ++m) {
        const int t = 1 + w + 4 * m;
        ro[m] = min(max(j_ld + t, 0), g.J + 1) * sx + pc;
        cA[m] = sw_cell(g, c_ld, j_ld, t, lane, qa, R);
        cB[m] = sw_cell(g, c_ld, j_ld, t, lane, qa ^ 1, R);
    }

    auto slot = [](int kk) { return (kk + kSwSlots) % kSwSlots; };
    // planes -1 .. K+2 exist in memory (2-deep halo storage)
    auto plane = [&](int kk) { return (long long)min(max(kk, -1), g.K + 2) * sxy; };
    // red is computed on halo planes too where a neighbour rank owns them
    const int kr_lo = g.lo_phys ? 1 : 0, kr_hi = g.hi_phys ? g.K : g.K + 1;
    auto load_plane = [&](int kk, D2 (&v)[LR]) {
        const double* sp = src + plane(kk);
#pragma unroll
        for (int m = 0; m < LR; ++m) v[m] = *reinterpret_cast<const D2*>(sp + lo[m]);
    };
    auto store_plane = [&](int kk, const D2 (&v)[LR]) {
        double* Ls = L + slot(kk) * PL;
#pragma unroll
        for (int m = 0; m < LR; ++m) {
            Ls[ls[m]] = v[m].v[0];
            Ls[ls[m] + kSwOdd] = v[m].v[1];
        }
    };
    auto load_rhs = [&](int kk, D2 (&v)[RR]) {
        const double* rp = rhs + plane(kk);
#pragma unroll
        for (int m = 0; m < RR; ++m) v[m] = *reinterpret_cast<const D2*>(rp + ro[m]);
    };
    // owned cells of a finished plane (both colours) from LDS to dst in whole
    // rows -- full 128-B lines, one write per line -- with the Neumann face
    // mirrors of the boundary cells (solver.c:237-278)
    constexpr int BR = R / 4;
    int so[BR][2], sl[BR][2], sf[BR][2];
#pragma unroll
    for (int m = 0; m < BR; ++m) {
        const int t = 2 + w + 4 * m, j = j_ld + t;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int x = lane + 64 * h, i = c_ld + x;
            const bool own = x >= 2 && x <= kSwCols - 3 && i >= 1 && i <= g.I && j >= 1 &&
                             j <= g.J;
            so[m][h] = own ? j * sx + i : 0;
            sl[m][h] = t * kSwRow + (x & 1) * kSwOdd + (x >> 1);
            sf[m][h] = own ? (1 | (i == 1 ? 4 : 0) | (i == g.I ? 8 : 0) | (j == 1 ? 16 : 0) |
                              (j == g.J ? 32 : 0))
                           : 0;
        }
    }
    auto store_final = [&](int kk) {
        const double* Ls = L + slot(kk) * PL;
        double* dk = dst + (long long)kk * sxy;
#pragma unroll
        for (int m = 0; m < BR; ++m)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int f = sf[m][h];
                if (f & 1) {
                    const double v = Ls[sl[m][h]];
                    const int o = so[m][h];
                    dk[o] = v;
                    if (f & 4) dk[o - 1] = v;
                    if (f & 8) dk[o + 1] = v;
                    if (f & 16) dk[o - sx] = v;
                    if (f & 32) dk[o + sx] = v;
                    if (kk == 1 && g.lo_phys) dk[o - sxy] = v;
                    if (kk == g.K && g.hi_phys) dk[o + sxy] = v;
                }
            }
    };
    double acc = 0.0;
    // one update: the reference's arithmetic on LDS neighbours; returns the new value
    auto update = [&](const double* Lc, const double* Lm, const double* Lp, int o, int nbo,
                      double rh, double& r) {
        const double cc = Lc[o];
        const double tx = (Lc[nbo + 1] - 2.0 * cc) + Lc[nbo];
        const double ty = (Lc[o + kSwRow] - 2.0 * cc) + Lc[o - kSwRow];
        const double tz = (Lp[o] - 2.0 * cc) + Lm[o];
        r = rh - ((tx * idx2 + ty * idy2) + tz * idz2);
        return cc - (factor * r);
    };
    // step k: red of plane k (cells c: parity of k), black of plane k-1 (the
    // same lanes' other pair element, cells cp: parity of k-1)
    auto step = [&](const int k, D2 (&pl_in)[LR], const D2 (&pl_out)[LR], const SwCell (&c)[RR],
                    const SwCell (&cp)[RR], const D2 (&rk)[RR], const D2 (&rkm)[RR],
                    D2 (&rk_n)[RR]) {
        load_plane(k + 3, pl_in);
        load_rhs(k + (RA2 ? 2 : 1), rk_n);
        __syncthreads();  // plane k+1 in LDS, plane k-2 final; the slot reused below is free
        if (k - 2 >= k0 && k - 2 <= kend) store_final(k - 2);
        if (k >= kr_lo && k <= kr_hi) {
            double* Lc = L + slot(k) * PL;
            const double* Lm = L + slot(k - 1) * PL;
            const double* Lp = L + slot(k + 1) * PL;
            const bool own_k = k >= k0 && k <= kend;
#pragma unroll
            for (int m = 0; m < RR; ++m) {
                if (c[m].flags & 1) {
                    double r;
                    const double rh = c[m].sel ? rk[m].v[1] : rk[m].v[0];
                    const double np = update(Lc, Lm, Lp, c[m].lds, c[m].nb, rh, r);
                    Lc[c[m].lds] = np;
                    if (own_k && (c[m].flags & 2)) acc += r * r;
                }
            }
        }
        __syncthreads();  // red of plane k visible
        if (k - 1 >= k0 && k - 1 <= kend) {
            const int kb1 = k - 1;
            double* Lc = L + slot(kb1) * PL;
            const double* Lm = L + slot(kb1 - 1) * PL;
            const double* Lp = L + slot(k) * PL;
#pragma unroll
            for (int m = 0; m < RR; ++m) {
                if (cp[m].flags & 4) {
                    // the black cell is the pair element the red cell of plane k-1 is not
                    const int sb = cp[m].sel ^ 1;
                    const int o = cp[m].lds + (sb - cp[m].sel) * kSwOdd;
                    const int nbo = cp[m].nb + (cp[m].sel - sb) * kSwOdd + (sb - cp[m].sel);
                    const double rh = sb ? rkm[m].v[1] : rkm[m].v[0];
                    double r;
                    const double np = update(Lc, Lm, Lp, o, nbo, rh, r);
                    Lc[o] = np;
                    acc += r * r;
                }
            }
        }
        store_plane(k + 2, pl_out);
    };

    // preload planes k0-2 .. k0 (into LDS) and k0+1 (registers) and the first
    // rhs pairs: all loads issued together, so the march starts after one
    // memory latency instead of three
    D2 v0[LR], v1[LR], v2[LR];
    // (loads one step ahead of use; a variant with p three and rhs two steps
    // ahead -- 4 + 4 register sets -- ran 1.6-1.7x slower at 128^3 and 384^3,
    // profiles/r02_tune3d_depth.txt)
    D2 pl[2][LR];
    // rhs pairs of consecutive planes, rotating: 3 sets, loaded one step
    // ahead; RA2: 4 sets (set of plane x = (x - k0 + 1) & 3), two steps ahead
    constexpr int NRS = RA2 ? 4 : 3;
    D2 rs[NRS][RR];
    load_plane(k0 - 2, v0);
    load_plane(k0 - 1, v1);
    load_plane(k0, v2);
    load_plane(k0 + 1, pl[0]);
    if constexpr (RA2) {
        load_rhs(k0 - 2, rs[NRS - 1]);
        load_rhs(k0 - 1, rs[0]);
        load_rhs(k0, rs[1]);
    } else {
        load_rhs(k0 - 2, rs[2]);
        load_rhs(k0 - 1, rs[0]);
    }
    if (F.in) {
        // folded loop test (single rank): its partial-sum loads queue behind
        // the preloads, so it costs the LDS tree, not another memory latency;
        // L is free until the planes are stored
        if (fold_test(F, L)) return;  // uniform: every thread reads the same state
        __syncthreads();                 // scratch reads done before the planes land
    }
    store_plane(k0 - 2, v0);
    store_plane(k0 - 1, v1);
    store_plane(k0, v2);
    // step k uses the pairs of planes k (red) and k-1 (black) and loads k+1;
    // with k = k0-1+3n+u the three sets rotate with period 3, the planes with
    // period 2: unroll by 6
    if constexpr (RA2) {
        // step k = k0-1+u (mod 4): red uses rhs set u, black set u+3, loads
        // rhs k+2 into set u+2; p planes alternate as below
        for (int k = k0 - 1; k <= kend + 1; k += 4) {
            step(k, pl[1], pl[0], cA, cB, rs[0], rs[NRS - 1], rs[2]);
            if (k + 1 > kend + 1) break;
            step(k + 1, pl[0], pl[1], cB, cA, rs[1], rs[0], rs[NRS - 1]);
            if (k + 2 > kend + 1) break;
            step(k + 2, pl[1], pl[0], cA, cB, rs[2], rs[1], rs[0]);
            if (k + 3 > kend + 1) break;
            step(k + 3, pl[0], pl[1], cB, cA, rs[NRS - 1], rs[2], rs[1]);
        }
    } else
    for (int k = k0 - 1; k <= kend + 1; k += 6) {
        step(k, pl[1], pl[0], cA, cB, rs[0], rs[2], rs[1]);
        if (k + 1 > kend + 1) break;
        step(k + 1, pl[0], pl[1], cB, cA, rs[1], rs[0], rs[2]);
        if (k + 2 > kend + 1) break;
        step(k + 2, pl[1], pl[0], cA, cB, rs[2], rs[1], rs[0]);
        if (k + 3 > kend + 1) break;
        step(k + 3, pl[0], pl[1], cB, cA, rs[0], rs[2], rs[1]);
        if (k + 4 > kend + 1) break;
        step(k + 4, pl[1], pl[0], cA, cB, rs[1], rs[0], rs[2]);
        if (k + 5 > kend + 1) break;
        step(k + 5, pl[0], pl[1], cB, cA, rs[2], rs[1], rs[0]);
    }
    __syncthreads();  // black of plane kend done
    store_final(kend);
    const double s = block_sum256(acc, sh);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
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
        if (g.lo_phys) h[g.ix(a, b, 0)] = w[g.ix(a, b, 0)];
        if (g.hi_phys) h[g.ix(a, b, g.K)] = w[g.ix(a, b, g.K)];
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
        if (a < g.I && b <= g.K && g.koff + b < g.Kg)
            u[g.ix(a, g.J + 1, b)] = 2.0 - u[g.ix(a, g.J, b)];
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
    hipLaunchKernelGGL(k3_finish, dim3(1), dim3(1024), 0, s, partials, nb, 2, st, cells, 0);
    return nb;
}

int sweep3_blocks(const G3& g, int rows, int kc) {
    const long long nstr = (g.I + kSwOwn - 1) / kSwOwn, nrb = (g.J + rows - 1) / rows,
                    nkc = (g.K + kc - 1) / kc;
    return (int)(nstr * nrb * nkc);
}

static void sweep3_kernel(hipStream_t s, const G3& g, const double* src, double* dst,
                          const double* rhs, double idx2, double idy2, double idz2,
                          double factor, int rows, int kc, double* partials,
                          const DevState* st, const Fold3& F, bool ra2) {
    const int nstr = (g.I + kSwOwn - 1) / kSwOwn, nrb = (g.J + rows - 1) / rows;
    const int nb = sweep3_blocks(g, rows, kc);
#define K3SW(RR_, A_)                                                                       \
    hipLaunchKernelGGL((k3_sweep<RR_, A_>), dim3(nb), dim3(256), 0, s, g, src, dst, rhs, idx2,  \
                       idy2, idz2, factor, nstr, nrb, kc, partials, st, F)
    switch (rows) {
    case 4: if (ra2) K3SW(4, true); else K3SW(4, false); break;
    case 12: if (ra2) K3SW(12, true); else K3SW(12, false); break;
    default: if (ra2) K3SW(8, true); else K3SW(8, false); break;
    }
#undef K3SW
}

int launch3_sweep(hipStream_t s, const G3& g, const double* src, double* dst, const double* rhs,
                  double idx2, double idy2, double idz2, double factor, int rows, int kc,
                  double* partials, DevState* st, double cells, bool sum_only, bool ra2) {
    const int nb = sweep3_blocks(g, rows, kc);
    sweep3_kernel(s, g, src, dst, rhs, idx2, idy2, idz2, factor, rows, kc, partials, st,
                  Fold3{nullptr, 0, nullptr, nullptr, cells}, ra2);
    hipLaunchKernelGGL(k3_finish, dim3(1), dim3(1024), 0, s, partials, nb, 1, st, cells,
                       sum_only ? 1 : 0);
    return nb;
}

void launch3_sweep_folded(hipStream_t s, const G3& g, const double* src, double* dst,
                          const double* rhs, double idx2, double idy2, double idz2,
                          double factor, int rows, int kc, double* partials,
                          const double* prev_partials, const DevState* st_in, DevState* st_out,
                          double cells, bool ra2) {
    const int nb = sweep3_blocks(g, rows, kc);
    sweep3_kernel(s, g, src, dst, rhs, idx2, idy2, idz2, factor, rows, kc, partials, st_in,
                  Fold3{prev_partials, nb, st_in, st_out, cells}, ra2);
}

void launch3_fold_decide(hipStream_t s, const G3& g, int rows, int kc,
                         const double* prev_partials, const DevState* st_in, DevState* st_out,
                         double cells) {
    const int nb = sweep3_blocks(g, rows, kc);
    hipLaunchKernelGGL(k3_fold_decide, dim3(1), dim3(256), 0, s,
                       Fold3{prev_partials, nb, st_in, st_out, cells});
}

void launch3_decide(hipStream_t s, DevState* st, double cells) {
    hipLaunchKernelGGL(k3_decide, dim3(1), dim3(64), 0, s, st, cells);
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

void launch3_interior_sum(hipStream_t s, const G3& g, const double* p, double* partials,
                          double* sum) {
    const dim3 grid = cells_grid(g, g.I);
    hipLaunchKernelGGL(k3_sum_interior, grid, dim3(kBx, kBy), 0, s, g, p, partials);
    hipLaunchKernelGGL(k3_sum_finish, dim3(1), dim3(1024), 0, s, partials,
                       (int)(grid.x * grid.y * grid.z), sum);
}

void launch3_sub_mean(hipStream_t s, const G3& g, double* p, const double* sum, double cells) {
    hipLaunchKernelGGL(k3_sub_mean, cells_grid(g, g.I), dim3(kBx, kBy), 0, s, g, p, sum, cells);
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
