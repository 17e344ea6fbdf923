// sor_tb.hip -- temporally blocked red-black SOR for gfx950: T complete
// solveRB iterations (assignment-4/src/solver.c:197-229, T = 1..4) per pass
// over HBM.
//
// The single-iteration sweep (sor_kernels.hip) already moves the algorithmic
// minimum of one iteration -- read p, read rhs, write p: 24 B per lattice
// update -- and runs at ~93% of the measured HBM copy rate, so one iteration
// per pass cannot go meaningfully faster.  The dependency cone of an
// iteration is only two cells wide in each direction (red needs the old
// 5-point neighbourhood, black needs the new red one), so a wave that streams
// rows of the OLD field can push them through T iteration stages held in
// registers and write only the field after the last stage: p and rhs are read
// once and p written once per T iterations, 24/T B of HBM traffic per update.
//
// Work decomposition
//   wave = one strip: loads 128 columns (lane l: ia = c_ld + 2l, ib = ia + 1,
//          one 16-byte load per array per row), outputs the inner OW = 128-4T
//          columns [c_out, c_out + OW), c_ld = c_out - 2T.  Each iteration
//          stage loses two columns of validity per side (red reads +-1, black
//          reads the new red +-1), so after T stages exactly lanes
//          T .. 63-T hold correct values.  Overlapping loads between strips
//          are L2 hits; nothing is exchanged between waves.
//   rows = a block of H output rows [j0, j1); the wave streams OLD rows
//          j0-2T .. j1-1+2T upward.  Stage t receives the output row stream of
//          stage t-1 (stage 1: the old field) and, on receiving row rin,
//          updates the red cells of row rin-1 and the black cells of row
//          rin-2, emitting row rin-2 of iteration t.  Stage T's rows
//          j0 .. j1-1 are stored.
//   Every stage keeps 3 rows (A = row rin-1, M1 = rin-2 half updated, M2 =
//   final rin-3) and the rhs rows it needs come from one ring of 2T rows, so
//   the T stages cost ~20 VGPRs each and rhs is read once.
//
// Boundary handling per stage -- identical to the reference's end-of-
// iteration ghost copy (:219-227), applied to every intermediate iteration:
//   column 0 := column 1, column ni+1 := column ni for rows 1..nj (physical
//   left/right sides); row 0 := row 1 and row nj+1 := row nj for columns
//   1..ni (physical bottom/top: done on the receiving side of the row stream,
//   when the row it copies from arrives); corners never change.  On a side
//   that borders another rank the 2T-deep halo (exchanged before the pass)
//   supplies the neighbour's old values and the stages simply keep updating
//   them: identical arithmetic, so identical bits to what the owner computes.
//
// Residual: stage t accumulates r^2 of the cells this wave owns (output
// lanes, rows [j0, j1)), partial per workgroup per stage in a fixed order;
// the finish kernel decides iteration by iteration exactly like the
// single-sweep path.  If convergence (or itermax) is reached at stage t < T,
// the host recomputes that pass with T' = t from the untouched source buffer
// (misor_api.hip), so the returned field is the one after exactly `it`
// iterations.
//
// Bit-exactness: same expression order as the reference, -ffp-contract=off.

#include "misor_internal.h"

namespace misor {

namespace {

__device__ __forceinline__ double from_left(double v) { return __shfl_up(v, 1, 64); }
__device__ __forceinline__ double from_right(double v) { return __shfl_down(v, 1, 64); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2 ldv(const double* p) { return *reinterpret_cast<const d2*>(p); }

template <bool NT>
__device__ __forceinline__ void stv(double* p, d2 v) {
    if (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p));
    else
        *reinterpret_cast<d2*>(p) = v;
}

// per-lane constants shared by all stages
struct Lane {
    int ia, ib;            // the lane's two columns (ia odd)
    bool up_a, up_b;       // columns that are updated (inside [upd_lo_i, upd_hi_i])
    bool own_a, own_b;     // columns whose residual this lane counts
    bool fix0_b;           // ib == 0 on a physical left side: column 0 := column 1
    bool fixr_a, fixr_b;   // ia / ib == ni+1 on a physical right side
    int lo_j, hi_j;        // updated rows
    int j0, j1;            // owned rows
    int parity;
    int gb, gt, nj;
    double idx2, idy2, coef;
};

// One iteration stage.  In = row rin of the previous stage's output (stage 1:
// of the field in memory).  Returns row rin-2 of this stage's output.
// fixrows (stages 2..T; a constant after unrolling): complete the previous iteration's ghost-row copy on
// the incoming stream.  Stage 1 reads the ghost rows as they are in memory --
// the state after the previous pass, or whatever the caller uploaded, as the
// reference's first iteration does.
__device__ __forceinline__ d2 stage(const Lane& c, bool fixrows, d2 In, int rin, d2& A, d2& M1,
                                    d2& M2, d2 Ra, d2 Rb, double& acc) {
    if (fixrows) {
        if (c.gb && rin == 1) {  // row 0 := row 1 (A holds row 0)
            if (c.up_a) A.x = In.x;
            if (c.up_b) A.y = In.y;
        }
        if (c.gt && rin == c.nj + 1) {  // row nj+1 := row nj (A holds row nj)
            if (c.up_a) In.x = A.x;
            if (c.up_b) In.y = A.y;
        }
    }
    const int rr = rin - 1;  // red row
    const int rb = rin - 2;  // black row
    const int q = (c.parity + 1 + rr) & 1;  // 0: column ia is red in row rr (black in rb)
    const double idx2 = c.idx2, idy2 = c.idy2, coef = c.coef;

    // red pass on row rr
    d2 Mr = A;
    if (rr >= c.lo_j && rr <= c.hi_j) {
        const bool own = (rr >= c.j0) && (rr < c.j1);
        if (q == 0) {
            const double Lf = from_left(A.y);
            const double cc = A.x;
            const double r = Ra.x - (((A.y - 2.0 * cc) + Lf) * idx2 +
                                     ((In.x - 2.0 * cc) + M1.x) * idy2);
            if (c.up_a) Mr.x = cc - coef * r;
            if (c.own_a && own) acc += r * r;
        } else {
            const double Rf = from_right(A.x);
            const double cc = A.y;
            const double r = Ra.y - (((Rf - 2.0 * cc) + A.x) * idx2 +
                                     ((In.y - 2.0 * cc) + M1.y) * idy2);
            if (c.up_b) Mr.y = cc - coef * r;
            if (c.own_b && own) acc += r * r;
        }
    }

    // black pass on row rb (+ the ghost column copy of this finished row)
    d2 F = M1;
    if (rb >= c.lo_j && rb <= c.hi_j) {
        const bool own = (rb >= c.j0) && (rb < c.j1);
        if (q == 0) {
            const double Ln = from_left(M1.y);
            const double cc = M1.x;
            const double r = Rb.x - (((M1.y - 2.0 * cc) + Ln) * idx2 +
                                     ((Mr.x - 2.0 * cc) + M2.x) * idy2);
            if (c.up_a) F.x = cc - coef * r;
            if (c.own_a && own) acc += r * r;
        } else {
            const double Rn = from_right(M1.x);
            const double cc = M1.y;
            const double r = Rb.y - (((Rn - 2.0 * cc) + M1.x) * idx2 +
                                     ((Mr.y - 2.0 * cc) + M2.y) * idy2);
            if (c.up_b) F.y = cc - coef * r;
            if (c.own_b && own) acc += r * r;
        }
        const double f1 = from_right(F.x);  // column ib+1 (lane l+1's ia)
        const double fl = from_left(F.y);   // column ia-1 (lane l-1's ib)
        if (c.fix0_b) F.y = f1;
        if (c.fixr_a) F.x = fl;
        if (c.fixr_b) F.y = F.x;
    }
    M2 = F;
    M1 = Mr;
    A = In;
    return F;
}

}  // namespace

template <int T, int WAVES, int D, bool NT>
__global__ __launch_bounds__(kLanes* WAVES) void rb_tb_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, int force) {
    constexpr int OW = kStripCells - 4 * T;
    __shared__ double wsum[T][WAVES];
    if (!force && st->done) return;

    int L = blockIdx.x;
    if (prm.xcd_remap) {
        const int nwg = prm.nblocks, qq = nwg / 8, rr = nwg % 8, x = L % 8;
        L = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + L / 8;
    }
    const int bx = L % prm.nbx, by = L / prm.nbx;
    const int ni = prm.ni, nj = prm.nj;
    const int j0 = 1 + by * prm.rows_per_block;
    const int j1 = min(j0 + prm.rows_per_block, nj + 1);
    if (prm.part != 0) {  // overlapped decomposed pass: blocks clear of the halo first
        const int lo = 1 + bx * WAVES * OW - 2 * T;
        const int hi = 1 + (bx * WAVES + WAVES - 1) * OW - 2 * T + kStripCells - 1;
        const bool interior = lo >= prm.int_lo_i && hi <= prm.int_hi_i &&
                              j0 - 2 * T >= prm.int_lo_j && j1 - 1 + 2 * T <= prm.int_hi_j;
        if (interior != (prm.part == 1)) return;
    }

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int strip = bx * WAVES + wave;
    const int c_out = 1 + strip * OW;
    const long long pitch = prm.pitch;

    Lane c;
    c.ia = c_out - 2 * T + 2 * lane;
    c.ib = c.ia + 1;
    c.up_a = c.ia >= prm.upd_lo_i && c.ia <= prm.upd_hi_i;
    c.up_b = c.ib >= prm.upd_lo_i && c.ib <= prm.upd_hi_i;
    const bool own_lane = lane >= T && lane < kLanes - T;
    c.own_a = own_lane && c.ia <= ni;
    c.own_b = own_lane && c.ib <= ni;
    c.fix0_b = prm.ghost_left && c.ib == 0;
    c.fixr_a = prm.ghost_right && c.ia == ni + 1;
    c.fixr_b = prm.ghost_right && c.ib == ni + 1;
    c.lo_j = prm.upd_lo_j;
    c.hi_j = prm.upd_hi_j;
    c.j0 = j0;
    c.j1 = j1;
    c.parity = prm.parity;
    c.gb = prm.ghost_bottom;
    c.gt = prm.ghost_top;
    c.nj = nj;
    c.idx2 = prm.idx2;
    c.idy2 = prm.idy2;
    c.coef = prm.coef;
    // columns this lane stores: owned interior + the physical ghost columns
    const bool st_a = c.own_a || c.fixr_a;
    const bool st_b = c.own_b || c.fix0_b || c.fixr_b;

    double acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = 0.0;

    // physical corners are never touched by solveRB; carry them into dst
    if (L == 0 && threadIdx.x < 4) {
        const int t = threadIdx.x;
        const int ci = (t & 1) ? ni + 1 : 0, cj = (t & 2) ? nj + 1 : 0;
        const bool phys = ((t & 1) ? prm.ghost_right : prm.ghost_left) &&
                          ((t & 2) ? prm.ghost_top : prm.ghost_bottom);
        if (phys) {
            const long long k = (long long)(cj + kYOff) * pitch + (ci + kXOff);
            dst[k] = src[k];
        }
    }

    if (c_out <= ni) {  // wave-uniform
        const long long base = (long long)kYOff * pitch + kXOff + c.ia;
        const double* sp = src + base;
        const double* rp = rhs + base;
        double* dp = dst + base;
        auto ldp = [&](int j) { return ldv(sp + (long long)j * pitch); };
        auto ldr = [&](int j) { return ldv(rp + (long long)j * pitch); };

        const int rs = j0 - 2 * T;  // first streamed row
        d2 Pq[D], Rq[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            Pq[k] = ldp(rs + k);
            Rq[k] = ldr(rs - 1 + k);
        }
        d2 A[T], M1[T], M2[T], R[2 * T];
#pragma unroll
        for (int t = 0; t < T; ++t) A[t] = M1[t] = M2[t] = d2{0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 2 * T; ++k) R[k] = d2{0.0, 0.0};

        for (int r0 = rs; r0 <= j1 - 1 + 2 * T; ++r0) {
            const d2 nP = ldp(r0 + D);
            const d2 nR = ldr(r0 - 1 + D);
            // rhs ring: R[k] = rhs(r0 - 1 - k)
#pragma unroll
            for (int k = 2 * T - 1; k > 0; --k) R[k] = R[k - 1];
            R[0] = Rq[0];

            d2 v = Pq[0];
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const d2 prevM2 = M2[t];
                v = stage(c, t > 0, v, r0 - 2 * t, A[t], M1[t], M2[t], R[2 * t], R[2 * t + 1], acc[t]);
                if (t == T - 1) {
                    const int jw = r0 - 2 * T;  // row finished by the last stage
                    if (jw >= j0 && jw < j1) {
                        double* drow = dp + (long long)jw * pitch;
                        auto put = [&](double* p, d2 o) {
                            if (st_a && st_b)
                                stv<NT>(p, o);
                            else if (st_a)
                                p[0] = o.x;
                            else if (st_b)
                                p[1] = o.y;
                        };
                        put(drow, v);
                        // ghost rows of the stored field: interior columns from
                        // the finished row, corners from the (unchanged) ghost row
                        if (c.gb && jw == 1) {
                            const d2 g0 = prevM2;  // the stage's row 0
                            put(drow - pitch, d2{c.up_a ? v.x : g0.x, c.up_b ? v.y : g0.y});
                        }
                        if (c.gt && jw == nj) {
                            const d2 gn = M1[t];  // the stage's row nj+1 (after its fix)
                            put(drow + pitch, d2{c.up_a ? v.x : gn.x, c.up_b ? v.y : gn.y});
                        }
                    }
                }
            }

#pragma unroll
            for (int k = 0; k + 1 < D; ++k) {
                Pq[k] = Pq[k + 1];
                Rq[k] = Rq[k + 1];
            }
            Pq[D - 1] = nP;
            Rq[D - 1] = nR;
        }
    }

    // deterministic reduction per stage: lane tree, then waves in order
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const double s = wave_sum(acc[t]);
        if (lane == 0) wsum[t][wave] = s;
    }
    __syncthreads();
    if (threadIdx.x < T) {
        const int t = threadIdx.x;
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += wsum[t][w];
        partials[(long long)t * prm.nblocks + L] = s;
    }
}

int tb_out_width(int T) { return kStripCells - 4 * T; }

int tb_waves(int variant) { return kTbVariants[variant].waves; }

int tb_partials(int ni, int nj, int T, int rows_per_block, int waves, int* nbx, int* nby) {
    const int ow = tb_out_width(T);
    const int strips = (ni + ow - 1) / ow;
    *nbx = (strips + waves - 1) / waves;
    *nby = (nj + rows_per_block - 1) / rows_per_block;
    return (*nbx) * (*nby);
}

void launch_tb(hipStream_t s, int T, const SweepParams& prm, const double* src, double* dst,
               const double* rhs, double* partials, const DevState* st, int force) {
#define TB(TT, W, DD)                                                                      \
    hipLaunchKernelGGL((rb_tb_kernel<TT, W, DD, true>), dim3(prm.nblocks), dim3(kLanes * W), \
                       0, s, prm, src, dst, rhs, partials, st, force)
#define TB_T(TT)                              \
    switch (prm.variant) {                    \
    case 0: TB(TT, 4, 2); break;              \
    case 1: TB(TT, 8, 2); break;              \
    case 2: TB(TT, 4, 3); break;              \
    default: TB(TT, 8, 3); break;             \
    }
    // must match kTbVariants (misor_internal.h)
    switch (T) {
    case 1: TB_T(1); break;
    case 2: TB_T(2); break;
    case 3: TB_T(3); break;
    default: TB_T(4); break;
    }
#undef TB_T
#undef TB
}

}  // namespace misor
