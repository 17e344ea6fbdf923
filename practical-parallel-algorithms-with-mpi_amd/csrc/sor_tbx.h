// sor_tbx.h -- temporally blocked red-black SOR whose strips exchange their
// edge columns (TB variant 6; device code, included by sor_tb_inst.hip after
// sor_tb.h, whose helpers it uses).  T complete solveRB iterations
// (assignment-4/src/solver.c:197-229) per pass over HBM, as rb_tb_kernel.
//
// Why a second kernel.  rb_tb_kernel's waves are independent: each loads 128
// columns and owns the inner 128 - 4T of them, because every iteration stage
// loses a column of validity per side and colour.  That halo is recomputed
// work: x 1.33 at T = 8, x 1.45 at T = 10, and the kernel is VALU-issue-bound
// (DESIGN.md section 4), so it is a third of its time -- and it grows with T,
// which keeps T at 8 and a 20-iteration solve at three HBM passes.
//
// Here the W waves of a workgroup hold W adjacent 128-column strips and give
// each other the one column a stage needs across a strip boundary.  A stage
// at step n (streamed row r0) needs of its neighbour strip exactly the values
// that neighbour had at the end of step n-1 (its A and M1 registers: the row
// the red update reads, and the row whose black cells it updates next), so:
//   end of step n:   each wave writes, for every stage, the two values its
//                    neighbour needs next step (lane 0's A.x, M1.x for the
//                    left neighbour or lane 63's A.y, M1.y for the right one:
//                    the colour of step n+1 decides which) to LDS, waits for
//                    its LDS writes, and joins one s_barrier;
//   step n+1:        lane 0 (or 63) of the neighbour reads them (broadcast
//                    LDS reads) and the x-neighbour DPP shift takes them as its
//                    `old` operand (update_dpp with bound_ctrl off: the lane
//                    without a source lane keeps old) -- no VALU instruction.
// Only the workgroup's two outer sides lose validity: it loads 128 W columns
// and owns 128 W - 4T of them (x 1.085 at W = 4, T = 10).  Two buffers by
// step parity (a wave may write step n+1's values while its neighbour still
// reads step n's).  The per-update arithmetic is rb_tb_kernel's, bit for bit.
//
// The rhs ring moves to LDS so that T = 10 fits the 256 VGPRs of two waves per
// SIMD: rhs row y (block-relative: absolute row rs - 1 + y) is used by stage t
// at steps y + 2t (red) and y + 2t + 1 (black).  Stage 0 reads it from the
// registers it was loaded into (D rows ahead); at the end of step y + 1 it is
// written to LDS slot y mod S, S = 2T - 2, for stages 1 .. T-1 (row y + S
// overwrites the slot at the end of step y + S + 1 = y + 2T - 1, after row y's
// last read).  Each slot holds the row split by column parity (ia | ib), so a
// stage reads the 64 doubles of its colour conflict-free.  LDS per workgroup
// at W = 4, T = 10: 4 x 18 KB ring + 2 KB exchange: two workgroups per CU.
//
// Interior blocks (every column updated, rows clear of the physical bottom /
// top sides, H a multiple of S) march in chunks of S statically unrolled steps
// (ring slots and colours compile-time); the block's stream starts Wu = 4T
// rounded up to a multiple of S rows early (the warm-up is whole chunks whose
// stores go out of range and whose residual is discarded).  All other blocks
// (a physical side in the cone, a ragged height) take the general march: pairs
// of steps with run-time ring slots, per-lane masks and row tests, and the
// physical ghost column/row copies of the reference (:219-227) per stage.
// At a physical right side the ghost column ni+1 may be the first column of
// the next strip, whose value that strip can only give a step late; for
// stages t >= 1 the ghost equals the old value of column ni itself (the
// previous iteration's copy), so the lane of column ni uses its own value as
// its right neighbour there (stage 0 reads the ghost as it is in memory, as
// the reference's first iteration does) and also stores the ghost column.
//
// Residual windows, partials (one per block and stage, waves in a fixed
// order), block order and persistent queues are rb_tb_kernel's.
#pragma once

#include "sor_tb.h"

namespace misor {

namespace {

#ifndef XHOIST
#define XHOIST 1
#endif
#ifndef XLA
#define XLA 2   // stages of LDS reads in flight ahead of the computing stage
#endif
#ifndef XEARLY
#define XEARLY 1  // publish a stage's edge values right after the stage, not at the step's end
#endif

// LDS ring slots (rows of rhs for stages 1 .. T-1) and the warm-up length
template <int T>
__host__ __device__ constexpr int xslots() {
    return 2 * T - 2 > 2 ? 2 * T - 2 : 2;
}
template <int T>
__host__ __device__ constexpr int xwarm() {
    return (4 * T + xslots<T>() - 1) / xslots<T>() * xslots<T>();
}

// lane l receives lane l-1's v; lane 0 keeps `old` (the left neighbour strip's value)
__device__ __forceinline__ double shr_in(double v, double old) {
    return __hiloint2double(
        __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x138, 0xf, 0xf, false),
        __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x138, 0xf, 0xf, false));
}
// lane l receives lane l+1's v; lane 63 keeps `old` (the right neighbour strip's value)
__device__ __forceinline__ double shl_in(double v, double old) {
    return __hiloint2double(
        __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false),
        __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false));
}

template <int T, int W>
struct XShared {
    double ring[W][xslots<T>()][2][kLanes];  // [wave][slot][column parity][lane]
    double xch[2][W + 2][T][2];              // [step parity][1 + writer wave][stage][A, M1]
    double wsum[T][W];
    int ticket;
};

template <int T, int D>
struct XMarch {
    d2 A[T], M1[T], M2[T];
    d2 Pq[D], Rq[D];  // rows in flight
    d2 R0, R1;        // rhs rows n and n-1 (stage 0)
    double acc[T];
    d2 keep[2];
};

// per-lane state of the general march (rb_tb_kernel's Lane, plus the right
// ghost rule of the header)
struct XLane {
    bool up_a, up_b, own_a, own_b, fix0_b, fixr_a, fixr_b;
    bool ccr;   // ib == ni on a physical right side: right neighbour = own old value (t >= 1)
    int lo_j, hi_j, j0, j1, wlo, whi, gb, gt, nj;
};

// One stage with the neighbour strips' values nA, nM (see the header).  In =
// row rin (previous stage's output), returns row rin - 2 of this stage.
// MODE: kSteady (interior: no masks, no row tests) or kEdge (general).
template <int T, int Q, int MODE, bool P2>
__device__ __forceinline__ d2 xstage(const XLane& c, int t, int rin, d2 In, d2& A, d2& M1, d2& M2,
                                     double Rr, double Rb, double nA, double nM, double idx2,
                                     double idy2, double coef, double& acc) {
    constexpr bool EDGE = MODE == kEdge;
    if (EDGE && t > 0) {  // complete the previous iteration's ghost-row copy on the stream
        if (c.gb && rin == 1) {
            if (c.up_a) A.x = In.x;
            if (c.up_b) A.y = In.y;
        }
        if (c.gt && rin == c.nj + 1) {
            if (c.up_a) In.x = A.x;
            if (c.up_b) In.y = A.y;
        }
    }
    const int rr = rin - 1, rb = rin - 2;
    const int sh = 2 * T - 1 - 2 * t;
    auto tally = [&](double r, int row, int wsh, bool own_col) {
        if (!EDGE) {
            acc = __builtin_fma(r, r, acc);
        } else {
            const bool own_row = row >= (c.wlo ? 1 : c.j0 + wsh) &&
                                 row < (c.whi ? c.nj + 1 : c.j1 + wsh);
            if (own_row && own_col) acc = __builtin_fma(r, r, acc);
        }
    };
    d2 Mr = A;
    if (!EDGE || (rr >= c.lo_j && rr <= c.hi_j)) {
        if (Q == 0) {
            const double cc = A.x;
            const double r = resid<P2>(Rr, m2c(A.y, cc) + shr_in(A.y, nA), m2c(In.x, cc) + M1.x,
                                       idx2, idy2);
            if (!EDGE || c.up_a) Mr.x = cc - coef * r;
            tally(r, rr, sh, c.own_a);
        } else {
            const double cc = A.y;
            double Rf = shl_in(A.x, nA);
            if (EDGE && t > 0 && c.ccr) Rf = cc;
            const double r = resid<P2>(Rr, m2c(Rf, cc) + A.x, m2c(In.y, cc) + M1.y, idx2, idy2);
            if (!EDGE || c.up_b) Mr.y = cc - coef * r;
            tally(r, rr, sh, c.own_b);
        }
    }
    d2 F = M1;
    if (!EDGE || (rb >= c.lo_j && rb <= c.hi_j)) {
        if (Q == 0) {
            const double cc = M1.x;
            const double r = resid<P2>(Rb, m2c(M1.y, cc) + shr_in(M1.y, nM), m2c(Mr.x, cc) + M2.x,
                                       idx2, idy2);
            if (!EDGE || c.up_a) F.x = cc - coef * r;
            tally(r, rb, sh - 1, c.own_a);
        } else {
            const double cc = M1.y;
            double Rn = shl_in(M1.x, nM);
            if (EDGE && t > 0 && c.ccr) Rn = cc;
            const double r = resid<P2>(Rb, m2c(Rn, cc) + M1.x, m2c(Mr.y, cc) + M2.y, idx2, idy2);
            if (!EDGE || c.up_b) F.y = cc - coef * r;
            tally(r, rb, sh - 1, c.own_b);
        }
        if (EDGE) {  // ghost columns of the finished row (within the strip)
            const double f1 = from_right(F.x);
            const double fl = from_left(F.y);
            if (c.fix0_b) F.y = f1;
            if (c.fixr_a) F.x = fl;
            if (c.fixr_b) F.y = F.x;
        }
    }
    M2 = F;
    M1 = Mr;
    A = In;
    return F;
}

// the LDS traffic of a step's end: this step's edge values for the neighbours'
// next step (colour 1 - Q), rhs row n-1 into its ring slot; then the barrier
// stage t's edge values (its A and M1 after the stage) for the neighbours' next step
template <int Q>
__device__ __forceinline__ void xpub_stage(const d2& A, const d2& M1, double* xw, int t,
                                           int lane) {
    if (Q == 1) {  // next step is colour 0: the right neighbour reads lane 63's .y
        if (lane == kLanes - 1) {
            xw[2 * t] = A.y;
            xw[2 * t + 1] = M1.y;
        }
    } else {  // next step is colour 1: the left neighbour reads lane 0's .x
        if (lane == 0) {
            xw[2 * t] = A.x;
            xw[2 * t + 1] = M1.x;
        }
    }
}

template <int T, int D, int Q>
__device__ __forceinline__ void xpublish(XMarch<T, D>& m, double* xw, double* ringslot, int lane,
                                         bool stages = true) {
    if (stages) {
#pragma unroll
        for (int t = 0; t < T; ++t) xpub_stage<Q>(m.A[t], m.M1[t], xw, t, lane);
    }
    ringslot[lane] = m.R1.x;
    ringslot[kLanes + lane] = m.R1.y;
}

__device__ __forceinline__ void xbarrier() {
    // the LDS writes of this step are done before any wave passes; no vector
    // memory wait (loads run D rows ahead across the barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // no code motion across steps (as rb_tb_kernel's steady_step)
    __builtin_amdgcn_sched_barrier(0);
}

// buffer descriptors of one strip (wave-uniform base, lane byte offsets)
struct XIo {
    __amdgpu_buffer_rsrc_t p, r, d;
    unsigned lane;      // lane * 16
    unsigned st_lane;   // lane * 16 if the lane stores both columns, else out of range
    unsigned row_bytes;
    double idx2, idy2, coef;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xrsrc(const double* b, long long pitch, int row0,
                                                        int col0, int rows) {
    const unsigned long long a =
        (unsigned long long)(b + (long long)(kYOff + row0) * pitch + kXOff + col0);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo),
                                             (short)0, (int)((long long)rows * pitch * 8),
                                             0x00020000);
}

// step n of an interior march, n mod S = PH, colour Q, exchange parity PAR =
// n & 1.  off_n: byte offset of streamed row n; so: store offset of the row
// the last stage finishes (out of range in warm-up chunks)
template <int T, int W, int D, int Q, int PH, int PAR, bool P2>
__device__ __forceinline__ void xsteady_step(XMarch<T, D>& m, const XLane& c, const XIo& io,
                                             XShared<T, W>& sh, int wave, int lane, unsigned off_n,
                                             unsigned so) {
    constexpr int S = xslots<T>();
    const unsigned ld = off_n + (unsigned)D * io.row_bytes;
    const d2 nP = bload(io.p, io.lane, ld);
    const d2 nR = bload(io.r, io.lane, ld);
    m.R1 = m.R0;
    m.R0 = m.Rq[0];
    // the neighbour written at step n-1: left (Q = 0) or right (Q = 1)
    const double* xr = &sh.xch[PAR ^ 1][wave + (Q == 0 ? 0 : 2)][0][0];
    const double* ring = &sh.ring[wave][0][0][0];
    // every LDS read of the step issued at its start: the step is a serial
    // chain of 2T updates, so a read issued at its stage would put its latency
    // on that chain T times over
    // (a sliding window: the reads of stages 0 .. XLA at the start, those of
    // stage t + XLA + 1 once stage t is done -- all of them at once do not
    // fit the registers at T = 10)
    constexpr int LA = XLA < T ? XLA : T - 1;
    double nA[T], nM[T], rr[T], rb[T];
    rr[0] = Q == 0 ? m.R0.x : m.R0.y;
    rb[0] = Q == 0 ? m.R1.x : m.R1.y;
    auto issue = [&](int t) {
        nA[t] = xr[2 * t];
        nM[t] = xr[2 * t + 1];
        if (t > 0) {
            const int sr = (PH - 2 * t + 4 * S) % S, sb = (PH - 2 * t - 1 + 4 * S) % S;
            rr[t] = ring[(sr * 2 + Q) * kLanes + lane];
            rb[t] = ring[(sb * 2 + Q) * kLanes + lane];
        }
    };
#pragma unroll
    for (int t = 0; t <= LA; ++t) issue(t);
    if (XHOIST) __builtin_amdgcn_sched_barrier(0);
    double* const xw = &sh.xch[PAR][wave + 1][0][0];
    double* const rslot = &sh.ring[wave][(PH - 1 + S) % S][0][0];
    d2 v = m.Pq[0];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        v = xstage<T, Q, kSteady, P2>(c, t, 0, v, m.A[t], m.M1[t], m.M2[t], rr[t], rb[t], nA[t],
                                      nM[t], io.idx2, io.idy2, io.coef, m.acc[t]);
        // XEARLY: the stage's edge values go out at once, so the step's closing
        // wait covers the last stage's write only; rhs row n-1 goes into its slot
        // once the last read of that slot (stage T-1's black, in this step) is
        // issued (a wave's LDS operations complete in order)
        if (XEARLY) xpub_stage<Q>(m.A[t], m.M1[t], xw, t, lane);
        if (t + LA + 1 < T) {
            issue(t + LA + 1);
            if (XEARLY && t + LA + 1 == T - 1) {
                rslot[lane] = m.R1.x;
                rslot[kLanes + lane] = m.R1.y;
            }
            if (XHOIST) __builtin_amdgcn_sched_barrier(0);
        }
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), io.d, io.st_lane, so, 2);
    if (!XEARLY || LA + 1 >= T) {  // (LA + 1 >= T: every read was issued at the start)
        xpublish<T, D, Q>(m, xw, rslot, lane, !XEARLY);
    }
    // the store reads its data VGPRs after it issues (sor_tb.h steady_step)
    asm volatile("" ::"v"(m.keep[0]));
    m.keep[0] = m.keep[1];
    m.keep[1] = v;
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) {
        m.Pq[k] = m.Pq[k + 1];
        m.Rq[k] = m.Rq[k + 1];
    }
    m.Pq[D - 1] = nP;
    m.Rq[D - 1] = nR;
    // the residual sums stay materialised step by step: without this the
    // compiler sinks a chunk's tallies below the post-warm-up reset (where
    // they are dead) and keeps every r of the chunk alive -- spilled
#pragma unroll
    for (int t = 0; t < T; ++t) asm volatile("" : "+v"(m.acc[t]));
    xbarrier();
}

template <int T, int W, int D, int Q0, bool P2, int... NN>
__device__ __forceinline__ void xsteady_chunk(XMarch<T, D>& m, const XLane& c, const XIo& io,
                                              XShared<T, W>& sh, int wave, int lane, unsigned off,
                                              unsigned so, std::integer_sequence<int, NN...>) {
    (xsteady_step<T, W, D, Q0 ^ (NN & 1), NN, NN & 1, P2>(
         m, c, io, sh, wave, lane, off + (unsigned)NN * io.row_bytes,
         so + (unsigned)NN * io.row_bytes),
     ...);
}

// General march: step n (block-relative, any n), colour Q, parity PAR = n & 1
// (pairs of steps start at even n), ring slot phase ph = n mod S at run time.
// Rows r0 = rs + n; stores of the row the last stage finishes (row r0 - 2T)
// if it is one of the block's, with the physical ghost rows and column.
struct XGio {
    __amdgpu_buffer_rsrc_t p, r, d;  // p rows from rs, rhs rows from rs - 1, dst rows from j0 - 1
    unsigned lane, row_bytes;
    unsigned st_a, st_b, st_r;  // byte offsets of the lane's stores (out of range: none)
    double idx2, idy2, coef;
};

template <int T, int W, int D, int Q, int PAR, bool P2>
__device__ __forceinline__ void xgen_step(XMarch<T, D>& m, const XLane& c, const XGio& io,
                                          XShared<T, W>& sh, int wave, int lane, int n, int rs,
                                          int ph) {
    constexpr int S = xslots<T>();
    const unsigned ld = (unsigned)(n + D) * io.row_bytes;
    const d2 nP = bload(io.p, io.lane, ld);
    const d2 nR = bload(io.r, io.lane, ld);
    m.R1 = m.R0;
    m.R0 = m.Rq[0];
    const double* xr = &sh.xch[PAR ^ 1][wave + (Q == 0 ? 0 : 2)][0][0];
    const double* ring = &sh.ring[wave][0][0][0];
    const int r0 = rs + n;
    d2 v = m.Pq[0];
    d2 g0{0.0, 0.0}, gn{0.0, 0.0};
#pragma unroll
    for (int t = 0; t < T; ++t) {
        double rr, rb;
        if (t == 0) {
            rr = Q == 0 ? m.R0.x : m.R0.y;
            rb = Q == 0 ? m.R1.x : m.R1.y;
        } else {
            int sr = ph - 2 * t, sb = ph - 2 * t - 1;
            sr += sr < 0 ? S : 0;
            sr += sr < 0 ? S : 0;
            sb += sb < 0 ? S : 0;
            sb += sb < 0 ? S : 0;
            rr = ring[(sr * 2 + Q) * kLanes + lane];
            rb = ring[(sb * 2 + Q) * kLanes + lane];
        }
        if (t == T - 1) g0 = m.M2[t];  // the stage's row 0 (before this step), for the corner
        v = xstage<T, Q, kEdge, P2>(c, t, r0 - 2 * t, v, m.A[t], m.M1[t], m.M2[t], rr, rb,
                                    xr[2 * t], xr[2 * t + 1], io.idx2, io.idy2, io.coef,
                                    m.acc[t]);
        if (t == T - 1) gn = m.M1[t];  // the stage's row nj+1 (after its fix)
        // stage by stage: the general march is register-heavy (masks, run-time
        // ring addresses); no hoisting of later stages' LDS reads
        __builtin_amdgcn_sched_barrier(0);
    }
    const int jw = r0 - 2 * T;  // row finished by the last stage
    if (jw >= c.j0 && jw < c.j1) {
        // dst descriptor from row j0 - 1
        const unsigned o = (unsigned)(jw - c.j0 + 1) * io.row_bytes;
        const double vx = v.x, vy = v.y;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vx), io.d, io.st_a, o, 2);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vy), io.d, io.st_b, o, 2);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vy), io.d, io.st_r, o, 2);
        // ghost rows of the stored field: interior columns from the finished
        // row, the others unchanged (corners: copy_corners)
        if (c.gb && jw == 1) {
            const double ax = c.up_a ? vx : g0.x, by_ = c.up_b ? vy : g0.y;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, ax), io.d, io.st_a,
                                                  o - io.row_bytes, 2);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, by_), io.d, io.st_b,
                                                  o - io.row_bytes, 2);
        }
        if (c.gt && jw == c.nj) {
            const double ax = c.up_a ? vx : gn.x, by_ = c.up_b ? vy : gn.y;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, ax), io.d, io.st_a,
                                                  o + io.row_bytes, 2);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, by_), io.d, io.st_b,
                                                  o + io.row_bytes, 2);
        }
    }
    int sw = ph - 1;
    sw += sw < 0 ? S : 0;
    xpublish<T, D, Q>(m, &sh.xch[PAR][wave + 1][0][0], &sh.ring[wave][sw][0][0], lane);
    asm volatile("" ::"v"(m.keep[0]));
    m.keep[0] = m.keep[1];
    m.keep[1] = v;
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) {
        m.Pq[k] = m.Pq[k + 1];
        m.Rq[k] = m.Rq[k + 1];
    }
    m.Pq[D - 1] = nP;
    m.Rq[D - 1] = nR;
    // the residual sums stay materialised step by step: without this the
    // compiler sinks a chunk's tallies below the post-warm-up reset (where
    // they are dead) and keeps every r of the chunk alive -- spilled
#pragma unroll
    for (int t = 0; t < T; ++t) asm volatile("" : "+v"(m.acc[t]));
    xbarrier();
}

}  // namespace

// one block (bx, by) of a pass: logical block L, all W waves
template <int T, int W, int D, bool P2>
__device__ __forceinline__ void tbx_block(const SweepParams& prm, const double* __restrict__ src,
                                          double* __restrict__ dst,
                                          const double* __restrict__ rhs,
                                          double* __restrict__ partials, const int L,
                                          XShared<T, W>& sh) {
    constexpr int S = xslots<T>();
    constexpr int WU = xwarm<T>();
    constexpr int OWG = kStripCells * W - 4 * T;  // owned columns of the workgroup
    const int bx = L % prm.nbx, by = L / prm.nbx;
    int j0, j1;
    block_rows(prm, by, j0, j1);
    const int C0 = 1 + bx * OWG, cL = C0 - 2 * T;  // first owned / loaded column
    if (prm.part != 0) {  // overlapped decomposed pass: blocks clear of the halo first
        const bool interior = cL >= prm.int_lo_i && cL + kStripCells * W - 1 <= prm.int_hi_i &&
                              j0 - 2 * T >= prm.int_lo_j && j1 - 1 + 2 * T <= prm.int_hi_j;
        if (interior != (prm.part == 1)) return;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (L == 0) copy_corners(prm, src, dst);
    const int ni = prm.ni, nj = prm.nj;
    const long long pitch = prm.pitch;
    const int own_end = min(ni, C0 + OWG - 1);
    const int c_ld = cL + kStripCells * wave;

    XLane c;
    const int ia = c_ld + 2 * lane, ib = ia + 1;
    c.up_a = ia >= prm.upd_lo_i && ia <= prm.upd_hi_i;
    c.up_b = ib >= prm.upd_lo_i && ib <= prm.upd_hi_i;
    c.own_a = ia >= C0 && ia <= own_end;
    c.own_b = ib >= C0 && ib <= own_end;
    c.fix0_b = prm.ghost_left && ib == 0;
    c.fixr_a = prm.ghost_right && ia == ni + 1;
    c.fixr_b = prm.ghost_right && ib == ni + 1;
    c.ccr = prm.ghost_right && ib == ni;
    c.lo_j = prm.upd_lo_j;
    c.hi_j = prm.upd_hi_j;
    c.j0 = j0;
    c.j1 = j1;
    c.wlo = by == 0 && prm.ghost_bottom;
    c.whi = by == prm.nby - 1 && prm.ghost_top;
    c.gb = prm.ghost_bottom;
    c.gt = prm.ghost_top;
    c.nj = nj;

    XMarch<T, D> m;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        m.A[t] = m.M1[t] = m.M2[t] = d2{0.0, 0.0};
        m.acc[t] = 0.0;
    }
    m.keep[0] = m.keep[1] = d2{0.0, 0.0};
    m.R0 = m.R1 = d2{0.0, 0.0};

    // interior: every column of the workgroup's cone updated, the owned
    // columns end between lanes (a 16-byte store per owning lane), rows clear
    // of the physical sides and inside the allocation, height on the ring
    const bool cols_in = cL >= prm.upd_lo_i && cL + kStripCells * W - 1 <= prm.upd_hi_i &&
                         (C0 + OWG - 1 <= ni || (ni & 1) == 0);
    const int rs_in = j0 - 2 * T - (WU - 4 * T);
    const bool rows_in = rs_in >= prm.upd_lo_j && rs_in >= 1 - 2 * T &&
                         j1 - 1 + 2 * T <= prm.upd_hi_j && (j1 - j0) % S == 0 && j1 > j0;
#ifdef TBX_NO_INT
    if (false) {
#else
    if (cols_in && rows_in) {
#endif
        const int rs = rs_in;
        const int nsteps = WU + (j1 - j0);
        XIo io;
        io.p = xrsrc(src, pitch, rs, c_ld, nsteps + D);
        io.r = xrsrc(rhs, pitch, rs - 1, c_ld, nsteps + D);
        io.d = xrsrc(dst, pitch, j0, c_ld, j1 - j0);
        io.lane = (unsigned)lane * 16u;
        io.st_lane = c.own_a && c.own_b ? (unsigned)lane * 16u : 0x40000000u;
        io.row_bytes = (unsigned)(pitch * 8);
        io.idx2 = prm.idx2;
        io.idy2 = prm.idy2;
        io.coef = prm.coef;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            m.Pq[k] = bload(io.p, io.lane, (unsigned)k * io.row_bytes);
            m.Rq[k] = bload(io.r, io.lane, (unsigned)k * io.row_bytes);
        }
        const bool q1 = ((prm.parity + rs) & 1) != 0;
        // one loop per colour of the first row (a single chunk body per loop)
        auto march = [&](auto qc) {
            constexpr int Q0 = decltype(qc)::value;
            const int nch = nsteps / S, nwarm = WU / S;
            unsigned off = 0;
            for (int k = 0; k < nch; ++k) {
                // rows the last stage finishes in this chunk: j0 + (k - nwarm) S ..
                const unsigned so =
                    k < nwarm ? 0x40000000u : (unsigned)(k - nwarm) * S * io.row_bytes;
                xsteady_chunk<T, W, D, Q0, P2>(m, c, io, sh, wave, lane, off, so,
                                               std::make_integer_sequence<int, S>{});
                off += (unsigned)S * io.row_bytes;
                if (k == nwarm - 1) {  // warm-up residuals are not the block's
#pragma unroll
                    for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
                }
            }
        };
        if (q1) march(std::integral_constant<int, 1>{});
        else    march(std::integral_constant<int, 0>{});
#pragma unroll
        for (int t = 0; t < T; ++t) m.acc[t] = (c.own_a && c.own_b) ? m.acc[t] : 0.0;
    } else {
#ifndef TBX_NO_GEN
        const int rs = j0 - 2 * T, rend = j1 - 1 + 2 * T;
        const int nsteps = rend - rs + 1;
        XGio io;
        io.p = xrsrc(src, pitch, rs, c_ld, nsteps + D);
        io.r = xrsrc(rhs, pitch, rs - 1, c_ld, nsteps + D);
        io.d = xrsrc(dst, pitch, j0 - 1, c_ld, j1 - j0 + 2);
        io.lane = (unsigned)lane * 16u;
        io.row_bytes = (unsigned)(pitch * 8);
        // stored columns: owned cells, the physical ghost column 0 (lane of
        // column 0), and the right ghost column from the lane of column ni
        const bool st_a = c.own_a, st_b = c.own_b || c.fix0_b || c.fixr_b;
        io.st_a = st_a ? (unsigned)lane * 16u : 0x40000000u;
        io.st_b = st_b ? (unsigned)lane * 16u + 8u : 0x40000000u;
        io.st_r = c.ccr && c.own_b ? (unsigned)lane * 16u + 16u : 0x40000000u;
        io.idx2 = prm.idx2;
        io.idy2 = prm.idy2;
        io.coef = prm.coef;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            m.Pq[k] = bload(io.p, io.lane, (unsigned)k * io.row_bytes);
            m.Rq[k] = bload(io.r, io.lane, (unsigned)k * io.row_bytes);
        }
        const bool q1 = ((prm.parity + rs) & 1) != 0;
        int ph = 0;
        auto pair = [&](auto qc, int n) {
            constexpr int Q0 = decltype(qc)::value;
            xgen_step<T, W, D, Q0, 0, P2>(m, c, io, sh, wave, lane, n, rs, ph);
            ph = ph + 1 == S ? 0 : ph + 1;
            xgen_step<T, W, D, 1 - Q0, 1, P2>(m, c, io, sh, wave, lane, n + 1, rs, ph);
            ph = ph + 1 == S ? 0 : ph + 1;
        };
        for (int n = 0; n < nsteps; n += 2) {  // (an odd last step runs a step past rend:
            if (q1) pair(std::integral_constant<int, 1>{}, n);  // its row is never stored)
            else    pair(std::integral_constant<int, 0>{}, n);
        }
#endif
    }
    block_partials<T, W>(prm, m.acc, partials, L, sh.wsum);
}

// persistent (queue) or one-workgroup-per-block pass of the exchange variant
template <int T, int W, int D, bool P2>
__global__ __launch_bounds__(kLanes* W, 2) void rb_tbx_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, int force, int* __restrict__ queue) {
    __shared__ XShared<T, W> sh;
    if (!force && st->done) return;
    for_each_block(prm, queue, &sh.ticket, [&](int L) {
        tbx_block<T, W, D, P2>(prm, src, dst, rhs, partials, L, sh);
    });
}

}  // namespace misor
