// sor_tbh.h -- the temporally blocked sweep with a split rhs ring (TB
// variant kHrTbVariant: rb_tbhc_kernel, chained runs, below).  Device code;
// included by sor_tb_inst.hip after sor_tb.h, whose stage() arithmetic it runs
// unchanged.
//
// Why.  A pass of the 2-column march (sor_tb.h) costs, at 32768^2, about
// 4.7 ms of streaming (T = 1: 4.68 ms per launch) plus ~0.19 ms per stage
// (profiles/r04_tcurve.txt): the launch is close to HBM-bound, so the
// driver's 20-iteration solve is cheapest in as few passes as possible.  The
// register budget caps T at 8 (passes of 7 + 7 + 6): the rhs ring alone holds
// 2T + D rows of the strip, 4 VGPRs each (88 at T = 10), beside the stages'
// 10 VGPRs each, and T = 9 / 10 spill inside the steady chunk (8.1 / 9.2 ms
// per launch against 5.6 at T = 8).
//
// What.  Stages 0 .. K-1 read their rhs rows from a register ring of S slots
// as before; the older rows -- those stages K .. T-1 read -- move to an LDS
// ring of the same S slots (row j in slot j mod S, so a chunk of S steps has
// static slots in both rings): the row stage K-1 reads last in step n (row
// n - 2K + 1) is written to LDS in that step, two 512-byte halves (column a
// | column b, so a stage's read of one colour's column is one conflict-free
// ds_read_b64).  K is chosen to balance the rings: S = max(2K + D,
// 2(T - K) + 1), even -- 12 slots at T = 10 (48 VGPRs of ring instead of 88,
// 12 KB of LDS per wave, 96 KB per CU at two workgroups of four waves; with the
// skew of hrs_step, 18 slots: 18 KB per wave).
//
// Every block runs the static ring from its first step: interior blocks warm
// up for exactly 4T steps (4T + 1 skewed) -- whole kPre chunks, then a partial
// one -- and run kSteady chunks from that ring phase on (the warm-up rounded
// up to whole chunks cost ~3% of a T = 10 pass); blocks at a physical side
// or of a height the ring does not divide run kEdge / kRowEdge chunks over
// ceil((H + 4T) / S) chunks, the steps past the block's last row reading
// zeros (range-checked buffer loads) and storing / counting nothing (the row
// tests).  Rows the LDS stages read before any step wrote them belong to
// rows below the stream, outside every stage's valid cone.
#pragma once

#include "sor_tb.h"

namespace misor {

namespace {

// SK: the skewed form (hrs_step), T >= 2
template <int T, int D, int SK = 0>
struct Hr {
    static constexpr int K = hr_k(T, D, SK);      // stages 0 .. K-1: rhs from registers
    static constexpr int S = hr_slots(T, D, SK);  // slots of both rings (misor_internal.h)
    static constexpr int SKH = SK ? T / 2 : 0;    // leading stages of the skewed form
    // interior warm-up steps: 4T -- 4T + 1 in the skewed form, whose leading
    // stages never see the stream's first row: WU / S whole chunks, then WR
    // steps; the steady chunks start at ring phase WR
    static constexpr int WU = 4 * T + SK;
    static constexpr int WR = WU % S;
    static_assert(!SK || (T >= 2 && K <= SKH), "skewed split ring");
};

template <int T, int D>
struct HrMarch {
    d2 A[T], M1[T], M2[T];
    d2 Pq[D];
    TallyAcc acc[T];
    d2 keep[2];
    d2 B;  // skewed form: stage SKH-1's output of the previous step
};

struct HrIo {
    __amdgpu_buffer_rsrc_t p, r, d;  // p rows from rs0, rhs rows from rs0 - 1, dst rows from j0
    unsigned lane;                   // lane * 16
    unsigned st_lane;                // kSteady: lane * 16 if the lane stores, else out of range
    unsigned st_a, st_b;             // kSteadyEdge: per column (lane * 16 (+ 8) or out of range)
    unsigned row_bytes;
    lds_double* lx;                  // the wave's LDS ring (+ lane): slot s at lx + 128 s
    double* dp;                      // kEdge / kRowEdge stores: dst at row 0 of the lane's columns
    long long pitch;
};

__device__ __forceinline__ void hr_stv(double* p, d2 v) { stv(p, v); }

// step n of the split-ring march (stream row r0 = rs0 + n; PH = n mod S)
template <int T, int D, int MODE, int Q, int PH, bool P2>
__device__ __forceinline__ void hr_step(HrMarch<T, D>& m, d2* R, const Lane& c, const HrIo& io,
                                        int r0, unsigned off_n, unsigned st_base) {
    constexpr int K = Hr<T, D>::K, S = Hr<T, D>::S;
    const unsigned ld = off_n + (unsigned)D * io.row_bytes;
    const d2 nP = bload(io.p, io.lane, ld);
    R[(PH + D) % S] = bload(io.r, io.lane, ld);
    // the LDS stages' rhs: column a (Q = 0) or b of rows n - 2t and n - 2t - 1
    double lr[T], lb[T];
#pragma unroll
    for (int t = K; t < T; ++t) {
        lr[t] = io.lx[((PH - 2 * t + 4 * S) % S) * 128 + Q * 64];
        lb[t] = io.lx[((PH - 2 * t - 1 + 4 * S) % S) * 128 + Q * 64];
    }
    d2 v = m.Pq[0];
    d2 prevM2 = d2{0.0, 0.0};
#pragma unroll
    for (int t = 0; t < T; ++t) {
        d2 Ra, Rb;
        if (t < K) {
            Ra = R[(PH - 2 * t + 4 * S) % S];
            Rb = R[(PH - 2 * t - 1 + 4 * S) % S];
        } else {
            Ra = Q == 0 ? d2{lr[t], 0.0} : d2{0.0, lr[t]};
            Rb = Q == 0 ? d2{lb[t], 0.0} : d2{0.0, lb[t]};
        }
        if (t == T - 1) prevM2 = m.M2[t];
        v = stage<T, Q, MODE, false, P2>(c, t, t > 0, v, r0 - 2 * t, m.A[t], m.M1[t], m.M2[t], Ra,
                                         Rb, m.acc[t]);
    }
    // row n - 2K + 1 leaves the register ring for the LDS one (read next step
    // by stage K); its slot is not one this step's LDS stages read
    {
        constexpr int s = (PH - 2 * K + 1 + 4 * S) % S;
        const d2 w = R[s];
        io.lx[s * 128] = w.x;
        io.lx[s * 128 + 64] = w.y;
    }
    if (MODE == kSteady) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), io.d, io.st_lane,
                                               off_n - st_base, 2);
    } else if (MODE == kSteadyEdge) {  // per column (hrs_step)
        const double vx = v.x, vy = v.y;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vx), io.d, io.st_a,
                                              off_n - st_base, 2);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vy), io.d, io.st_b,
                                              off_n - st_base, 2);
    } else if (MODE == kEdge || MODE == kRowEdge) {
        const int jw = r0 - 2 * T;  // row finished by the last stage (tb_step)
        if (jw >= c.j0 && jw < c.j1) {
            double* drow = io.dp + (long long)jw * io.pitch;
            if (MODE == kRowEdge) {
                if (c.st_a) {
                    hr_stv(drow, v);
                    if (c.gb && jw == 1) hr_stv(drow - io.pitch, v);
                    if (c.gt && jw == c.nj) hr_stv(drow + io.pitch, v);
                }
            } else {
                auto put = [&](double* p, d2 o) {
                    if (c.st_a && c.st_b) {
                        hr_stv(p, o);
                    } else if (c.st_a) {
                        p[0] = o.x;
                    } else if (c.st_b) {
                        p[1] = o.y;
                    }
                };
                put(drow, v);
                if (c.gb && jw == 1) put(drow - io.pitch, d2{c.up_a ? v.x : prevM2.x, c.up_b ? v.y : prevM2.y});
                if (c.gt && jw == c.nj) {
                    const d2 gn = m.M1[T - 1];
                    put(drow + io.pitch, d2{c.up_a ? v.x : gn.x, c.up_b ? v.y : gn.y});
                }
            }
        }
    }
    // the stored row's registers stay live through the next two steps' loads
    // (sor_tb.h steady_step)
    asm volatile("" ::"v"(m.keep[0]));
    m.keep[0] = m.keep[1];
    m.keep[1] = v;
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) m.Pq[k] = m.Pq[k + 1];
    m.Pq[D - 1] = nP;
    __builtin_amdgcn_sched_barrier(0);
}

// Step n of the skewed split-ring march (two independent stage chains per
// step on the split ring): the trailing stages SKH .. T-1 run stream row r0 = rs0 + n
// on m.B, the leading stages 0 .. SKH-1 row r0 + 1 on the streamed row; their
// residual windows sit one row higher (stage<..., SKH>).  Register ring: rows
// n - 2K + 2 .. n + 1 + D; the row the leading register stages read last (n -
// 2K + 2) moves to the LDS ring, which holds rows down to n - 2T + 1.
//
// NW >= 0: step NW of an interior warm-up (kPre, from the stream's first row
// rs0 = rs - 1, rs = j0 - 2T the first row of the block's cone).  Stage t's
// outputs matter from row rs + 2t + 2 on (the cone narrows by two rows per
// iteration), which read its input rows from rs + 2t: a stage must take in
// (A := In) every input row from there.  Its input row is rin = rs + n - 2t
// (leading stages) or rs - 1 + n - 2t (trailing), so it matters from step 4t
// (4t + 1); the stages are skipped before that, less a two-step margin --
// 167 of the 410 stage steps of a T = 10 warm-up.  A skipped stage's rows
// stay zero where the full march held values outside every cone.
template <int T, int SKH>
__host__ __device__ constexpr int hr_warm_start(int t) {
    return t < SKH ? 4 * t - 2 : 4 * t - 1;
}

template <int T, int D, int MODE, int Q, int PH, bool P2, bool LITE = false, int NW = -1>
__device__ __forceinline__ void hrs_step(HrMarch<T, D>& m, d2* R, const Lane& c, const HrIo& io,
                                         int r0, unsigned off_n, unsigned st_base) {
    using G = Hr<T, D, 1>;
    constexpr int K = G::K, S = G::S, SKH = G::SKH;
    const unsigned ld = off_n + (unsigned)(D + 1) * io.row_bytes;
    const d2 nP = bload(io.p, io.lane, ld);
    R[(PH + 1 + D) % S] = bload(io.r, io.lane, ld);
    // LDS stages' rhs: trailing t >= SKH rows n - 2t, n - 2t - 1 (colour Q),
    // leading K <= t < SKH rows n + 1 - 2t, n - 2t (colour 1 - Q)
    double lr[T], lb[T];
#pragma unroll
    for (int t = K; t < T; ++t) {
        const int j = t < SKH ? PH + 1 - 2 * t : PH - 2 * t;
        const int h = t < SKH ? 1 - Q : Q;
        lr[t] = io.lx[((j + 4 * S) % S) * 128 + h * 64];
        lb[t] = io.lx[((j - 1 + 4 * S) % S) * 128 + h * 64];
    }
    auto rr = [&](int t, bool red) -> d2 {  // stage t's rhs row (red: rows rin - 1)
        const int q = t < SKH ? 1 - Q : Q;
        if (t < K) {
            const int j = (t < SKH ? PH + 1 - 2 * t : PH - 2 * t) - (red ? 0 : 1);
            return R[(j + 4 * S) % S];
        }
        const double x = red ? lr[t] : lb[t];
        return q == 0 ? d2{x, 0.0} : d2{0.0, x};
    };
    d2 v = m.Pq[0];
    d2 u = m.B;
    d2 prevM2 = m.M2[T - 1];
    if constexpr (MODE == kSteady || MODE == kSteadyEdge) {
        constexpr bool EM = MODE == kSteadyEdge;
        // LITE: the residual of the stages before the last one only on the
        // chunk's first step (a lower bound of each iteration's sum: the loop
        // test, rb_partsum_kernel, takes it as a certificate or redoes the
        // pass with every cell counted)
        constexpr bool kAll = !LITE || PH == 0;
#pragma unroll
        for (int k = 0; k < SKH; ++k) {
            const int ta = SKH + k, tb = k;
            stage_pair<Q, 1 - Q, P2, EM>(c, u, m.A[ta], m.M1[ta], m.M2[ta], rr(ta, true),
                                         rr(ta, false), m.acc[ta], v, m.A[tb], m.M1[tb],
                                         m.M2[tb], rr(tb, true), rr(tb, false), m.acc[tb],
                                         kAll || ta == T - 1, kAll || tb == T - 1);
        }
        if (T - SKH > SKH)
            u = stage<T, Q, MODE, false, P2, SKH>(c, T - 1, true, u, r0 - 2 * (T - 1),
                                                  m.A[T - 1], m.M1[T - 1], m.M2[T - 1],
                                                  rr(T - 1, true), rr(T - 1, false),
                                                  m.acc[T - 1]);
    } else {
        // (NW: the warm-up's stages before their cone, skipped)
        auto runs = [](int t) { return NW < 0 || NW >= hr_warm_start<T, SKH>(t); };
#pragma unroll
        for (int t = SKH; t < T; ++t) {
            if (!runs(t)) continue;
            if (t == T - 1) prevM2 = m.M2[t];
            u = stage<T, Q, MODE, false, P2, SKH>(c, t, true, u, r0 - 2 * t, m.A[t], m.M1[t],
                                                  m.M2[t], rr(t, true), rr(t, false), m.acc[t]);
        }
#pragma unroll
        for (int t = 0; t < SKH; ++t) {
            if (!runs(t)) continue;
            v = stage<T, 1 - Q, MODE, false, P2, SKH>(c, t, t > 0, v, r0 + 1 - 2 * t, m.A[t],
                                                      m.M1[t], m.M2[t], rr(t, true),
                                                      rr(t, false), m.acc[t]);
        }
    }
    m.B = v;
    {
        constexpr int s = (PH - 2 * K + 2 + 4 * S) % S;
        const d2 w = R[s];
        io.lx[s * 128] = w.x;
        io.lx[s * 128 + 64] = w.y;
    }
    if (MODE == kSteady) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, u), io.d, io.st_lane,
                                               off_n - st_base, 2);
    } else if (MODE == kSteadyEdge) {  // per column: owned cells and the ghost column
        const double ux = u.x, uy = u.y;  // (scalar copies: sor_tb.h steady_step)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, ux), io.d, io.st_a,
                                              off_n - st_base, 2);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, uy), io.d, io.st_b,
                                              off_n - st_base, 2);
    } else if (MODE == kEdge || MODE == kRowEdge) {
        const int jw = r0 - 2 * T;
        if (jw >= c.j0 && jw < c.j1) {
            double* drow = io.dp + (long long)jw * io.pitch;
            if (MODE == kRowEdge) {
                if (c.st_a) {
                    hr_stv(drow, u);
                    if (c.gb && jw == 1) hr_stv(drow - io.pitch, u);
                    if (c.gt && jw == c.nj) hr_stv(drow + io.pitch, u);
                }
            } else {
                auto put = [&](double* p, d2 o) {
                    if (c.st_a && c.st_b) {
                        hr_stv(p, o);
                    } else if (c.st_a) {
                        p[0] = o.x;
                    } else if (c.st_b) {
                        p[1] = o.y;
                    }
                };
                put(drow, u);
                if (c.gb && jw == 1)
                    put(drow - io.pitch, d2{c.up_a ? u.x : prevM2.x, c.up_b ? u.y : prevM2.y});
                if (c.gt && jw == c.nj) {
                    const d2 gn = m.M1[T - 1];
                    put(drow + io.pitch, d2{c.up_a ? u.x : gn.x, c.up_b ? u.y : gn.y});
                }
            }
        }
    }
    asm volatile("" ::"v"(m.keep[0]));
    m.keep[0] = m.keep[1];
    m.keep[1] = u;
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) m.Pq[k] = m.Pq[k + 1];
    m.Pq[D - 1] = nP;
    __builtin_amdgcn_sched_barrier(0);
}

// steps NN of a chunk whose first step has ring phase P0 and colour Q0 (N0 >=
// 0: an interior warm-up chunk from its step N0, hrs_step NW)
template <int T, int D, int SK, int MODE, int Q0, bool P2, int P0 = 0, bool LITE = false,
          int N0 = -1, int... NN>
__device__ __forceinline__ void hr_chunk(HrMarch<T, D>& m, d2* R, const Lane& c, const HrIo& io,
                                         int r0, unsigned off_n, unsigned st_base,
                                         std::integer_sequence<int, NN...>) {
    constexpr int S = Hr<T, D, SK>::S;
    if constexpr (SK)
        (hrs_step<T, D, MODE, Q0 ^ (NN & 1), (P0 + NN) % S, P2, LITE, N0 < 0 ? -1 : N0 + NN>(
             m, R, c, io, r0 + NN, off_n + (unsigned)NN * io.row_bytes, st_base),
         ...);
    else
        (hr_step<T, D, MODE, Q0 ^ (NN & 1), (P0 + NN) % S, P2>(
             m, R, c, io, r0 + NN, off_n + (unsigned)NN * io.row_bytes, st_base),
         ...);
}

// chunks [k0, k1) of a march of colour Q0 (colour of step 0), the first
// starting at step n0 (ring phase n0 mod S = P0)
template <int T, int D, int SK, int MODE, int Q0, bool P2, int P0 = 0, bool LITE = false>
__device__ __forceinline__ void hr_run(HrMarch<T, D>& m, d2* R, const Lane& c, const HrIo& io,
                                       int rs0, int k0, int k1, unsigned st_base, int n0 = 0) {
    constexpr int S = Hr<T, D, SK>::S;
    for (int k = k0; k < k1; ++k) {
        // (the chunk's row offset is a scalar: readfirstlane keeps the compiler
        // from taking it for a per-lane value where the march runs inside the
        // chained loop, hr_chain_steady -- a waterfall loop per buffer access)
        const int n = __builtin_amdgcn_readfirstlane(n0 + (k - k0) * S);
        hr_chunk<T, D, SK, MODE, Q0 ^ (P0 & 1), P2, P0, LITE>(
            m, R, c, io, rs0 + n, __builtin_amdgcn_readfirstlane((unsigned)n * io.row_bytes),
            st_base, std::make_integer_sequence<int, S>{});
    }
}

// the warm-up of a block or chained run: WU steps from the stream's first row
// (KW whole chunks and WR steps, colour Q at step 0).  The interior warm-up
// (kPre, skewed) is unrolled step by step and skips each stage's steps before
// its cone (hrs_step NW); the others march the KW chunks in a loop.
template <int T, int D, int SK, int MODE, int Q, bool P2, int... KK>
__device__ __forceinline__ void hr_warm_chunks(HrMarch<T, D>& m, d2* R, const Lane& c,
                                               const HrIo& io, int rs0, unsigned sb,
                                               std::integer_sequence<int, KK...>) {
    constexpr int S = Hr<T, D, SK>::S;
    (hr_chunk<T, D, SK, MODE, Q, P2, 0, false, KK * S>(
         m, R, c, io, rs0 + KK * S, __builtin_amdgcn_readfirstlane((unsigned)(KK * S) * io.row_bytes),
         sb, std::make_integer_sequence<int, S>{}),
     ...);
}

template <int T, int D, int SK, int MODE, int Q, bool P2>
__device__ __forceinline__ void hr_warm(HrMarch<T, D>& m, d2* R, const Lane& c, const HrIo& io,
                                        int rs0, unsigned sb) {
    using G = Hr<T, D, SK>;
    constexpr int S = G::S, KW = G::WU / S, WR = G::WR;
    constexpr bool kSkip = MODE == kPre && SK != 0;
    if constexpr (kSkip)
        hr_warm_chunks<T, D, SK, MODE, Q, P2>(m, R, c, io, rs0, sb,
                                              std::make_integer_sequence<int, KW>{});
    else
        hr_run<T, D, SK, MODE, Q, P2>(m, R, c, io, rs0, 0, KW, sb);
    if constexpr (WR > 0)
        hr_chunk<T, D, SK, MODE, Q, P2, 0, false, kSkip ? KW * S : -1>(
            m, R, c, io, rs0 + KW * S,
            __builtin_amdgcn_readfirstlane((unsigned)(KW * S) * io.row_bytes), sb,
            std::make_integer_sequence<int, WR>{});
}

// the per-lane constants of the strip whose owned columns start at c_out,
// for block rows [j0, j1) of block row `by` (tb_strip2's lane setup)
template <int T>
__device__ __forceinline__ void hr_lane(const SweepParams& prm, const int c_out, const int j0,
                                        const int j1, const int by, const int lane, Lane& c) {
    const int ni = prm.ni, nj = prm.nj;
    const int c_ld = c_out - 2 * T;
    const int own_end = ni;
    c.ia = c_ld + 2 * lane;
    c.ib = c.ia + 1;
    c.up_a = c.ia >= prm.upd_lo_i && c.ia <= prm.upd_hi_i;
    c.up_b = c.ib >= prm.upd_lo_i && c.ib <= prm.upd_hi_i;
    const bool own_lane = lane >= T && lane < kLanes - T;
    c.own_a = own_lane && c.ia <= own_end;
    c.own_b = own_lane && c.ib <= own_end;
    c.fix0_b = prm.ghost_left && c.ib == 0;
    c.fixr_a = prm.ghost_right && c.ia == ni + 1;
    c.fixr_b = prm.ghost_right && c.ib == ni + 1;
    c.st_a = c.own_a || c.fixr_a;
    c.st_b = c.own_b || c.fix0_b || c.fixr_b;
    c.lo_j = prm.upd_lo_j;
    c.hi_j = prm.upd_hi_j;
    c.j0 = j0;
    c.j1 = j1;
    c.wlo = by == 0 && prm.ghost_bottom;
    c.whi = by == prm.nby - 1 && prm.ghost_top;
    c.parity = prm.parity;
    c.gb = prm.ghost_bottom;
    c.gt = prm.ghost_top;
    c.nj = nj;
    c.idx2 = prm.idx2;
    c.idy2 = prm.idy2;
    c.coef = prm.coef;
    c.bl = ((lane + 63) & 63) * 4;
    c.br = ((lane + 1) & 63) * 4;
}

// columns interior: every column of the cone an updated cell and ownership
// uniform per lane (tb_strip2's cols_in)
template <int T>
__device__ __forceinline__ bool hr_cols_in(const SweepParams& prm, int c_out) {
    constexpr int OW = kStripCells - 4 * T;
    const int c_ld = c_out - 2 * T;
    return c_ld >= prm.upd_lo_i && c_ld + kStripCells - 1 <= prm.upd_hi_i &&
           (c_out + OW - 1 <= prm.ni || (prm.ni & 1) == 0);
}

// wave-uniform buffer descriptor over the strip's 128 columns of `rows` rows
// from row0.  Every input passes through readfirstlane: a descriptor the
// compiler cannot prove uniform (e.g. one rebuilt in a loop, hr_chain_steady)
// gets a waterfall loop around every buffer operation (cdna_hip_programming.md
// T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hr_rsrc(const SweepParams& prm, const double* b,
                                                         int c_ld, int row0, int rows) {
    const long long pitch = prm.pitch;
    const unsigned long long a =
        (unsigned long long)(b + (long long)(kYOff + row0) * pitch + kXOff + c_ld);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)((long long)rows * pitch * 8));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo),
                                             (short)0, bytes, 0x00020000);
}

// one wave's strip (tb_strip2's geometry and lane setup) through the
// split-ring march; lx: the wave's LDS ring
template <int T, int D, bool P2, int SK = 0>
__device__ __forceinline__ void hr_strip(const SweepParams& prm, const double* __restrict__ src,
                                         double* __restrict__ dst, const double* __restrict__ rhs,
                                         const int c_out, const int j0, const int j1, const int by,
                                         const int lane, double (&acc)[T], lds_double* lx) {
    constexpr int S = Hr<T, D, SK>::S, WU = Hr<T, D, SK>::WU;
    const int c_ld = c_out - 2 * T;
    const long long pitch = prm.pitch;
    Lane c;
    hr_lane<T>(prm, c_out, j0, j1, by, lane, c);

    const int rs = j0 - 2 * T;  // first row of the cone
    const int rend = j1 - 1 + 2 * T;
    const bool cols_in = hr_cols_in<T>(prm, c_out);
    const bool rows_in = rs >= prm.upd_lo_j && rend <= prm.upd_hi_j && (j1 - j0) % S == 0 &&
                         j1 - j0 > 0;
    const bool steady = cols_in && rows_in;
    // skewed: the leading stages run one row ahead (they take rows rs0 + 1 ..
    // rend + 1), so every block's stream starts one row early (its leading
    // stages then see row rs first)
    const int rs0 = rs - SK;
    const int nsteps = rend - rs0 + 1;
    const int nchunks = (nsteps + S - 1) / S;

    HrIo io;
    io.p = hr_rsrc(prm, src, c_ld, rs0, nsteps + D + SK);
    io.r = hr_rsrc(prm, rhs, c_ld, rs0 - 1, nsteps + D + SK);
    io.d = hr_rsrc(prm, dst, c_ld, j0, j1 - j0);
    io.lane = (unsigned)lane * 16u;
    io.st_lane = c.own_a ? (unsigned)lane * 16u : 0x40000000u;
    io.row_bytes = (unsigned)(pitch * 8);
    io.lx = lx + lane;
    io.dp = dst + (long long)kYOff * pitch + kXOff + c.ia;
    io.pitch = pitch;

    HrMarch<T, D> m;
    d2 R[S];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        m.acc[t] = 0.0;
        m.A[t] = m.M1[t] = m.M2[t] = d2{0.0, 0.0};
    }
    m.keep[0] = m.keep[1] = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < S; ++k) R[k] = d2{0.0, 0.0};
    m.B = d2{0.0, 0.0};
    // p rows SK .. SK + D - 1 (the leading stages' first), rhs rows 0 .. SK + D - 1
#pragma unroll
    for (int k = 0; k < D; ++k) m.Pq[k] = bload(io.p, io.lane, (unsigned)(k + SK) * io.row_bytes);
#pragma unroll
    for (int k = 0; k < D + SK; ++k) R[k] = bload(io.r, io.lane, (unsigned)k * io.row_bytes);
    const bool q1 = ((c.parity + rs0) & 1) != 0;  // colour of step 0 (S even: of every chunk)
    if (steady) {
        // stores: step n finishes row rs0 + n - 2T = j0 + n - WU; the warm-up:
        // KW whole chunks and WR steps, then H / S steady chunks from phase WR
        const unsigned sb = (unsigned)WU * io.row_bytes;
        constexpr int WR = Hr<T, D, SK>::WR;
        const int nsteady = (j1 - j0) / S;
        auto warm_steady = [&](auto q_c) {
            constexpr int Q = decltype(q_c)::value;
            hr_warm<T, D, SK, kPre, Q, P2>(m, R, c, io, rs0, sb);
            hr_run<T, D, SK, kSteady, Q, P2, WR>(m, R, c, io, rs0, 0, nsteady, sb, WU);
        };
        if (q1) warm_steady(std::integral_constant<int, 1>{});
        else    warm_steady(std::integral_constant<int, 0>{});
    } else if (cols_in) {
        if (q1) hr_run<T, D, SK, kRowEdge, 1, P2>(m, R, c, io, rs0, 0, nchunks, 0);
        else    hr_run<T, D, SK, kRowEdge, 0, P2>(m, R, c, io, rs0, 0, nchunks, 0);
    } else {
        if (q1) hr_run<T, D, SK, kEdge, 1, P2>(m, R, c, io, rs0, 0, nchunks, 0);
        else    hr_run<T, D, SK, kEdge, 0, P2>(m, R, c, io, rs0, 0, nchunks, 0);
    }
    if (cols_in && !c.own_a) {
#pragma unroll
        for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] += m.acc[t];
}

// ---------------------------------------------------------------------------
// Chained split-ring passes (rb_tbhc_kernel): sor_tb.h's chained runs --
// segments of block rows of one column, claimed block by block, work stealing,
// residual partials per wave and block at fixed slots (chain_acquire,
// chain_block_end) -- on the split-ring march.  A run of steady-able blocks
// (a height the ring divides, the cone clear of the physical bottom / top
// sides) warms up once, at its first block (WU steps), and then marches
// kSteady chunks from block to block with its registers and LDS ring live:
// the 4T + 1 warm-up steps an unchained block spends per H rows (7% of a
// 576-row block at T = 10, all of it VALU work the VALU-bound pass pays for)
// are spent once per run.  A strip at a physical left / right side chains the
// same way in kSteadyEdge chunks (the paired stages with lane masks and the
// ghost column copies); the columns with such a strip form the pass's second list
// (sor_tb.h), run by a second launch of the same kernel beside the main one.
// Blocks that are not steady-able are marched one by one from scratch
// (hr_strip).
// ---------------------------------------------------------------------------
template <int T, int D, int SK>
__host__ __device__ inline bool hr_chain_rows_ok(const SweepParams& prm, int j0, int j1) {
    constexpr int S = Hr<T, D, SK>::S;
    return j0 - 2 * T >= prm.upd_lo_j && j1 - 1 + 2 * T <= prm.upd_hi_j && (j1 - j0) % S == 0 &&
           j1 > j0;
}

// a chained run of steady blocks on one wave's strip, from block row by;
// colour Q of the run's first streamed row (the same at every block start: the
// heights are multiples of the even S).  EM: a strip at a physical left /
// right side -- kSteadyEdge chunks after a kEdge warm-up
template <int T, int WAVES, int D, bool P2, int SK, int Q, bool EM, bool LITE = false>
__device__ __forceinline__ void hr_chain_steady(const SweepParams& prm,
                                                const double* __restrict__ src,
                                                double* __restrict__ dst,
                                                const double* __restrict__ rhs,
                                                double* __restrict__ partials, int* sh,
                                                unsigned long long* seg, const int c_out,
                                                const int bx, int by, const int slot,
                                                int own_end, const int lane, lds_double* lx) {
    using G = Hr<T, D, SK>;
    constexpr int S = G::S, WU = G::WU, WR = G::WR;
    const int c_ld = c_out - 2 * T;
    int j0, j1;
    block_rows(prm, by, j0, j1);
    Lane c;
    hr_lane<T>(prm, c_out, j0, j1, by, lane, c);
    HrIo io;
    io.lane = (unsigned)lane * 16u;
    io.st_lane = c.own_a ? (unsigned)lane * 16u : 0x40000000u;
    io.row_bytes = (unsigned)(prm.pitch * 8);
    io.st_a = c.st_a ? (unsigned)lane * 16u : 0x40000000u;
    io.st_b = c.st_b ? (unsigned)lane * 16u + 8u : 0x40000000u;
    io.lx = lx + lane;
    // kEdge stores: dst at row 0 of the lane's columns (kSteady: buffer stores)
    io.dp = dst + (long long)kYOff * prm.pitch + kXOff + c.ia;
    io.pitch = prm.pitch;
    // a strip at a physical side: kEdge warm-up (its row tests keep it from
    // tallying and storing), kSteadyEdge chunks (the paired stages with lane
    // masks and the ghost column copies)
    constexpr int WM = EM ? kEdge : kPre, SM = EM ? kSteadyEdge : kSteady;
    // the descriptors of block [j0, j1): stream rows from rs0 = j0 - 2T - SK
    // (step n streams row rs0 + n; the steady chunks of the block are steps
    // WU .. WU + H - 1, loading up to D + SK rows past them)
    // (plain assignments, no capturing lambda: state a lambda captures by
    // reference can end up in private memory, whose loads are per-lane values
    // to the compiler -- a waterfall loop around every buffer operation)
    int rs0 = j0 - 2 * T - SK;
    io.p = hr_rsrc(prm, src, c_ld, rs0, (j1 - j0) + WU + D + SK);
    io.r = hr_rsrc(prm, rhs, c_ld, rs0 - 1, (j1 - j0) + WU + D + SK);
    io.d = hr_rsrc(prm, dst, c_ld, j0, j1 - j0);
    HrMarch<T, D> m;
    d2 R[S];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        m.acc[t] = 0.0;
        m.A[t] = m.M1[t] = m.M2[t] = d2{0.0, 0.0};
    }
    m.keep[0] = m.keep[1] = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < S; ++k) R[k] = d2{0.0, 0.0};
    m.B = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < D; ++k) m.Pq[k] = bload(io.p, io.lane, (unsigned)(k + SK) * io.row_bytes);
#pragma unroll
    for (int k = 0; k < D + SK; ++k) R[k] = bload(io.r, io.lane, (unsigned)k * io.row_bytes);
    // the warm-up of the run's first block (hr_warm)
    const unsigned sb = (unsigned)WU * io.row_bytes;
    hr_warm<T, D, SK, WM, Q, P2>(m, R, c, io, rs0, sb);
    for (;;) {
        // the block's H / S steady chunks from ring phase WR (step WU stores row j0)
        hr_run<T, D, SK, SM, Q, P2, WR, LITE>(m, R, c, io, rs0, 0, (j1 - j0) / S, sb, WU);
        if (!EM && !c.own_a) {  // lanes that do not own their columns tallied garbage
#pragma unroll
            for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
        }
        // (zeroes m.acc)
        const int nb = chain_block_end<T, WAVES>(prm, m.acc, partials, by * prm.nbx + bx, sh, seg,
                                                 slot, by, own_end);
        if (nb < 0) break;
        // the next block of the run continues the stream: same ring phase
        // (H is a multiple of S), descriptors rebased at its rows
        rs0 = __builtin_amdgcn_readfirstlane(rs0 + (j1 - j0));
        by = nb;
        block_rows(prm, by, j0, j1);
        j0 = __builtin_amdgcn_readfirstlane(j0);
        j1 = __builtin_amdgcn_readfirstlane(j1);
        io.p = hr_rsrc(prm, src, c_ld, rs0, (j1 - j0) + WU + D + SK);
        io.r = hr_rsrc(prm, rhs, c_ld, rs0 - 1, (j1 - j0) + WU + D + SK);
        io.d = hr_rsrc(prm, dst, c_ld, j0, j1 - j0);
    }
    // (the LDS ring is the wave's own; the next run overwrites it from its
    // warm-up on, after its first writes)
}

// one run of a chained split-ring pass: column bx from block row by (all
// waves; sor_tb.h chain_run): runs of steady blocks chained (hr_chain_steady),
// every other block alone (hr_strip); EDGE = 1 (an A/B form): every block
// alone.  Every wave calls chain_block_end at every block end of the run.
template <int T, int WAVES, int D, bool P2, int SK, int EDGE, bool LITE = false>
__device__ __forceinline__ void hr_chain_run(const SweepParams& prm,
                                             const double* __restrict__ src,
                                             double* __restrict__ dst,
                                             const double* __restrict__ rhs,
                                             double* __restrict__ partials, int* sh,
                                             unsigned long long* seg, int bx, int by, int slot,
                                             int own_end, lds_double* lx) {
    constexpr int OW = kStripCells - 4 * T;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c_out = 1 + (bx * WAVES + wave) * OW;
    if (bx == 0 && by == 0) copy_corners(prm, src, dst);
    int j0, j1;
    block_rows(prm, by, j0, j1);
    const bool chained =
        EDGE == 0 && c_out <= prm.ni && hr_chain_rows_ok<T, D, SK>(prm, j0, j1);
    if (chained) {
        // the colour of the run's first streamed row (rs0 = j0 - 2T - SK)
        const bool q1 = ((prm.parity + j0 - 2 * T - SK) & 1) != 0;
        if (hr_cols_in<T>(prm, c_out)) {
            if (q1)
                hr_chain_steady<T, WAVES, D, P2, SK, 1, false, LITE>(prm, src, dst, rhs, partials, sh,
                                                               seg, c_out, bx, by, slot, own_end,
                                                               lane, lx);
            else
                hr_chain_steady<T, WAVES, D, P2, SK, 0, false, LITE>(prm, src, dst, rhs, partials, sh,
                                                               seg, c_out, bx, by, slot, own_end,
                                                               lane, lx);
        } else {
            if (q1)
                hr_chain_steady<T, WAVES, D, P2, SK, 1, true, LITE>(prm, src, dst, rhs, partials, sh,
                                                              seg, c_out, bx, by, slot, own_end,
                                                              lane, lx);
            else
                hr_chain_steady<T, WAVES, D, P2, SK, 0, true, LITE>(prm, src, dst, rhs, partials, sh,
                                                              seg, c_out, bx, by, slot, own_end,
                                                              lane, lx);
        }
        return;
    }
    // block by block from scratch (and the waves with no strip: block ends only)
    for (;;) {
        double acc[T];
#pragma unroll
        for (int t = 0; t < T; ++t) acc[t] = 0.0;
        if (c_out <= prm.ni)
            hr_strip<T, D, P2, SK>(prm, src, dst, rhs, c_out, j0, j1, by, lane, acc, lx);
        by = chain_block_end<T, WAVES>(prm, acc, partials, by * prm.nbx + bx, sh, seg, slot, by,
                                       own_end);
        if (by < 0) return;
        block_rows(prm, by, j0, j1);
    }
}

}  // namespace

// the chained split-ring pass (sor_tb.h rb_tbc_kernel's work area and
// segment lists; EDGE: the kernel of the columns at a physical left / right
// side, launched beside the main one)
template <int T, int WAVES, int D, bool P2, int SK, int EDGE, bool LITE = false>
__global__ __launch_bounds__(kLanes* WAVES, 2) void rb_tbhc_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, int force, int* __restrict__ work) {
    // sh[0..3]: the run (chain_acquire), sh[4..5]: trace clock, sh[6]: run start,
    // sh[7]: own_end of the last claim, sh[8]: unclaimed blocks seen then
    __shared__ __attribute__((aligned(8))) int sh[12];
    constexpr int S = Hr<T, D, SK>::S;
    __shared__ __attribute__((aligned(16))) double ring[WAVES * S * kStripCells];
    if (!force && st->done) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    lds_double* lx = (lds_double*)(ring + wave * S * kStripCells);
    unsigned long long* seg = reinterpret_cast<unsigned long long*>(work + kChainHead);
    // the edge kernel, its own list done: steals from the main list's runs
    // (prm.alt_work), whose work area was initialised before this launch
    bool alt = false;
    for (;;) {
        __syncthreads();  // every wave has read the last claim of the previous run
        if (threadIdx.x < kLanes) {
            if (alt) chain_acquire(prm, prm.alt_work, seg, sh, prm.alt_nseg0);
            else     chain_acquire(prm, work, seg, sh);
        }
        if (prm.trace && threadIdx.x == 0) {
            *reinterpret_cast<volatile unsigned long long*>(sh + 4) = wall_clock64();
            sh[6] = 1;
        }
        __syncthreads();
        const int bx = __builtin_amdgcn_readfirstlane(sh[0]);
        const int by = __builtin_amdgcn_readfirstlane(sh[1]);
        const int slot = __builtin_amdgcn_readfirstlane(sh[2]);
        const int own_end = __builtin_amdgcn_readfirstlane(sh[3]);
        __syncthreads();  // sh is rewritten by the run's block ends
        if (bx < 0) {
            if (alt || prm.alt_work == nullptr) break;
            alt = true;
            seg = reinterpret_cast<unsigned long long*>(prm.alt_work + kChainHead);
            continue;
        }
        hr_chain_run<T, WAVES, D, P2, SK, EDGE, LITE>(prm, src, dst, rhs, partials, sh, seg, bx,
                                                      by, slot, own_end, lx);
    }
}

}  // namespace misor
