// sor_tb.hip -- temporally blocked red-black SOR for gfx950: T complete
// solveRB iterations (assignment-4/src/solver.c:197-229, T = 1..8) per pass
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
//   final rin-3) and the rhs rows it needs come from one ring of the last 2T
//   streamed rows, so rhs is read from HBM once.  The ring lives in registers
//   (8 VGPRs per stage) or -- to keep 3-4 waves per SIMD at T >= 4 -- in a
//   lane-private LDS ring (LDS_RING variants).
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
// Instruction economy (the kernel is VALU-issue-bound once T >= 3):
//  - strips whose 128 columns are all updated cells ("interior" strips: no
//    physical ghost column, no padding) run a path with no per-lane masks,
//    the row colour as a compile-time constant (rows unrolled by two) and the
//    residual accumulated in every lane, non-owned lanes dropped at the end;
//    only strips at a physical left/right side run the masked path;
//  - lane shifts are DPP wave_shr:1 / wave_shl:1 moves, not LDS permutes;
//  - r^2 is accumulated with an FMA (the residual's rounding is not part of
//    the bit-exact contract; p is).
//
// Bit-exactness: same expression order as the reference, -ffp-contract=off.

#include "misor_internal.h"

namespace misor {

namespace {

// Lane shifts by DPP wave_shr:1 / wave_shl:1 (bound_ctrl: the lane shifted in
// from outside the wave reads 0).  Lanes 0 and 63 are never output lanes (the
// T outermost lanes on each side are the strip's halo), so their value is
// irrelevant; no copy of the old value is needed.
// lane l receives lane l-1's value
__device__ __forceinline__ double from_left(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true));
}
// lane l receives lane l+1's value
__device__ __forceinline__ double from_right(double v) {
    return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true),
                            __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// a - 2c as one FMA: 2c is exact in binary floating point, so the single
// rounding of fma(-2, c, a) equals the rounding of the reference's a - 2.0*c
// (bit-exact, one VALU instruction instead of a multiply and a subtract)
__device__ __forceinline__ double m2c(double a, double c) { return __builtin_fma(-2.0, c, a); }

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

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
    bool st_a, st_b;       // columns this lane stores
    int lo_j, hi_j;        // updated rows
    int j0, j1;            // owned rows
    int parity;
    int gb, gt, nj;
    double idx2, idy2, coef;
};

// How a step is compiled:
//  kEdge   general: colour from the row, per-lane update / residual masks,
//          ghost-row and ghost-column copies, row tests.  Blocks whose cone
//          reaches a physical side (first/last strip, first/last block row).
//  kWarm   interior: colour a constant, every streamed row is an updatable
//          row (rows outside the valid cone hold garbage that never reaches a
//          stored value); only the residual (select on the row's ownership)
//          and the store are row-tested.  The 4T+1 warm-up and 2T drain steps.
//  kSteady interior, every row touched is owned: no tests at all.
//  kRowEdge columns interior (every lane's two columns updated, ownership
//          uniform per lane), rows general: the first/last block row at a
//          physical bottom/top side.  Row tests and ghost-row copies are
//          wave-uniform; no lane masks, the residual as in kWarm.
enum { kEdge = 0, kWarm = 1, kSteady = 2, kRowEdge = 3 };

// One iteration stage.  In = row rin of the previous stage's output (stage 1:
// of the field in memory).  Returns row rin-2 of this stage's output.
// fixrows (stages 2..T; a constant after unrolling): complete the previous
// iteration's ghost-row copy on the incoming stream.  Stage 1 reads the ghost
// rows as they are in memory -- the state after the previous pass, or
// whatever the caller uploaded, as the reference's first iteration does.
// Q: colour of the rows (0: column ia is red in row rin-1), -1 = from c.
template <int Q, int MODE>
__device__ __forceinline__ d2 stage(const Lane& c, bool fixrows, d2 In, int rin, d2& A, d2& M1,
                                    d2& M2, d2 Ra, d2 Rb, double& acc) {
    constexpr bool EDGE = MODE == kEdge;                // lane masks
    constexpr bool ROWS = EDGE || MODE == kRowEdge;     // row tests, ghost rows
    if (ROWS && fixrows) {
        if (c.gb && rin == 1) {  // row 0 := row 1 (A holds row 0)
            if (!EDGE || c.up_a) A.x = In.x;
            if (!EDGE || c.up_b) A.y = In.y;
        }
        if (c.gt && rin == c.nj + 1) {  // row nj+1 := row nj (A holds row nj)
            if (!EDGE || c.up_a) In.x = A.x;
            if (!EDGE || c.up_b) In.y = A.y;
        }
    }
    const int rr = rin - 1;  // red row
    const int rb = rin - 2;  // black row
    const int q = Q >= 0 ? Q : ((c.parity + 1 + rr) & 1);
    const double idx2 = c.idx2, idy2 = c.idy2, coef = c.coef;
    // r^2 into the stage's residual if (row, column) is owned
    auto tally = [&](double r, bool own_row, bool own_col) {
        if (MODE == kSteady) {
            acc = __builtin_fma(r, r, acc);
        } else if (MODE == kWarm || MODE == kRowEdge) {
            const double rm = own_row ? r : 0.0;  // uniform select: no branch, NaN-safe
            acc = __builtin_fma(rm, rm, acc);
        } else if (own_row && own_col) {
            acc = __builtin_fma(r, r, acc);
        }
    };

    // red pass on row rr
    d2 Mr = A;
    if (!ROWS || (rr >= c.lo_j && rr <= c.hi_j)) {
        const bool own = (rr >= c.j0) && (rr < c.j1);
        if (q == 0) {
            const double Lf = from_left(A.y);
            const double cc = A.x;
            const double r = Ra.x - ((m2c(A.y, cc) + Lf) * idx2 +
                                     (m2c(In.x, cc) + M1.x) * idy2);
            if (!EDGE || c.up_a) Mr.x = cc - coef * r;
            tally(r, own, c.own_a);
        } else {
            const double Rf = from_right(A.x);
            const double cc = A.y;
            const double r = Ra.y - ((m2c(Rf, cc) + A.x) * idx2 +
                                     (m2c(In.y, cc) + M1.y) * idy2);
            if (!EDGE || c.up_b) Mr.y = cc - coef * r;
            tally(r, own, c.own_b);
        }
    }

    // black pass on row rb (+ the ghost column copy of this finished row)
    d2 F = M1;
    if (!ROWS || (rb >= c.lo_j && rb <= c.hi_j)) {
        const bool own = (rb >= c.j0) && (rb < c.j1);
        if (q == 0) {
            const double Ln = from_left(M1.y);
            const double cc = M1.x;
            const double r = Rb.x - ((m2c(M1.y, cc) + Ln) * idx2 +
                                     (m2c(Mr.x, cc) + M2.x) * idy2);
            if (!EDGE || c.up_a) F.x = cc - coef * r;
            tally(r, own, c.own_a);
        } else {
            const double Rn = from_right(M1.x);
            const double cc = M1.y;
            const double r = Rb.y - ((m2c(Rn, cc) + M1.x) * idx2 +
                                     (m2c(Mr.y, cc) + M2.y) * idy2);
            if (!EDGE || c.up_b) F.y = cc - coef * r;
            tally(r, own, c.own_b);
        }
        if (EDGE) {
            const double f1 = from_right(F.x);  // column ib+1 (lane l+1's ia)
            const double fl = from_left(F.y);   // column ia-1 (lane l-1's ib)
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

// the registers of one wave's march
template <int T, int D, int LR>
struct March {
    d2 A[T], M1[T], M2[T];
    // LR 0: register rhs ring, R[k] = rhs(r0 - 1 - k).  LR 2 (re-read): R[2t] =
    // rhs(r0 - 2t - 1) for stage t >= 1, loaded during the previous step, and
    // R[2t + 1] = rhs(r0 - 2t - 2), stage t's red row of the previous step
    d2 R[LR == 1 ? 1 : 2 * T];
    d2 Pq[D], Rq[D];       // rows in flight: p(r0 .. r0+D-1), rhs(r0-1 .. r0+D-2)
    double acc[T];
};

struct Io {
    const double* sp;
    const double* rp;
    double* dp;
    long long pitch;
    // LDS rhs ring (LDS_RING variants): this lane's element (row slot k,
    // component c) at ring[k * 128 + c * 64].  Lane-private (a lane reads back
    // only what it wrote: no barrier), component-major so each wave access is
    // one contiguous 512-byte ds_*_b64.  Row x lives in slot x mod 2T.
    double* ring;
    // re-read rhs (LR == 2): buffer descriptor whose base is row rlo of this
    // wave's strip (wave-uniform), lane byte offset, row stride in bytes
    __amdgpu_buffer_rsrc_t rrs;
    int lane_off, rlo, row_bytes;
    // steady-state stores (SST variants): the strip's 128 columns of row 0 of
    // dst as a wave-uniform address, and this lane's byte offset in a row, out
    // of range (the store is dropped) on lanes that do not store
    unsigned long long dwave;
    unsigned st_off;
};

// LR >= 2: stages 1 .. K re-read their rhs rows (K = LR - 1, at most T - 1)
template <int T, int LR>
__device__ __forceinline__ constexpr int rr_stages() {
    return LR - 1 < T - 1 ? LR - 1 : T - 1;
}

// slot of row x in a ring of 2T rows (x >= -kYOff - 2T - 1; scalar arithmetic)
template <int T>
__device__ __forceinline__ int ring_slot(int x) {
    return (x + 2 * T * 64) % (2 * T);
}

// one step of the march: stream in old row r0, push it through the T stages,
// store the row the last stage finished (r0 - 2T) if this block owns it
template <int T, int D, int LR, int NT, int Q, int MODE>
__device__ __forceinline__ void tb_step(March<T, D, LR>& m, const Lane& c, const Io& io, int r0) {
    // NT bit 0: non-temporal stores; bit 1: branch-free steady-state stores
    constexpr bool SST = (NT & 2) != 0;
    const long long pitch = io.pitch;
    const d2 nP = ldv(io.sp + (long long)(r0 + D) * pitch);
    const d2 nR = ldv(io.rp + (long long)(r0 - 1 + D) * pitch);
    if (LR == 1) {  // rhs(r0 - 1) joins the LDS ring
        double* w = io.ring + ring_slot<T>(r0 - 1) * 128;
        w[0] = m.Rq[0].x;
        w[64] = m.Rq[0].y;
    } else if (LR == 0) {
#pragma unroll
        for (int k = 2 * T - 1; k > 0; --k) m.R[k] = m.R[k - 1];
        m.R[0] = m.Rq[0];
    }

    d2 v = m.Pq[0];
    d2 Rk = d2{0.0, 0.0};  // LR >= 2: stage K's black rhs row, the ring's next newest
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const d2 prevM2 = m.M2[t];
        d2 Ra, Rb;
        if (LR == 1) {  // only component q of rows r0-2t-1 (red) and r0-2t-2 (black) is used
            const int q = Q >= 0 ? Q : ((c.parity + r0) & 1);
            const double ra = io.ring[ring_slot<T>(r0 - 2 * t - 1) * 128 + q * 64];
            const double rb = io.ring[ring_slot<T>(r0 - 2 * t - 2) * 128 + q * 64];
            Ra = d2{ra, ra};
            Rb = d2{rb, rb};
        } else if (LR == 0) {
            Ra = m.R[2 * t];
            Rb = m.R[2 * t + 1];
        } else {
            Ra = t == 0 ? m.Rq[0] : m.R[2 * t];
            Rb = m.R[2 * t + 1];
        }
        constexpr int K = LR >= 2 ? rr_stages<T, LR>() : 0;
        v = stage<Q, MODE>(c, t > 0, v, r0 - 2 * t, m.A[t], m.M1[t], m.M2[t], Ra, Rb, m.acc[t]);
        if (LR >= 2 && t <= K) {
            // Rb is dead: its register takes next step's red row (loaded from L2:
            // this wave streamed it 2t + D steps ago); rows below the stream
            // start were zeros in the ring and only feed cells outside the cone
            if (t == K) Rk = Rb;
            m.R[2 * t + 1] = Ra;
            if (t > 0) {
                const int row = max(r0 - 2 * t, io.rlo);
                m.R[2 * t] = __builtin_bit_cast(
                    d2, __builtin_amdgcn_raw_buffer_load_b128(
                            io.rrs, io.lane_off, (row - io.rlo) * io.row_bytes, 0));
            }
        }
        if (t == T - 1) {
            const int jw = r0 - 2 * T;  // row finished by the last stage
            if (MODE == kSteady && SST) {
                // no branch around the store: the two steps of a colour pair stay one
                // basic block, which the scheduler can interleave
                const unsigned long long a = io.dwave + (unsigned long long)jw * (pitch * 8);
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    (void*)a, (short)0, kStripCells * 8, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rs, io.st_off,
                                                       0, (NT & 1) ? 2 : 0);
            } else if (MODE == kSteady) {
                if (c.st_a) stv<(NT & 1) != 0>(io.dp + (long long)jw * pitch, v);
            } else if (MODE == kWarm) {
                if (jw >= c.j0 && jw < c.j1 && c.st_a) stv<(NT & 1) != 0>(io.dp + (long long)jw * pitch, v);
            } else if (MODE == kRowEdge) {
                // every column of the lane updated and stored alike (st_a == st_b);
                // ghost rows 0 / nj+1 of the stored field are copies of rows 1 / nj
                if (jw >= c.j0 && jw < c.j1 && c.st_a) {
                    double* drow = io.dp + (long long)jw * pitch;
                    stv<(NT & 1) != 0>(drow, v);
                    if (c.gb && jw == 1) stv<(NT & 1) != 0>(drow - pitch, v);
                    if (c.gt && jw == c.nj) stv<(NT & 1) != 0>(drow + pitch, v);
                }
            } else if (jw >= c.j0 && jw < c.j1) {
                double* drow = io.dp + (long long)jw * pitch;
                auto put = [&](double* p, d2 o) {
                    if (c.st_a && c.st_b) {
                        stv<(NT & 1) != 0>(p, o);
                    } else if (c.st_a) {
                        p[0] = o.x;
                    } else if (c.st_b) {
                        p[1] = o.y;
                    }
                };
                put(drow, v);
                // ghost rows of the stored field: interior columns from the
                // finished row, corners from the (unchanged) ghost row
                if (c.gb && jw == 1) {
                    const d2 g0 = prevM2;  // the stage's row 0
                    put(drow - pitch, d2{c.up_a ? v.x : g0.x, c.up_b ? v.y : g0.y});
                }
                if (c.gt && jw == c.nj) {
                    const d2 gn = m.M1[t];  // the stage's row nj+1 (after its fix)
                    put(drow + pitch, d2{c.up_a ? v.x : gn.x, c.up_b ? v.y : gn.y});
                }
            }
        }
    }
    if (LR >= 2) {
        // stages K+1 .. T-1 keep the register ring, R[k] = rhs(r0 - 1 - k) for
        // k >= 2K + 2 (shifted after every stage has read it)
        constexpr int K = rr_stages<T, LR>();
#pragma unroll
        for (int k = 2 * T - 1; k > 2 * K + 2; --k) m.R[k] = m.R[k - 1];
        if (K < T - 1) m.R[2 * K + 2] = Rk;
    }
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) {
        m.Pq[k] = m.Pq[k + 1];
        m.Rq[k] = m.Rq[k + 1];
    }
    m.Pq[D - 1] = nP;
    m.Rq[D - 1] = nR;
}

// Interior blocks: the colour alternates by row, so steps go in pairs with
// the colour a constant (Q0 = colour of row r0).  Steps r0 in
// [j0+2T+1, j1-1] touch only owned rows and store unconditionally (kSteady);
// the 4T+1 warm-up steps before and the 2T drain steps after are kWarm.
template <int T, int D, int LR, int NT, int Q0>
__device__ __forceinline__ void march_interior_q(March<T, D, LR>& m, const Lane& c,
                                                 const Io& io, int r0, int rend) {
    const int sbeg = c.j0 + 2 * T + 1, send = c.j1 - 1;
    // warm-up, in pairs (keeps the colour phase); may run into the steady range
    for (; r0 + 1 < sbeg && r0 + 1 <= rend; r0 += 2) {
        tb_step<T, D, LR, NT, Q0, kWarm>(m, c, io, r0);
        tb_step<T, D, LR, NT, 1 - Q0, kWarm>(m, c, io, r0 + 1);
    }
    for (; r0 + 1 <= send; r0 += 2) {
        tb_step<T, D, LR, NT, Q0, kSteady>(m, c, io, r0);
        tb_step<T, D, LR, NT, 1 - Q0, kSteady>(m, c, io, r0 + 1);
    }
    for (; r0 + 1 <= rend; r0 += 2) {
        tb_step<T, D, LR, NT, Q0, kWarm>(m, c, io, r0);
        tb_step<T, D, LR, NT, 1 - Q0, kWarm>(m, c, io, r0 + 1);
    }
    if (r0 <= rend) tb_step<T, D, LR, NT, Q0, kWarm>(m, c, io, r0);
}

// Blocks with a physical side in their cone (kEdge / kRowEdge): every step
// general, but still in colour pairs so the colour is a compile-time constant.
template <int T, int D, int LR, int NT, int Q0, int MODE>
__device__ __forceinline__ void march_edge_q(March<T, D, LR>& m, const Lane& c, const Io& io,
                                             int r0, int rend) {
    for (; r0 + 1 <= rend; r0 += 2) {
        tb_step<T, D, LR, NT, Q0, MODE>(m, c, io, r0);
        tb_step<T, D, LR, NT, 1 - Q0, MODE>(m, c, io, r0 + 1);
    }
    if (r0 <= rend) tb_step<T, D, LR, NT, Q0, MODE>(m, c, io, r0);
}

template <int T, int D, int LR, int NT, int MODE>
__device__ __forceinline__ void march_edge(March<T, D, LR>& m, const Lane& c, const Io& io,
                                           int rs, int rend) {
    if (((c.parity + rs) & 1) == 0)
        march_edge_q<T, D, LR, NT, 0, MODE>(m, c, io, rs, rend);
    else
        march_edge_q<T, D, LR, NT, 1, MODE>(m, c, io, rs, rend);
}

template <int T, int D, int LR, int NT>
__device__ __forceinline__ void march_interior(March<T, D, LR>& m, const Lane& c, const Io& io,
                                               int rs, int rend) {
    if (((c.parity + rs) & 1) == 0)
        march_interior_q<T, D, LR, NT, 0>(m, c, io, rs, rend);
    else
        march_interior_q<T, D, LR, NT, 1>(m, c, io, rs, rend);
}

}  // namespace

template <int T, int WAVES, int D, int LR, int MINW, int NT>
__global__ __launch_bounds__(kLanes* WAVES, MINW) void rb_tb_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, int force) {
    constexpr int OW = kStripCells - 4 * T;
    __shared__ double wsum[T][WAVES];
    __shared__ double ring[LR == 1 ? WAVES : 1][LR == 1 ? 2 * T * kStripCells : 1];
    if (!force && st->done) return;

    int L = blockIdx.x;
    if (prm.xcd_remap) {
        const int nwg = prm.nblocks, qq = nwg / 8, rr = nwg % 8, x = L % 8;
        L = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + L / 8;
    }
    const int bx = L % prm.nbx, by = L / prm.nbx;
    const int ni = prm.ni, nj = prm.nj;
    const int j0 = 1 + (int)(((long long)by * nj) / prm.nby);
    const int j1 = 1 + (int)(((long long)(by + 1) * nj) / prm.nby);
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
    const int c_ld = c_out - 2 * T;
    const long long pitch = prm.pitch;

    Lane c;
    c.ia = c_ld + 2 * lane;
    c.ib = c.ia + 1;
    c.up_a = c.ia >= prm.upd_lo_i && c.ia <= prm.upd_hi_i;
    c.up_b = c.ib >= prm.upd_lo_i && c.ib <= prm.upd_hi_i;
    const bool own_lane = lane >= T && lane < kLanes - T;
    c.own_a = own_lane && c.ia <= ni;
    c.own_b = own_lane && c.ib <= ni;
    c.fix0_b = prm.ghost_left && c.ib == 0;
    c.fixr_a = prm.ghost_right && c.ia == ni + 1;
    c.fixr_b = prm.ghost_right && c.ib == ni + 1;
    // columns this lane stores: owned interior + the physical ghost columns
    c.st_a = c.own_a || c.fixr_a;
    c.st_b = c.own_b || c.fix0_b || c.fixr_b;
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

    March<T, D, LR> m;
#pragma unroll
    for (int t = 0; t < T; ++t) m.acc[t] = 0.0;

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
        Io io{src + base, rhs + base, dst + base, pitch,
              LR == 1 ? &ring[LR == 1 ? wave : 0][LR == 1 ? lane : 0] : nullptr};
        const int rs = j0 - 2 * T;  // first streamed row
        const int rend = j1 - 1 + 2 * T;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            m.Pq[k] = ldv(io.sp + (long long)(rs + k) * pitch);
            m.Rq[k] = ldv(io.rp + (long long)(rs - 1 + k) * pitch);
        }
#pragma unroll
        for (int t = 0; t < T; ++t) m.A[t] = m.M1[t] = m.M2[t] = d2{0.0, 0.0};
        if (NT & 2) {
            const unsigned long long a =
                (unsigned long long)(dst + (long long)kYOff * pitch + kXOff + c_ld);
            const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
            const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
            io.dwave = ((unsigned long long)hi << 32) | lo;
            io.st_off = c.st_a ? (unsigned)lane * 16u : 0x80000000u;
        }
        if (LR >= 2) {
            // wave-uniform descriptor over rows rs-1 .. rend of the strip's
            // 128 columns (the base is made scalar explicitly)
            io.rlo = rs - 1;
            io.row_bytes = (int)(pitch * 8);
            io.lane_off = lane * 16;
            const long long off = ((long long)(kYOff + rs - 1) * pitch + kXOff + c_ld) * 8;
            const unsigned long long a = (unsigned long long)(const char*)rhs + off;
            const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
            const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
            const int nrec = (rend - rs + 2) * io.row_bytes;
            io.rrs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(((unsigned long long)hi << 32) | lo), (short)0, nrec, 0x00020000);
        }
        if (LR == 1) {
#pragma unroll
            for (int k = 0; k < 4 * T; ++k) io.ring[k * 64] = 0.0;
        } else {
#pragma unroll
            for (int k = 0; k < 2 * T; ++k) m.R[k] = d2{0.0, 0.0};
        }

        // columns interior: every column of the cone an updated cell (no lane
        // masks, no ghost columns) and ownership uniform per lane -- the strip
        // is whole, or it runs past column ni into a neighbour's halo (or the
        // padding beyond it) with ni even, so ni | ni+1 falls between lanes;
        // those lanes are neither stored nor counted.  Rows interior: no
        // ghost rows in the cone.
        const bool cols_in = c_ld >= prm.upd_lo_i && c_ld + kStripCells - 1 <= prm.upd_hi_i &&
                             (c_out + OW - 1 <= ni || (ni & 1) == 0);
        const bool rows_in = rs >= prm.upd_lo_j && rend <= prm.upd_hi_j;
        if (!cols_in) {
            march_edge<T, D, LR, NT, kEdge>(m, c, io, rs, rend);
        } else {
            if (rows_in)
                march_interior<T, D, LR, NT>(m, c, io, rs, rend);
            else
                march_edge<T, D, LR, NT, kRowEdge>(m, c, io, rs, rend);
            if (!c.own_a) {
#pragma unroll
                for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
            }
        }
    }

    // deterministic reduction per stage: lane tree, then waves in order
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const double s = wave_sum(m.acc[t]);
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

int tb_nbx(int ni, int T, int waves) {
    const int ow = tb_out_width(T);
    const int strips = (ni + ow - 1) / ow;
    return (strips + waves - 1) / waves;
}

void launch_tb(hipStream_t s, int T, const SweepParams& prm, const double* src, double* dst,
               const double* rhs, double* partials, const DevState* st, int force) {
#define TB(TT, W, DD, LR, MW)                                                  \
    hipLaunchKernelGGL((rb_tb_kernel<TT, W, DD, LR, MW, true>), dim3(prm.nblocks), \
                       dim3(kLanes * W), 0, s, prm, src, dst, rhs, partials, st, force)
#define TBN(TT, W, DD, LR, MW, NTF)                                           \
    hipLaunchKernelGGL((rb_tb_kernel<TT, W, DD, LR, MW, NTF>), dim3(prm.nblocks), \
                       dim3(kLanes * W), 0, s, prm, src, dst, rhs, partials, st, force)
#define TB_T(TT)                              \
    switch (prm.variant) {                    \
    case 0: TB(TT, 4, 2, false, 1); break;    \
    case 1: TB(TT, 8, 2, false, 1); break;    \
    case 2: TB(TT, 4, 3, false, 1); break;    \
    case 3: TB(TT, 4, 2, true, 1); break;     \
    case 4: TB(TT, 4, 2, true, (TT <= 4 ? 4 : 1)); break; \
    case 5: TB(TT, 4, 3, true, 1); break;     \
    case 6: TB(TT, 8, 2, true, 1); break;     \
    case 7: TB(TT, 6, 2, true, 1); break;     \
    case 8: TB(TT, 2, 3, false, 1); break;    \
    case 9: TB(TT, 1, 3, false, 1); break;    \
    case 14: TBN(TT, 4, 3, 0, 1, 3); break;   \
    case 10: TB(TT, 4, 3, 8, 1); break;       \
    case 11: TB(TT, 4, 3, 2, 1); break;       \
    case 12: TB(TT, 4, 3, 3, 1); break;       \
    default: TB(TT, 4, 3, 4, 1); break;       \
    }
    // must match kTbVariants (misor_internal.h)
    switch (T) {
    case 1: TB_T(1); break;
    case 2: TB_T(2); break;
    case 3: TB_T(3); break;
    case 4: TB_T(4); break;
    case 5: TB_T(5); break;
    case 6: TB_T(6); break;
    case 7: TB_T(7); break;
    default: TB_T(8); break;
    }
#undef TB_T
#undef TBN
#undef TB
}

}  // namespace misor
