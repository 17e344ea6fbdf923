// sor_tb.h -- device code of the temporally blocked sweep (included by the
// per-T instantiation units sor_tb_inst.hip; launchers in sor_tb.hip).
#pragma once
// sor_tb.hip -- temporally blocked red-black SOR for gfx950: T complete
// solveRB iterations (assignment-4/src/solver.c:197-229, T = 2..kMaxT) per
// pass over HBM.
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
//          j0-2T .. j1-1+2T upward (N = H + 4T steps).  Stage t receives the
//          output row stream of stage t-1 (stage 0: the old field) and, on
//          receiving row rin, updates the red cells of row rin-1 and the black
//          cells of row rin-2, emitting row rin-2 of iteration t+1.  The last
//          stage's rows j0 .. j1-1 are stored.
//   Every stage keeps 3 rows (A = row rin-1, M1 = rin-2 half updated, M2 =
//   final rin-3); the rhs rows come from one register ring of the last 2T
//   streamed rows (+ the D rows in flight), so rhs is read from HBM once.
//
// The static ring.  Every block of interior rows is H = a multiple of the
// ring's S = 2T + D (+1 if odd) slots tall.  Its march starts with 4T
// "warm-up" steps (no residual, no store; the ring shifts one register per
// step, in pairs of steps) and then runs the remaining H steps in chunks of S
// steps fully unrolled, with rhs row x in ring slot (x - rs + 1) mod S: every
// ring register keeps its row for its whole life and the loads land in the
// slot of the row that just died, so the steady march has no register moves
// for the ring (the round-1 kernel spent 36 64-bit moves per step on it).
// Stores go through a buffer descriptor with an out-of-range offset on lanes
// that do not store, so a chunk is one basic block.
//
// Residual windows.  The residual of stage t is tallied over red rows
// [j0 + 2T-1-2t, j1 + 2T-1-2t) and black rows [j0 + 2T-2-2t, j1 + 2T-2-2t)
// of the block (shifted by the same amount in every block, so every cell is
// counted exactly once per iteration; blocks on a physical bottom / top side
// extend theirs to row 1 / nj).  In step numbers both windows are [4T, N) for
// every stage: the steady chunks tally and store on every step, the warm-up
// steps never do, and no drain steps exist.  Every row in a window lies inside
// the stage's valid cone (red rows [rs+2t+1, rend-2t-1], black [rs+2t+2,
// rend-2t-2]).
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
//   Blocks whose cone reaches a physical side, and the last block row when
//   its height is not a multiple of S, march in pairs of steps with run-time
//   row tests (kRowEdge) and, at a physical left/right side, lane masks
//   (kEdge).
//
// Residual: stage t accumulates r^2 of the cells this wave counts; partial per
// workgroup per stage in a fixed order; the finish kernel decides iteration by
// iteration exactly like the single-sweep path.  If convergence (or itermax)
// is reached at stage t < T, the host recomputes that pass with T' = t from
// the untouched source buffer (misor_api.hip), so the returned field is the
// one after exactly `it` iterations.
//
// Bit-exactness: same expression order as the reference, -ffp-contract=off.

#include <algorithm>
#include <utility>

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

// the same shifts through the LDS crossbar (ds_bpermute: an LDS-pipe
// instruction, so the shift costs no VALU issue slot); addr = source lane * 4
__device__ __forceinline__ double bperm(double v, int addr) {
    return __hiloint2double(__builtin_amdgcn_ds_bpermute(addr, __double2hiint(v)),
                            __builtin_amdgcn_ds_bpermute(addr, __double2loint(v)));
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

// The reference's r = rhs - (a*idx2 + b*idy2) (a, b: the x and y second
// differences), rounded exactly as written.  P2: idx2 == idy2 == k = 2^m,
// m >= 0 (a power-of-two spacing, e.g. every 2^n x 2^n grid on the unit
// square): a*k and b*k are then exact, so fl(fl(a k) + fl(b k)) = fl(a + b) k
// (a subnormal a + b is exact too) and rhs minus that exact product is one
// fma -- the same bits with 2 of the 11 FP64 instructions of an update fewer.
// Holds while |a| k and |b| k stay below DBL_MAX (|p| < ~1e298 at k = 2^30);
// the host enables it only for such a spacing (misor_api.hip configure_tb).
template <bool P2>
__device__ __forceinline__ double resid(double rhs, double a, double b, double idx2, double idy2) {
    if (P2) return __builtin_fma(-(a + b), idx2, rhs);
    return rhs - (a * idx2 + b * idy2);
}

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2 ldv(const double* p) { return *reinterpret_cast<const d2*>(p); }

__device__ __forceinline__ void stv(double* p, d2 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p));
}

// ring slots of the steady march: 2T rows in use + D in flight (+ SK: one
// more in the skewed march, whose trailing stages read a row one step longer),
// even (the colour of a chunk's first step is then the same for every chunk)
template <int T, int D, int SK = 0>
__host__ __device__ constexpr int ring_slots() {
    return 2 * T + D + SK + ((D + SK) & 1);
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
    int j0, j1;            // owned (stored) rows
    int wlo, whi;          // residual window reaches the physical bottom / top side
    int parity;
    int gb, gt, nj;
    int bl, br;            // ds_bpermute addresses of lanes l-1 and l+1
    double idx2, idy2, coef;
};

// The per-lane residual accumulator.  MISOR_RES_BINNED (a cost experiment,
// never the product build: tools/gpu_res_cost.sh) makes
// the steady chunks deposit r^2 into two fixed bins instead (q1 = (M1 + x) -
// M1, q2 = (M2 + (x - q1)) - M2, each added exactly): an order-independent
// sum, i.e. what a partition-independent residual costs in the sweep.
#ifdef MISOR_RES_BINNED
struct TallyAcc {
    double s1, s2;
    __device__ TallyAcc& operator=(double v) {
        s1 = v;
        s2 = 0.0;
        return *this;
    }
    __device__ operator double() const { return s1 + s2; }
};
__device__ __forceinline__ void tally_steady(TallyAcc& a, double r) {
    constexpr double M1 = 0x1.8p+40, M2 = 0x1.8p-12;  // bins of 2^-12 and 2^-64
    const double x = r * r;
    const double q1 = (M1 + x) - M1;
    const double q2 = (M2 + (x - q1)) - M2;
    a.s1 += q1;
    a.s2 += q2;
}
#else
using TallyAcc = double;
__device__ __forceinline__ void tally_steady(double& a, double r) { a = __builtin_fma(r, r, a); }
#endif

// How a step is compiled:
//  kEdge    general: per-lane update / residual masks, ghost-row and
//           ghost-column copies, row tests.  Strips at a physical left /
//           right side.
//  kPre     interior warm-up: every streamed row is an updatable row (rows
//           outside the valid cone hold garbage that never reaches a stored
//           value); no residual, no store.
//  kSteady  interior, static ring: residual and store on every step.
//  kRowEdge columns interior (every lane's two columns updated, ownership
//           uniform per lane), rows general: blocks whose cone reaches a
//           physical bottom / top side, and a last block row whose height is
//           not a multiple of the ring.  Row tests and ghost-row copies are
//           wave-uniform; no lane masks.
//  kSteadyEdge rows interior, static ring (as kSteady), columns general:
//           the lane masks and ghost-column copies of kEdge, no row tests.
//           Strips at a physical left / right side in chained runs.
enum { kEdge = 0, kPre = 1, kSteady = 2, kRowEdge = 3, kSteadyEdge = 4 };

// One iteration stage (stage index t, 0-based).  In = row rin of the previous
// stage's output (stage 0: of the field in memory).  Returns row rin-2 of this
// stage's output.  fixrows (stages 1..T-1; a constant after unrolling):
// complete the previous iteration's ghost-row copy on the incoming stream.
// Stage 0 reads the ghost rows as they are in memory -- the state after the
// previous pass, or whatever the caller uploaded, as the reference's first
// iteration does.  Q: colour of the rows (0: column ia is red in row rin-1).
template <int T, int Q, int MODE, bool BP = false, bool P2 = false, int SKH = 0, class Acc>
__device__ __forceinline__ d2 stage(const Lane& c, int t, bool fixrows, d2 In, int rin, d2& A,
                                    d2& M1, d2& M2, d2 Ra, d2 Rb, Acc& acc) {
    // BP: x-neighbours through ds_bpermute instead of DPP (interior modes)
    auto fl = [&](double v) { return BP ? bperm(v, c.bl) : from_left(v); };
    auto fr = [&](double v) { return BP ? bperm(v, c.br) : from_right(v); };
    constexpr bool EDGE = MODE == kEdge || MODE == kSteadyEdge;  // lane masks
    constexpr bool ROWS = MODE == kEdge || MODE == kRowEdge;     // row tests, ghost rows
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
    const double idx2 = c.idx2, idy2 = c.idy2, coef = c.coef;
    // residual windows of this stage (header): red rows [j0 + sh, j1 + sh),
    // black rows one lower, extended to the physical sides; in a skewed pass
    // (SKH > 0, sor_tbh.h hrs_step) the leading stages t < SKH one row higher
    const int sh = 2 * T - 1 - 2 * t + (t < SKH ? 1 : 0);
    auto tally = [&](double r, int row, int wsh, bool own_col) {
        if (MODE == kSteady) {
            tally_steady(acc, r);
        } else if (MODE == kSteadyEdge) {
            const double rm = own_col ? r : 0.0;  // select: no branch, NaN-safe
            acc = __builtin_fma(rm, rm, acc);
        } else if (MODE == kPre) {
        } else {
            const bool own_row = row >= (c.wlo ? 1 : c.j0 + wsh) &&
                                 row < (c.whi ? c.nj + 1 : c.j1 + wsh);
            if (!EDGE) {
                const double rm = own_row ? r : 0.0;  // uniform select: no branch, NaN-safe
                acc = __builtin_fma(rm, rm, acc);
            } else if (own_row && own_col) {
                acc = __builtin_fma(r, r, acc);
            }
        }
    };

    // red pass on row rr
    d2 Mr = A;
    if (!ROWS || (rr >= c.lo_j && rr <= c.hi_j)) {
        if (Q == 0) {
            const double Lf = fl(A.y);
            const double cc = A.x;
            const double r = resid<P2>(Ra.x, m2c(A.y, cc) + Lf, m2c(In.x, cc) + M1.x, idx2, idy2);
            if (!EDGE || c.up_a) Mr.x = cc - coef * r;
            tally(r, rr, sh, c.own_a);
        } else {
            const double Rf = fr(A.x);
            const double cc = A.y;
            const double r = resid<P2>(Ra.y, m2c(Rf, cc) + A.x, m2c(In.y, cc) + M1.y, idx2, idy2);
            if (!EDGE || c.up_b) Mr.y = cc - coef * r;
            tally(r, rr, sh, c.own_b);
        }
    }

    // black pass on row rb (+ the ghost column copy of this finished row)
    d2 F = M1;
    if (!ROWS || (rb >= c.lo_j && rb <= c.hi_j)) {
        if (Q == 0) {
            const double Ln = fl(M1.y);
            const double cc = M1.x;
            const double r = resid<P2>(Rb.x, m2c(M1.y, cc) + Ln, m2c(Mr.x, cc) + M2.x, idx2, idy2);
            if (!EDGE || c.up_a) F.x = cc - coef * r;
            tally(r, rb, sh - 1, c.own_a);
        } else {
            const double Rn = fr(M1.x);
            const double cc = M1.y;
            const double r = resid<P2>(Rb.y, m2c(Rn, cc) + M1.x, m2c(Mr.y, cc) + M2.y, idx2, idy2);
            if (!EDGE || c.up_b) F.y = cc - coef * r;
            tally(r, rb, sh - 1, c.own_b);
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
template <int T, int D>
struct March {
    d2 A[T], M1[T], M2[T];
    d2 R[2 * T];     // paired march: R[k] = rhs(r0 - 1 - k)
    d2 Pq[D], Rq[D];  // rows in flight: p(r0 .. r0+D-1), rhs(r0-1 .. r0+D-2)
    TallyAcc acc[T];
    d2 keep[2];
};

struct Io {
    const double* sp;
    const double* rp;
    double* dp;
    long long pitch;
};

// one paired-march step: stream in old row r0, push it through the T stages,
// store the row the last stage finished (r0 - 2T) if this block owns it
template <int T, int D, int Q, int MODE, bool BP = false, bool P2 = false>
__device__ __forceinline__ void tb_step(March<T, D>& m, const Lane& c, const Io& io, int r0) {
    const long long pitch = io.pitch;
    const d2 nP = ldv(io.sp + (long long)(r0 + D) * pitch);
    const d2 nR = ldv(io.rp + (long long)(r0 - 1 + D) * pitch);
#pragma unroll
    for (int k = 2 * T - 1; k > 0; --k) m.R[k] = m.R[k - 1];
    m.R[0] = m.Rq[0];

    d2 v = m.Pq[0];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const d2 prevM2 = m.M2[t];
        v = stage<T, Q, MODE, BP, P2>(c, t, t > 0, v, r0 - 2 * t, m.A[t], m.M1[t], m.M2[t],
                                      m.R[2 * t], m.R[2 * t + 1], m.acc[t]);
        if (t == T - 1 && MODE != kPre) {
            const int jw = r0 - 2 * T;  // row finished by the last stage
            if (MODE == kRowEdge) {
                // every column of the lane updated and stored alike (st_a == st_b);
                // ghost rows 0 / nj+1 of the stored field are copies of rows 1 / nj
                if (jw >= c.j0 && jw < c.j1 && c.st_a) {
                    double* drow = io.dp + (long long)jw * pitch;
                    stv(drow, v);
                    if (c.gb && jw == 1) stv(drow - pitch, v);
                    if (c.gt && jw == c.nj) stv(drow + pitch, v);
                }
            } else if (jw >= c.j0 && jw < c.j1) {
                double* drow = io.dp + (long long)jw * pitch;
                auto put = [&](double* p, d2 o) {
                    if (c.st_a && c.st_b) {
                        stv(p, o);
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
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) {
        m.Pq[k] = m.Pq[k + 1];
        m.Rq[k] = m.Rq[k + 1];
    }
    m.Pq[D - 1] = nP;
    m.Rq[D - 1] = nR;
}

// paired march over steps r0 = rs .. rend (the colour Q0 of row rs a constant)
template <int T, int D, int Q0, int MODE, bool BP = false, bool P2 = false>
__device__ __forceinline__ void march_pairs(March<T, D>& m, const Lane& c, const Io& io, int r0,
                                            int rend) {
    for (; r0 + 1 <= rend; r0 += 2) {
        tb_step<T, D, Q0, MODE, BP, P2>(m, c, io, r0);
        tb_step<T, D, 1 - Q0, MODE, BP, P2>(m, c, io, r0 + 1);
    }
    if (r0 <= rend) tb_step<T, D, Q0, MODE, BP, P2>(m, c, io, r0);
}

// Steady march: buffer descriptors over the wave's strip (wave-uniform base,
// lane byte offset); the byte offset of a row is a scalar
typedef __attribute__((address_space(3))) double lds_double;

struct Sio {
    __amdgpu_buffer_rsrc_t p, r, d;  // p rows from rs, rhs rows from rs-1, dst rows from j0
    unsigned lane;                   // lane * 16
    unsigned st_lane;                // lane * 16 if the lane stores, else out of range
    unsigned st_a, st_b;             // kSteadyEdge: per column (lane * 16 (+ 8) or out of range)
    unsigned row_bytes;              // pitch * 8
};

__device__ __forceinline__ d2 bload(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
    return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

// one step of the steady march: stream row r0 = rs + n, tally and store.  PH
// = n mod S (a constant): rhs row rs - 1 + j lives in ring slot j mod S, and
// stage t reads rows j = n - 2t (red) and n - 2t - 1 (black)
template <int T, int D, int Q, int PH, bool BP, bool P2, bool EM = false>
__device__ __forceinline__ void steady_step(March<T, D>& m, d2* R, const Lane& c, const Sio& io,
                                            int r0, unsigned off_n) {
    constexpr int S = ring_slots<T, D>();
    // p row r0 + D (p descriptor starts at row rs), rhs row r0 - 1 + D (rhs
    // descriptor starts at row rs - 1): both n + D rows in; the rhs row lands
    // in the slot of the row stage T-1 finished with in the previous step
    const unsigned ld = off_n + (unsigned)D * io.row_bytes;
    const d2 nP = bload(io.p, io.lane, ld);
    R[(PH + D) % S] = bload(io.r, io.lane, ld);
    d2 v = m.Pq[0];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        v = stage<T, Q, EM ? kSteadyEdge : kSteady, BP, P2>(
            c, t, t > 0, v, r0 - 2 * t, m.A[t], m.M1[t], m.M2[t], R[(PH - 2 * t + 4 * S) % S],
            R[(PH - 2 * t - 1 + 4 * S) % S], m.acc[t]);
    }
    // row r0 - 2T = j0 + (n - 4T): dst descriptor starts at row j0; lanes that
    // do not store carry an out-of-range offset (the write is dropped)
    if (EM) {  // per column: owned cells and the physical ghost column
        // (through scalar copies: clang's __builtin_bit_cast of a vector
        // element lvalue, bit_cast(v2u, v.y), reads element 0 -- both stores
        // then wrote v.x)
        const double vx = v.x, vy = v.y;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vx), io.d, io.st_a,
                                              off_n - 4u * T * io.row_bytes, 2);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, vy), io.d, io.st_b,
                                              off_n - 4u * T * io.row_bytes, 2);
    } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), io.d, io.st_lane,
                                               off_n - 4u * T * io.row_bytes, 2);
    }
    // The store reads its data VGPRs after it issues, and on gfx950 a later
    // buffer_load can land in those VGPRs first: with the registers of step
    // n's row reused by a load a few instructions after the store, lanes 12-15
    // of every 16 stored the loaded rhs instead (tools/debug_tb.py).
    // The compiler does not guard this, so the row stays live through the
    // next two steps' loads (one step already suffices in every test).
    asm volatile("" ::"v"(m.keep[0]));
    m.keep[0] = m.keep[1];
    m.keep[1] = v;
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) m.Pq[k] = m.Pq[k + 1];
    m.Pq[D - 1] = nP;
    // steps are scheduled one at a time (one basic block per chunk, but no
    // code motion across steps: measured faster, 0.856 vs 0.867 ms/iteration)
    __builtin_amdgcn_sched_barrier(0);
}

// S steps of the steady march, the first (step n) at slot phase P0 (colour Q0)
template <int T, int D, int Q0, int P0, bool BP, bool P2, bool EM = false, int... NN>
__device__ __forceinline__ void steady_chunk(March<T, D>& m, d2* R, const Lane& c, const Sio& io,
                                             int r0, unsigned off_n,
                                             std::integer_sequence<int, NN...>) {
    constexpr int S = ring_slots<T, D>();
    (steady_step<T, D, Q0 ^ (NN & 1), (P0 + NN) % S, BP, P2, EM>(
         m, R, c, io, r0 + NN, off_n + (unsigned)NN * io.row_bytes),
     ...);
}

// One update's operands: x-part m2c(x1, cc) + x2, y-part m2c(y1, cc) + y2
// (stage()'s expressions, the same rounding tree), rhs rh
struct Upd {
    double x1, x2, y1, y2, cc, rh;
};

// the update of cell c of colour Q's red (RED) or black column: operands of
// stage()'s kSteady form; Nb = the row the update reads above (In / Mr)
template <int Q, bool RED, class FL, class FR>
__device__ __forceinline__ Upd upd_ops(d2 Cur, d2 Nb, d2 Lo, d2 Rr, FL fl, FR fr) {
    // Cur: the row updated (A or M1), Lo: the row below (M1 or M2), Rr: rhs row
    if (Q == 0) return Upd{Cur.y, fl(Cur.y), Nb.x, Lo.x, Cur.x, Rr.x};
    return Upd{fr(Cur.x), Cur.x, Nb.y, Lo.y, Cur.y, Rr.y};
}

// two independent updates, their operations interleaved one by one (the
// compiler keeps the order under register pressure; one chain alone leaves
// every dependent FP64 operation's latency exposed)
template <bool P2>
__device__ __forceinline__ void upd2(const Lane& c, const Upd& a, const Upd& b, double& na,
                                     double& nb, double& ra, double& rb) {
    const double hxa = m2c(a.x1, a.cc), hxb = m2c(b.x1, b.cc);
    const double hya = m2c(a.y1, a.cc), hyb = m2c(b.y1, b.cc);
    const double sxa = hxa + a.x2, sxb = hxb + b.x2;
    const double sya = hya + a.y2, syb = hyb + b.y2;
    ra = resid<P2>(a.rh, sxa, sya, c.idx2, c.idy2);
    rb = resid<P2>(b.rh, sxb, syb, c.idx2, c.idy2);
    const double pa = c.coef * ra, pb = c.coef * rb;
    na = a.cc - pa;
    nb = b.cc - pb;
}

// the new value of colour Q's cell of a row (EM: only in an updated column,
// stage()'s kSteadyEdge lane masks), and its residual (EM: an owned column)
template <int Q, bool EM>
__device__ __forceinline__ void put_new(const Lane& c, d2& row, double v) {
    if (Q == 0) row.x = (!EM || c.up_a) ? v : row.x;
    else        row.y = (!EM || c.up_b) ? v : row.y;
}
template <int Q, bool EM>
__device__ __forceinline__ void tally_q(const Lane& c, TallyAcc& acc, double r) {
    if (!EM) {
        tally_steady(acc, r);
    } else {
        const double rm = (Q == 0 ? c.own_a : c.own_b) ? r : 0.0;  // select: NaN-safe
        acc = __builtin_fma(rm, rm, acc);
    }
}
// EM: the ghost column copies of a finished row at a physical left / right
// side (stage()'s EDGE block, in its order)
template <bool EM>
__device__ __forceinline__ void ghost_cols(const Lane& c, d2& F) {
    if (!EM) return;
    const double f1 = from_right(F.x);  // column ib+1 (lane l+1's ia)
    const double fl = from_left(F.y);   // column ia-1 (lane l-1's ib)
    if (c.fix0_b) F.y = f1;
    if (c.fixr_a) F.x = fl;
    if (c.fixr_b) F.y = F.x;
}

// stage ta of chain a (colour QA) and stage tb of chain b (colour QB), kSteady
// (EM: kSteadyEdge), interleaved: red of both, then black of both.  Same
// arithmetic as stage().
template <int QA, int QB, bool P2, bool EM = false>
__device__ __forceinline__ void stage_pair(const Lane& c, d2& InA, d2& A_a, d2& M1_a, d2& M2_a,
                                           d2 Ra_a, d2 Rb_a, TallyAcc& acc_a, d2& InB, d2& A_b,
                                           d2& M1_b, d2& M2_b, d2 Ra_b, d2 Rb_b,
                                           TallyAcc& acc_b, bool tally_a = true,
                                           bool tally_b = true) {
    auto fl = [](double v) { return from_left(v); };
    auto fr = [](double v) { return from_right(v); };
    double na, nb, ra, rb;
    // red: row rin-1 (A) of each chain
    upd2<P2>(c, upd_ops<QA, true>(A_a, InA, M1_a, Ra_a, fl, fr),
             upd_ops<QB, true>(A_b, InB, M1_b, Ra_b, fl, fr), na, nb, ra, rb);
    d2 Mr_a = A_a, Mr_b = A_b;
    put_new<QA, EM>(c, Mr_a, na);
    put_new<QB, EM>(c, Mr_b, nb);
    if (tally_a) tally_q<QA, EM>(c, acc_a, ra);
    if (tally_b) tally_q<QB, EM>(c, acc_b, rb);
    // black: row rin-2 (M1), reading the new red row above
    upd2<P2>(c, upd_ops<QA, false>(M1_a, Mr_a, M2_a, Rb_a, fl, fr),
             upd_ops<QB, false>(M1_b, Mr_b, M2_b, Rb_b, fl, fr), na, nb, ra, rb);
    d2 F_a = M1_a, F_b = M1_b;
    put_new<QA, EM>(c, F_a, na);
    put_new<QB, EM>(c, F_b, nb);
    if (tally_a) tally_q<QA, EM>(c, acc_a, ra);
    if (tally_b) tally_q<QB, EM>(c, acc_b, rb);
    ghost_cols<EM>(c, F_a);
    ghost_cols<EM>(c, F_b);
    M2_a = F_a; M1_a = Mr_a; A_a = InA; InA = F_a;
    M2_b = F_b; M1_b = Mr_b; A_b = InB; InB = F_b;
}

// interior block of H = k * S rows: 4T paired warm-up steps, then k chunks of
// S statically unrolled steps
template <int T, int D, int Q0, bool BP, bool P2>
__device__ __forceinline__ void march_interior(March<T, D>& m, const Lane& c, const Io& io,
                                               const Sio& sio, int rs, int nchunks) {
    constexpr int S = ring_slots<T, D>();
    march_pairs<T, D, Q0, kPre, BP, P2>(m, c, io, rs, rs + 4 * T - 1);  // 4T is even
    // ring in static slots: rhs row rs - 1 + j in slot j mod S; at step n = 4T
    // the paired ring holds j = 4T - 1 - k (k < 2T), the rows in flight j = 4T + k
    d2 R[S];
#pragma unroll
    for (int k = 0; k < S; ++k) R[k] = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 2 * T; ++k) R[(4 * T - 1 - k) % S] = m.R[k];
#pragma unroll
    for (int k = 0; k < D; ++k) R[(4 * T + k) % S] = m.Rq[k];
    // every chunk starts at slot phase 4T mod S (S is even, so colour Q0 too)
    constexpr int P0 = (4 * T) % S;
    int r0 = rs + 4 * T;
    unsigned off = 4u * T * sio.row_bytes;
    for (int k = 0; k < nchunks; ++k) {
        steady_chunk<T, D, Q0, P0, BP, P2>(m, R, c, sio, r0, off,
                                           std::make_integer_sequence<int, S>{});
        r0 += S;
        off += (unsigned)S * sio.row_bytes;
    }
}

}  // namespace

// One wave's march over the 128-column strip whose owned columns start at
// c_out (c_ld = c_out - 2T), rows [j0, j1) of block row `by`; the owned
// columns end at min(ni, own_hi) (own_hi: the 4-column path runs its strip
// at a physical side as several of these, clipped to its own columns; ni +
// anything for the 2-column kernel).  The wave's residual of every stage is
// added to acc[].
// STEADY = false: no static-ring path (the caller knows the block's rows are
// not steady-able; the chained kernel's edge blocks)
template <int T, int D, bool BP, bool P2 = false, bool STEADY = true>
__device__ __forceinline__ void tb_strip2(const SweepParams& prm, const double* __restrict__ src,
                                          double* __restrict__ dst,
                                          const double* __restrict__ rhs, const int c_out,
                                          const int own_hi, const int j0, const int j1,
                                          const int by, const int lane, double (&acc)[T]) {
    constexpr int OW = kStripCells - 4 * T;
    constexpr int S = ring_slots<T, D>();
    const int ni = prm.ni, nj = prm.nj;
    const int c_ld = c_out - 2 * T;
    const long long pitch = prm.pitch;
    const int own_end = min(ni, own_hi);

    Lane c;
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
    // columns this lane stores: owned interior + the physical ghost columns
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

    March<T, D> m;
#pragma unroll
    for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
    m.keep[0] = m.keep[1] = d2{0.0, 0.0};

    const long long base = (long long)kYOff * pitch + kXOff + c.ia;
    Io io{src + base, rhs + base, dst + base, pitch};
    const int rs = j0 - 2 * T;  // first streamed row
    const int rend = j1 - 1 + 2 * T;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        m.Pq[k] = ldv(io.sp + (long long)(rs + k) * pitch);
        m.Rq[k] = ldv(io.rp + (long long)(rs - 1 + k) * pitch);
    }
#pragma unroll
    for (int t = 0; t < T; ++t) m.A[t] = m.M1[t] = m.M2[t] = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 2 * T; ++k) m.R[k] = d2{0.0, 0.0};
    // the colour of row rs: the same for every block of the launch (H even)
    const bool q1 = ((c.parity + rs) & 1) != 0;

    // columns interior: every column of the cone an updated cell (no lane
    // masks, no ghost columns) and ownership uniform per lane -- the strip
    // is whole, or it runs past column ni into a neighbour's halo (or the
    // padding beyond it) with ni even, so ni | ni+1 falls between lanes;
    // those lanes are neither stored nor counted.  Rows interior: no
    // ghost rows in the cone, and a block height the static ring divides.
    const bool cols_in = c_ld >= prm.upd_lo_i && c_ld + kStripCells - 1 <= prm.upd_hi_i &&
                         (c_out + OW - 1 <= ni || (ni & 1) == 0);
    const bool rows_in = rs >= prm.upd_lo_j && rend <= prm.upd_hi_j &&
                         (j1 - j0) % S == 0 && j1 - j0 > 0;
    if (!cols_in) {
        if (q1) march_pairs<T, D, 1, kEdge, false, P2>(m, c, io, rs, rend);
        else    march_pairs<T, D, 0, kEdge, false, P2>(m, c, io, rs, rend);
    } else {
        if (STEADY && rows_in) {
            // wave-uniform descriptors over the strip's 128 columns
            auto rsrc = [&](const double* b, int row0, int rows) {
                const unsigned long long a = (unsigned long long)(
                    b + (long long)(kYOff + row0) * pitch + kXOff + c_ld);
                const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
                const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
                return __builtin_amdgcn_make_buffer_rsrc(
                    (void*)(((unsigned long long)hi << 32) | lo), (short)0,
                    (int)((long long)rows * pitch * 8), 0x00020000);
            };
            Sio sio;
            sio.p = rsrc(src, rs, rend - rs + 1 + D);
            sio.r = rsrc(rhs, rs - 1, rend - rs + 1 + D);
            sio.d = rsrc(dst, j0, j1 - j0);
            sio.lane = (unsigned)lane * 16u;
            sio.st_lane = c.own_a ? (unsigned)lane * 16u : 0x40000000u;
            sio.row_bytes = (unsigned)(pitch * 8);
            const int nchunks = (j1 - j0) / S;
            if (q1) march_interior<T, D, 1, BP, P2>(m, c, io, sio, rs, nchunks);
            else    march_interior<T, D, 0, BP, P2>(m, c, io, sio, rs, nchunks);
        } else {
            if (q1) march_pairs<T, D, 1, kRowEdge, false, P2>(m, c, io, rs, rend);
            else    march_pairs<T, D, 0, kRowEdge, false, P2>(m, c, io, rs, rend);
        }
        if (!c.own_a) {
#pragma unroll
            for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
        }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] += m.acc[t];
}

// block rows: nby_big of H = rows_per_block rows, then h_small-row ones
// (short blocks, which the work order takes last), the last takes the rest
// (misor_api.hip tb_geometry)
__device__ __forceinline__ void block_rows(const SweepParams& prm, int by, int& j0, int& j1) {
    const int H = prm.rows_per_block;
    j0 = by < prm.nby_big ? 1 + by * H : 1 + prm.nby_big * H + (by - prm.nby_big) * prm.h_small;
    j1 = by == prm.nby - 1 ? prm.nj + 1 : j0 + (by < prm.nby_big ? H : prm.h_small);
}

// physical corners are never touched by solveRB; carry them into dst
__device__ __forceinline__ void copy_corners(const SweepParams& prm, const double* src,
                                             double* dst) {
    if (threadIdx.x < 4) {
        const int t = threadIdx.x;
        const int ci = (t & 1) ? prm.ni + 1 : 0, cj = (t & 2) ? prm.nj + 1 : 0;
        const bool phys = ((t & 1) ? prm.ghost_right : prm.ghost_left) &&
                          ((t & 2) ? prm.ghost_top : prm.ghost_bottom);
        if (phys) {
            const long long k = (long long)(cj + kYOff) * prm.pitch + (ci + kXOff);
            dst[k] = src[k];
        }
    }
}

// deterministic reduction per stage: lane tree, then waves in order
template <int T, int WAVES>
__device__ __forceinline__ void block_partials(const SweepParams& prm, const double (&acc)[T],
                                               double* partials, int L, double (*wsum)[WAVES]) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
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
    __syncthreads();  // wsum is reused by the workgroup's next block
}

// one block (bx, by) of a pass: logical block L
template <int T, int WAVES, int D, bool BP, bool P2>
__device__ __forceinline__ void tb_block(const SweepParams& prm, const double* __restrict__ src,
                                         double* __restrict__ dst, const double* __restrict__ rhs,
                                         double* __restrict__ partials, const int L,
                                         double (*wsum)[WAVES]) {
    constexpr int OW = kStripCells - 4 * T;
    const int bx = L % prm.nbx, by = L / prm.nbx;
    int j0, j1;
    block_rows(prm, by, j0, j1);
    if (prm.part != 0) {  // overlapped decomposed pass: blocks clear of the halo first
        const int lo = 1 + bx * WAVES * OW - 2 * T;
        const int hi = 1 + (bx * WAVES + WAVES - 1) * OW - 2 * T + kStripCells - 1;
        const bool interior = lo >= prm.int_lo_i && hi <= prm.int_hi_i &&
                              j0 - 2 * T >= prm.int_lo_j && j1 - 1 + 2 * T <= prm.int_hi_j;
        if (interior != (prm.part == 1)) return;
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c_out = 1 + (bx * WAVES + wave) * OW;
    if (L == 0) copy_corners(prm, src, dst);
    double acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = 0.0;
    if (c_out <= prm.ni)  // wave-uniform
        tb_strip2<T, D, BP, P2>(prm, src, dst, rhs, c_out, 0x7fffffff, j0, j1, by, lane, acc);
    block_partials<T, WAVES>(prm, acc, partials, L, wsum);
}

// occupancy target: 2 waves per SIMD (the register file of one wave is 256
// VGPRs; below that the compiler would rather use AGPRs and run one wave).
//
// Two ways to hand out blocks:
//  - one workgroup per block (queue == nullptr): block L of workgroup
//    blockIdx.x, dealt to XCDs in contiguous runs (xcd_remap);
//  - persistent (queue != nullptr): as many workgroups as fit on the GPU at
//    once; workgroup w (on XCD w % 8, the hardware's round-robin) takes
//    tickets from its XCD's queue -- a contiguous run of blocks, as above --
//    and, once that is empty, from the other XCDs' queues.  The makespan then
//    ends within one block of the last one started, instead of a last,
//    partly filled round of workgroups (one rank's block at 8 GPUs runs
//    3.5 rounds of 512 workgroups).  queue[0..7] are zeroed before the launch.
template <class Block>
__device__ __forceinline__ void for_each_block(const SweepParams& prm, int* __restrict__ queue,
                                               int* ticket, Block&& block) {
    const int nwg = prm.nblocks, qq = nwg / 8, rr = nwg % 8;
    auto run_start = [&](int x) { return x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq; };
    // Work order (persistent launches): the blocks on the grid's border first
    // (the slower lane-masked / row-tested marches: strips at a physical
    // left/right side, block rows at a physical bottom/top side, the last
    // block row of non-uniform height), then the rest in row-major order (the
    // short block rows last); the XCD queues hold contiguous runs of that
    // order.  Slow blocks start early and the pass ends on short ones.
    const int nbx = prm.nbx, nby = prm.nby;
    auto order = [&](int k) -> int {  // k-th block of the work order -> L
        if (nby <= 2 || nbx <= 2) return k;
        if (k < nbx) return k;                                 // bottom row
        k -= nbx;
        if (k < nbx) return (nby - 1) * nbx + k;               // top row
        k -= nbx;
        if (k < nby - 2) return (1 + k) * nbx;                 // left column
        k -= nby - 2;
        if (k < nby - 2) return (1 + k) * nbx + nbx - 1;       // right column
        k -= nby - 2;
        const int w = nbx - 2;                                 // the rest
        return (1 + k / w) * nbx + 1 + k % w;
    };
    const int home = blockIdx.x % 8;
    bool first = true;
    for (int probe = 0; probe < 8;) {
        int L;
        if (!queue) {  // one workgroup per block: one trip
            if (!first) break;
            L = blockIdx.x;
            if (prm.xcd_remap) L = run_start(L % 8) + L / 8;
        } else {
            const int x = (home + probe) & 7;
            if (threadIdx.x == 0) *ticket = atomicAdd(&queue[x], 1);
            __syncthreads();
            const int b = *ticket;
            __syncthreads();
            if (b >= (x < rr ? qq + 1 : qq)) {
                ++probe;
                continue;
            }
            L = order(run_start(x) + b);
        }
        first = false;
        block(L);
    }
}

// ---------------------------------------------------------------------------
// Chained passes: vertical runs of blocks (SweepParams::chain)
//
// A block of H rows streams H + 4T rows (4T warm-up rows re-read from the
// block below), so short blocks waste HBM traffic and issue slots in their
// warm-up.  Here a workgroup that finishes block (bx, by) goes on with
// (bx, by + 1) with its stage registers live: the march continues, no
// warm-up, no re-read.  Blocks stay short (4 ring lengths, ~72 rows) -- they
// are the unit of residual partials (fixed slots: the sum order does not
// depend on who ran a block) and of work stealing -- while the runs are long.
//
// Work: segments = ranges of block rows of one column, one 64-bit word each
// (chain_word): the next unclaimed block row N, the end E (exclusive), the
// column.  A launch starts from a host-built list of segments (about one per
// resident workgroup, misor_api.hip chain_plan), in one run per XCD (the
// slow blocks first; neighbouring columns on one XCD share its L2: the
// strips' overlapping columns).  A workgroup takes a segment by ticket and
// claims its blocks one by one
// (atomicAdd(word, 1): block N is its if N < E).  Once the tickets are gone it
// steals: it scans the segments for the most unclaimed blocks r = E - N, and
// takes the top r/2 with a compare-and-swap of (N, E) -> (N, E - r/2) (the
// owner, which only ever increments N, keeps the block it claims next); the
// stolen range becomes a new segment so it can be split again.  A workgroup
// exits when no segment has 2 or more unclaimed blocks; every block is
// claimed exactly once, by a workgroup that runs it.
//
// Modes along a run (the colour of each row is the same as in tb_strip2):
// columns with a strip at a physical left / right side form a list of their
// own, run by a second kernel (EDGE = 1: steady chunks with lane masks,
// kSteadyEdge, one row in flight to stay within the registers) beside the
// main one; every strip keeps the static ring at every block boundary -- a block whose
// cone touches a physical bottom / top side (or the column's last block, of
// any height) is marched in pairs (kRowEdge) between two ring conversions,
// the rest run steady chunks.  Every block height but the column's last is a
// multiple of the ring's S slots, so every block boundary is at slot phase
// 4T mod S.
// ---------------------------------------------------------------------------
// a block row [j0, j1) that can be part of a run: its cone clear of the
// physical bottom / top sides and a height the static ring divides
// (tb_strip2's rows_in); misor_api.hip chain_plan uses the same test
template <int T, int D>
__host__ __device__ inline bool chain_rows_ok(const SweepParams& prm, int j0, int j1) {
    constexpr int S = ring_slots<T, D>();
    return j0 - 2 * T >= prm.upd_lo_j && j1 - 1 + 2 * T <= prm.upd_hi_j && (j1 - j0) % S == 0 &&
           j1 > j0;
}

__device__ __forceinline__ int chain_next(unsigned long long w) { return (int)(w & kChainMask); }
__device__ __forceinline__ int chain_end(unsigned long long w) {
    return (int)((w >> kChainBits) & kChainMask);
}
__device__ __forceinline__ int chain_col(unsigned long long w) { return (int)(w >> (2 * kChainBits)); }

__device__ __forceinline__ unsigned long long chain_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The run a workgroup takes next, into sh[0..3] = column, block row, segment
// slot (-1: a private range), end of the blocks it owns (own_end); sh[8] =
// the blocks its segment had unclaimed; sh[0] = -1: no work left.  Wave 0
// only.  alt_n0 >= 0: another launch's list of alt_n0 initial segments (the
// split ring's main list, taken by the edge kernel once its own is done):
// steals only -- its tickets are that launch's workgroups'
__device__ __forceinline__ void chain_acquire(const SweepParams& prm, int* head,
                                              unsigned long long* seg,
                                              int* sh, int alt_n0 = -1) {
    const int lane = threadIdx.x & 63;
    const int n0 = alt_n0 >= 0 ? alt_n0 : prm.nseg0;
    // 1. the initial segments, by ticket: the home XCD's run first
    int got = 0;
    if (lane == 0 && alt_n0 < 0) {
        const int home = blockIdx.x % 8;
        for (int probe = 0; probe < 8;) {
            const int x = (home + probe) & 7;
            const int cnt = prm.seg_run[x + 1] - prm.seg_run[x];
            const int b = atomicAdd(&head[x], 1);
            if (b >= cnt) {
                ++probe;
                continue;
            }
            const int k = prm.seg_run[x] + b;
            const unsigned long long old = atomicAdd(&seg[k], 1ull);
            if (chain_next(old) < chain_end(old)) {  // else stolen empty before its owner came
                sh[0] = chain_col(old);
                sh[1] = chain_next(old);
                sh[2] = k;
                sh[3] = chain_next(old) + 1;  // blocks claimed: the first
                sh[8] = chain_end(old) - chain_next(old);
                got = 1;
                break;
            }
        }
    }
    if (__shfl(got, 0, 64)) return;
    // 2. steal the top half of the segment with the most unclaimed blocks
    for (;;) {
        const int ndyn = min(__hip_atomic_load(&head[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                             prm.seg_cap);
        const int n = n0 + ndyn;
        // (another launch's list: only ranges of 2 blocks or more are taken, a
        // stolen run paying its warm-up once for them)
        const int r_min = alt_n0 >= 0 ? 4 : 2;
        int best_r = r_min - 1, best_k = -1;
        constexpr int U = 8;  // loads in flight per lane
        for (int k0 = 0; k0 < n; k0 += 64 * U) {
            unsigned long long w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u * 64 + lane;
                w[u] = k < n ? chain_load(seg + k) : 0ull;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = chain_end(w[u]) - chain_next(w[u]);
                if (r > best_r) {
                    best_r = r;
                    best_k = k0 + u * 64 + lane;
                }
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int r = __shfl_xor(best_r, o, 64), k = __shfl_xor(best_k, o, 64);
            if (r > best_r || (r == best_r && k > best_k)) {
                best_r = r;
                best_k = k;
            }
        }
        best_k = __shfl(best_k, 0, 64);
        if (best_k < 0) {  // nothing left to split: the owners finish the rest
            if (lane == 0) sh[0] = -1;
            return;
        }
        int ok = 0;
        if (lane == 0) {
            unsigned long long w = chain_load(seg + best_k);
            for (;;) {
                const int N = chain_next(w), E = chain_end(w), r = E - N;
                if (r < r_min) break;
                const int m = E - r / 2;  // the owner keeps [N, m)
                const unsigned long long nw =
                    chain_word(chain_col(w), N, m);
                const unsigned long long prev = atomicCAS(seg + best_k, w, nw);
                if (prev == w) {
                    sh[0] = chain_col(w);
                    sh[1] = m;
                    sh[2] = -1;
                    sh[3] = E;  // a private range: all its blocks are the thief's
                    sh[8] = E - m;
                    if (E - m >= 2) {  // the rest of the stolen range becomes stealable
                        const int d = atomicAdd(&head[8], 1);
                        if (d < prm.seg_cap) {
                            atomicExch(seg + n0 + d, chain_word(chain_col(w), m + 1, E));
                            sh[2] = n0 + d;
                            sh[3] = m + 1;  // stealable: blocks claimed one by one
                        }
                    }
                    ok = 1;
                    break;
                }
                w = prev;
            }
        }
        if (__shfl(ok, 0, 64)) return;
    }
}

// End of block L of a run: the block's residual partials, one per wave and
// stage at fixed slots (partials[(t * nblocks + L) * WAVES + wave]: no
// barrier), then the run's next block.  The owner of a segment claims its
// blocks a few at a time (sh[8]: the unclaimed blocks it saw at its last
// claim; k = that / 8, 1..4), so most block ends need no atomic and no
// barrier: own_end (wave-uniform, the same in every wave) is the end of the
// blocks already claimed.  Returns the next block row, or -1.
template <int T, int WAVES, class Acc>
__device__ __forceinline__ int chain_block_end(const SweepParams& prm, Acc (&acc)[T],
                                               double* partials, int L, int* sh,
                                               unsigned long long* seg, int slot, int by,
                                               int& own_end) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    double mine = 0.0;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const double s = wave_sum(acc[t]);
        if (lane == t) mine = s;
        acc[t] = 0.0;
    }
    if (lane < T)
        partials[((long long)lane * prm.nblocks + L) * WAVES + wave] = mine;
    if (threadIdx.x == 0 && prm.trace) {  // diagnostics: when this block began and ended, who ran it
        const unsigned long long now = wall_clock64();
        unsigned long long* tr = prm.trace + 3ll * L;
        tr[0] = *reinterpret_cast<volatile unsigned long long*>(sh + 4);
        tr[1] = now;
        tr[2] = blockIdx.x | (sh[6] ? 1ull << 32 : 0ull);
        *reinterpret_cast<volatile unsigned long long*>(sh + 4) = now;
        sh[6] = 0;
    }
    if (by + 1 < own_end) return by + 1;
    if (slot < 0) return -1;  // a private range: own_end is its end
    __syncthreads();  // every wave has read the last claim
    if (threadIdx.x == 0) {
        const int k = min(4, max(1, sh[8] / 8));
        const unsigned long long old = atomicAdd(seg + slot, (unsigned long long)k);
        const int N = chain_next(old), E = chain_end(old);
        sh[1] = N < E ? N : -1;
        sh[7] = min(N + k, E);
        sh[8] = E - N;
    }
    __syncthreads();
    // wave-uniform (the buffer descriptors and row offsets of the next block
    // derive from it: they must be scalars)
    own_end = __builtin_amdgcn_readfirstlane(sh[7]);
    return __builtin_amdgcn_readfirstlane(sh[1]);
}

// One wave's chained run over its strip of column bx, from block row by
// (the colour of the first streamed row: Q0): steady chunks over the static
// ring -- with the lane masks of a strip at a physical left / right side if
// EM (kSteadyEdge) -- or, for a block row that is not steady-able (general;
// such a block is a segment of its own), the general paired march (kEdge).
// Every wave of the workgroup calls chain_block_end at the same block ends.
template <int T, int WAVES, int D, int Q0, bool P2, bool EM>
__device__ __forceinline__ void chain_strip(const SweepParams& prm, const double* __restrict__ src,
                                            double* __restrict__ dst,
                                            const double* __restrict__ rhs,
                                            double* __restrict__ partials, double (*wsum)[WAVES],
                                            int* sh, unsigned long long* seg, Lane& c,
                                            const Io& io, bool general, int c_ld, int bx, int by,
                                            int slot, int own_end, int lane) {
    constexpr int S = ring_slots<T, D>();
    const long long pitch = prm.pitch;
    int j0, j1;
    block_rows(prm, by, j0, j1);
    auto set_block = [&](int b, int a0, int a1) {
        c.j0 = a0;
        c.j1 = a1;
        c.wlo = b == 0 && prm.ghost_bottom;
        c.whi = b == prm.nby - 1 && prm.ghost_top;
    };
    set_block(by, j0, j1);
    March<T, D> m;
#pragma unroll
    for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
    m.keep[0] = m.keep[1] = d2{0.0, 0.0};
    const int rs = j0 - 2 * T;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        m.Pq[k] = ldv(io.sp + (long long)(rs + k) * pitch);
        m.Rq[k] = ldv(io.rp + (long long)(rs - 1 + k) * pitch);
    }
#pragma unroll
    for (int t = 0; t < T; ++t) m.A[t] = m.M1[t] = m.M2[t] = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 2 * T; ++k) m.R[k] = d2{0.0, 0.0};

    if (!EM && general) {  // rows not steady-able: the general march, block by block
        march_pairs<T, D, Q0, kEdge, false, P2>(m, c, io, rs, j1 - 1 + 2 * T);
        for (;;) {
            const int nb = chain_block_end<T, WAVES>(prm, m.acc, partials, by * prm.nbx + bx, sh,
                                                     seg, slot, by, own_end);
            if (nb < 0) return;
            by = nb;
            block_rows(prm, by, j0, j1);
            set_block(by, j0, j1);
            march_pairs<T, D, Q0, kEdge, false, P2>(m, c, io, j0 + 2 * T, j1 - 1 + 2 * T);
        }
    }
    auto rsrc = [&](const double* b, int row0, int rows) {
        const unsigned long long a =
            (unsigned long long)(b + (long long)(kYOff + row0) * pitch + kXOff + c_ld);
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
        return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo),
                                                 (short)0, (int)((long long)rows * pitch * 8),
                                                 0x00020000);
    };
    // 4T warm-up steps, then the static ring: rhs row rs - 1 + j in slot j mod S.
    // (kPre updates every column it streams: right for interior strips, whose
    // garbage columns never reach an owned one; a strip at a physical side
    // needs the masks and ghost-column copies of kEdge -- its rows are
    // interior, so nothing is tallied or stored)
    march_pairs<T, D, Q0, EM ? kEdge : kPre, false, P2>(m, c, io, rs, rs + 4 * T - 1);
    d2 R[S];
#pragma unroll
    for (int k = 0; k < S; ++k) R[k] = d2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 2 * T; ++k) R[(4 * T - 1 - k) % S] = m.R[k];
#pragma unroll
    for (int k = 0; k < D; ++k) R[(4 * T + k) % S] = m.Rq[k];
    for (;;) {
        // the steady chunks of block [j0, j1): descriptors from its virtual
        // start j0 - 2T (the ring phase is the same at every block start:
        // the heights are multiples of S)
        {
            const int vrs = j0 - 2 * T, vrend = j1 - 1 + 2 * T;
            Sio sio;
            sio.p = rsrc(src, vrs, vrend - vrs + 1 + D);
            sio.r = rsrc(rhs, vrs - 1, vrend - vrs + 1 + D);
            sio.d = rsrc(dst, j0, j1 - j0);
            sio.lane = (unsigned)lane * 16u;
            sio.st_lane = c.own_a ? (unsigned)lane * 16u : 0x40000000u;
            sio.st_a = c.st_a ? (unsigned)lane * 16u : 0x40000000u;
            sio.st_b = c.st_b ? (unsigned)lane * 16u + 8u : 0x40000000u;
            sio.row_bytes = (unsigned)(pitch * 8);
            constexpr int P0 = (4 * T) % S;
            int r0 = vrs + 4 * T;
            unsigned off = 4u * T * sio.row_bytes;
            for (int k = 0; k < (j1 - j0) / S; ++k) {
                steady_chunk<T, D, Q0, P0, false, P2, EM>(m, R, c, sio, r0, off,
                                                         std::make_integer_sequence<int, S>{});
                r0 += S;
                off += (unsigned)S * sio.row_bytes;
            }
        }
        if (!EM && !c.own_a) {  // lanes that do not own their columns tallied garbage
#pragma unroll
            for (int t = 0; t < T; ++t) m.acc[t] = 0.0;
        }
        const int nb = chain_block_end<T, WAVES>(prm, m.acc, partials, by * prm.nbx + bx, sh, seg,
                                                 slot, by, own_end);
        if (nb < 0) return;
        by = nb;
        block_rows(prm, by, j0, j1);
        set_block(by, j0, j1);
    }
}

// the per-lane constants and pointers of a strip
template <int T>
__device__ __forceinline__ void chain_lane(const SweepParams& prm, const double* src,
                                           double* dst, const double* rhs, int c_ld, int lane,
                                           Lane& c, Io& io) {
    const int ni = prm.ni;
    const long long pitch = prm.pitch;
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
    c.st_a = c.own_a || c.fixr_a;
    c.st_b = c.own_b || c.fix0_b || c.fixr_b;
    c.lo_j = prm.upd_lo_j;
    c.hi_j = prm.upd_hi_j;
    c.parity = prm.parity;
    c.gb = prm.ghost_bottom;
    c.gt = prm.ghost_top;
    c.nj = prm.nj;
    c.idx2 = prm.idx2;
    c.idy2 = prm.idy2;
    c.coef = prm.coef;
    c.bl = ((lane + 63) & 63) * 4;
    c.br = ((lane + 1) & 63) * 4;
    const long long base = (long long)kYOff * pitch + kXOff + c.ia;
    io = Io{src + base, rhs + base, dst + base, pitch};
}

// one run of a chained pass: column bx from block row by (all waves).
// EDGE = 0: the columns clear of the physical left / right sides (steady
// chunks) and the blocks of non-steady rows (the general march); EDGE = 1:
// the steady rows of the columns at a physical left / right side, every
// strip in kSteadyEdge chunks.  The two are separate kernels (rb_tbc_kernel's
// EDGE), launched side by side: one kernel with both kinds of steady chunks
// makes the register allocator spill them at T = 8.
template <int T, int WAVES, int D, bool P2, int EDGE>
__device__ __forceinline__ void chain_run(const SweepParams& prm, const double* __restrict__ src,
                                          double* __restrict__ dst, const double* __restrict__ rhs,
                                          double* __restrict__ partials, double (*wsum)[WAVES],
                                          int* sh, unsigned long long* seg, int bx, int by,
                                          int slot, int own_end) {
    constexpr int OW = kStripCells - 4 * T;
    const int lane = threadIdx.x & 63;
    // wave-uniform (as known to the compiler: the strip's descriptors and
    // branches derive from it)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ni = prm.ni;
    const int c_out = 1 + (bx * WAVES + wave) * OW;
    if (bx == 0 && by == 0) copy_corners(prm, src, dst);
    if (c_out > ni) {  // no strip for this wave: only the block ends
        double acc[T];
#pragma unroll
        for (int t = 0; t < T; ++t) acc[t] = 0.0;
        for (;;) {
            by = chain_block_end<T, WAVES>(prm, acc, partials, by * prm.nbx + bx, sh, seg, slot,
                                           by, own_end);
            if (by < 0) return;
        }
    }
    const int c_ld = c_out - 2 * T;
    Lane c;
    Io io;
    chain_lane<T>(prm, src, dst, rhs, c_ld, lane, c, io);
    int j0, j1;
    block_rows(prm, by, j0, j1);
    // steady chunks for strips clear of the physical left / right sides, in
    // runs of steady-able block rows; the general lane-masked, row-tested
    // march (kEdge) for the rest: strips at a physical side, and the few
    // block rows whose cone reaches a physical bottom / top side (or a
    // column's last block of a height the ring does not divide) -- the host
    // keeps those in segments of their own.  (A row-tested-only march for
    // the latter, kRowEdge, in the same kernel as the steady runs makes the
    // register allocator spill the runs' ring.)
    // steady chunks in runs of steady-able block rows; the general
    // lane-masked, row-tested march (kEdge) for the few block rows whose cone
    // reaches a physical bottom / top side (or a column's last block of a
    // height the ring does not divide) -- the host keeps those in segments
    // of their own.  (A row-tested-only march for the latter, kRowEdge, in
    // the same kernel as the steady runs makes the register allocator spill
    // the runs' ring.)
    const bool general = !chain_rows_ok<T, D>(prm, j0, j1);
    // the colour of the run's first streamed row: every block but a column's
    // last is an even number of rows tall, so the same at every block start
    const bool q1 = ((prm.parity + j0 - 2 * T) & 1) != 0;
    // (EDGE strips keep one row in flight, not D: the lane masks need the
    // registers; the ring has the same S slots for D = 1 and 2)
    static_assert(ring_slots<T, 1>() == ring_slots<T, D>(), "edge ring");
    if constexpr (EDGE != 0) {  // kSteadyEdge for every strip
        if (q1)
            chain_strip<T, WAVES, 1, 1, P2, true>(prm, src, dst, rhs, partials, wsum, sh, seg, c,
                                                  io, false, c_ld, bx, by, slot, own_end, lane);
        else
            chain_strip<T, WAVES, 1, 0, P2, true>(prm, src, dst, rhs, partials, wsum, sh, seg, c,
                                                  io, false, c_ld, bx, by, slot, own_end, lane);
    } else {  // (the host puts every column with a strip at a physical side in the EDGE list)
        if (q1)
            chain_strip<T, WAVES, D, 1, P2, false>(prm, src, dst, rhs, partials, wsum, sh, seg, c,
                                                   io, general, c_ld, bx, by, slot, own_end, lane);
        else
            chain_strip<T, WAVES, D, 0, P2, false>(prm, src, dst, rhs, partials, wsum, sh, seg, c,
                                                   io, general, c_ld, bx, by, slot, own_end, lane);
    }
}

// chained persistent pass (2-column strips); work = the launch's work area
// (int head[kChainHead], then the segment words; misor_api.hip chain plans)
template <int T, int WAVES, int D, bool P2, int EDGE = 0>
__global__ __launch_bounds__(kLanes* WAVES, 2) void rb_tbc_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, int force, int* __restrict__ work) {
    __shared__ double wsum[T][WAVES];  // (unused by the chained march: per-wave partials)
    // sh[0..3]: the run (chain_acquire), sh[4..5]: trace clock, sh[6]: run start,
    // sh[7]: own_end of the last claim, sh[8]: unclaimed blocks seen then
    __shared__ __attribute__((aligned(8))) int sh[12];
    if (!force && st->done) return;
    unsigned long long* seg = reinterpret_cast<unsigned long long*>(work + kChainHead);
    for (;;) {
        // every wave has read the last claim of the previous run (a run's
        // last block end can leave the waves apart: no barrier on its way out)
        __syncthreads();
        if (threadIdx.x < kLanes) chain_acquire(prm, work, seg, sh);
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
        if (bx < 0) break;
        chain_run<T, WAVES, D, P2, EDGE>(prm, src, dst, rhs, partials, wsum, sh, seg, bx, by, slot,
                                         own_end);
    }
}

template <int T, int WAVES, int D, bool BP, bool P2 = false>
__global__ __launch_bounds__(kLanes* WAVES, 2) void rb_tb_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, int force, int* __restrict__ queue) {
    __shared__ double wsum[T][WAVES];
    __shared__ int ticket;
    if (force || !st->done) {
        for_each_block(prm, queue, &ticket, [&](int L) {
            tb_block<T, WAVES, D, BP, P2>(prm, src, dst, rhs, partials, L, wsum);
        });
    }
    // Persistent launch: the queue resets itself for the next one (instead of
    // a memset launch before every pass).  queue[8] counts the workgroups that
    // are done with the ticket counters -- every one of them, those that found
    // the solve done included -- and the last one zeroes all nine.  Its
    // atomics (agent scope) come after every other workgroup's last ticket:
    // each of those took its returned value before leaving the loop.
    if (queue && threadIdx.x == 0) {
        if (atomicAdd(&queue[8], 1) == (int)gridDim.x - 1) {
#pragma unroll
            for (int x = 0; x < 9; ++x) atomicExch(&queue[x], 0);
        }
    }
}


}  // namespace misor
