// misor_internal.h -- device layout, grid state and kernel launchers shared by
// the libmisor translation units.  Not part of the public ABI (include/misor.h).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>

#include "misor.h"

namespace misor {

// ---------------------------------------------------------------------------
// HBM layout of every field (p, p', rhs, u, v, f, g)
//
// Reference cell (i,j), i in [0, ni+1], j in [0, nj+1] (ghosts included), lives
// at   base[(j + kYOff) * pitch + (i + kXOff)].
//  - kXOff = 15 puts the first interior column i = 1 on a 128-byte boundary,
//    so every wave's 16-byte-per-lane row segment of 128 cells starts a cache
//    line; the ghost column i = 0 is the last double of the preceding line.
//  - kYOff = 2 * kMaxT + 16 rows below row 0 and as many (+ prefetch run-out)
//    above row nj+1: a block of the temporally blocked sweep streams rows
//    j0-2T-1 .. j1-1+2T (+ rows in flight; the split-ring march up to 14
//    more warm-up rows below, sor_tbh.h) without clamping, and its first
//    strip's columns from 1 - 2T (the tail of the row below, in the
//    allocation: a left halo of depth 2 kMaxT too).
//  - pitch = 160 + round_up(ni, kStripCells * kMaxWavesX): left pad line, the
//    strips, the run-out of the last (overlapping) strip and pad; a multiple
//    of 16 doubles (128 B) that is not a power of two.
// Padding cells are zero and never feed an interior result.
// ---------------------------------------------------------------------------
constexpr int kXOff = 15;
constexpr int kMaxT = 10;                // iterations per temporally blocked pass (max)
constexpr int kYOff = 2 * kMaxT + 16;
constexpr int kLanes = 64;                 // wavefront
constexpr int kStripCells = 2 * kLanes;    // 128 columns per wave (2 per lane)
constexpr int kMaxWavesX = 16;             // strips per sweep workgroup (max)
constexpr int kMaxAhead = 3;               // rows a sweep keeps in flight (max)

inline long long layout_pitch(int ni) {
    const int w = kStripCells * kMaxWavesX;
    return 160 + (long long)((ni + w - 1) / w) * w;
}
// rows j = -kYOff .. nj + 2*kMaxT + kMaxAhead + 1 (a temporally blocked block
// streams 2T rows past its last row, plus the rows it keeps in flight)
inline long long layout_rows(int nj) { return (long long)nj + 2 * kYOff + kMaxAhead + 3; }

// sweep kernel variants: strips per workgroup, rows in flight, nt stores
struct SweepVariant {
    int waves, ahead, nt_store, nt_load;
};
constexpr SweepVariant kSweepVariants[] = {
    {4, 1, 0, 0}, {4, 2, 0, 0}, {4, 3, 0, 0}, {4, 1, 1, 0}, {4, 2, 1, 0},
    {8, 1, 0, 0}, {8, 2, 0, 0}, {8, 2, 1, 0}, {8, 1, 1, 0}, {8, 3, 1, 0},
    {16, 1, 1, 0}, {16, 2, 1, 0}, {4, 3, 1, 0}, {8, 2, 1, 1}, {16, 2, 1, 1}};
constexpr int kNumSweepVariants = 15;
constexpr int kDefaultSweepVariant = 7;  // 8 strips, 2 rows ahead, nt stores (tools/tune_sweep.py)
int sweep_waves(int variant);

// temporally blocked sweep (sor_tb.hip): strips per workgroup, rows in flight
// (x-neighbour shifts through ds_bpermute instead of DPP -- the kernel's BP
// template flag -- measured 5% slower: profiles/r02_tune_bperm.txt)
// 128-column strips (2 columns per lane), 2 waves per SIMD.
// skew: the split-ring march in two independent stage chains per step (sor_tbh.h
// hrs_step); hr: the split rhs ring, registers + LDS (sor_tbh.h)
// max_t = 0: retired -- measured slower and no longer built (DESIGN.md section 4:
// 1 / 3 eight / one strips per workgroup, 4 three rows in flight, 5 four
// columns per lane at one wave per SIMD, 6-8 strips exchanging edge columns
// through LDS, 9 the skewed register-ring march, 10/11 an LDS row queue, 12 the
// unskewed split ring); configuring one fails.  The register-ring kernels run
// T <= kMaxT2 (above that their rhs ring spills); the split ring (13) runs T up
// to kMaxT.
constexpr int kMaxT2 = 8;
struct TbVariant {
    int waves, ahead, max_t, skew, hr;
};
constexpr TbVariant kTbVariants[] = {
    {4, 2, kMaxT2}, {4, 2, 0}, {2, 2, kMaxT2}, {4, 2, 0}, {4, 2, 0}, {4, 2, 0}, {4, 2, 0},
    {4, 2, 0},      {4, 2, 0}, {4, 2, 0},      {4, 2, 0}, {4, 2, 0}, {4, 2, 0},
    {4, 2, kMaxT, 1, 1}};
constexpr int kNumTbVariants = 14;
constexpr int kHrTbVariant = 13;   // the skewed split ring (T = 1 unskewed)
// the short plan of capped solves (misor_api.hip solve_rb_from)
constexpr int kShortTbVariant = kHrTbVariant;
constexpr int kShortT = 10;
constexpr long long kShortDistCells = 1LL << 28;  // decomposed: local blocks at least this big
constexpr long long kHrAllCells = 1LL << 26;      // chained blocks from here: every solve > 8
// iterations per pass: 8 on large local blocks, 7 below kTsteps8Cells cells
// (32768^2 0.744 vs 0.785 ms/iteration, profiles/r02_tune_t789.txt; one rank's
// 8192 x 16384 block at 8 GPUs 0.118-0.122 at T = 7 vs 0.125 at T = 8,
// profiles/r02_small_rows.txt, r02_tb_rows_t8.txt)
constexpr int kDefaultTsteps = 8;
constexpr int kSmallBlockTsteps = 7;
constexpr long long kTsteps8Cells = 1LL << 28;
constexpr int kDefaultTbVariant = 0;   // 4 strips, 2 rows in flight
// block heights tried, tallest first (misor_api.hip pick_tb_rows)
constexpr int kTbRowLadder[] = {576, 384, 288, 192};
constexpr int kTbRowLadderLen = 4;
constexpr int kTbSmallRows = 32;       // short block rows the work order takes last ...
constexpr int kTbSmallRounds = 2;      // ... about this many resident rounds of them
constexpr int kTbReserve = 16;         // slots a pipelined interior launch leaves free
int tb_waves(int variant);
// the split rhs ring (sor_tbh.h): stages 0 .. K-1 read registers, the rest LDS;
// both rings have S slots, S = max(2K + D, 2(T - K) + 1) rounded up to even.
// K: as few register stages as the LDS allows -- S <= kHrMaxSlots rows of 1 KB
// per wave (two workgroups of four waves: 144 KB of the CU's 160)
constexpr int kHrMaxSlots = 18;
// The skewed form (sk = 1) keeps one more row in each ring.
__host__ __device__ constexpr int hr_cost(int T, int D, int k, int sk = 0) {
    const int a = 2 * k + D + sk, b = 2 * (T - k) + 1 + sk;
    const int s = a > b ? a : b;
    return s + (s & 1);
}
__host__ __device__ constexpr int hr_k(int T, int D, int sk = 0) {
    for (int k = 0; k <= T; ++k)
        if (hr_cost(T, D, k, sk) <= kHrMaxSlots) return k;
    return T;
}
__host__ __device__ constexpr int hr_slots(int T, int D, int sk = 0) {
    return hr_cost(T, D, hr_k(T, D, sk), sk);
}
// rhs ring slots of the steady march: interior block heights are multiples of it
int tb_ring_slots(int T, int variant);
// workgroups of a persistent pass resident on the device at once
int tb_resident(int T, int variant);
int tb_max_t(int variant);
int tb_out_width(int T, int variant);           // owned columns of one wave's strip
int tb_nbx(int ni, int T, int variant);         // block columns of a pass of T iterations

// Solver state that lives on the device between launches.  Written only by
// the finish kernel (one workgroup) and read by the next sweep launch.
struct DevState {
    int it;        // iterations completed
    int done;      // 1 once (res >= eps^2 && it < itermax) is false
    int itermax;   // cap of the current solve call
    int near;      // 1: stopped before iteration it+1, whose res fell within nband of
                   // eps^2 (misor_api.hip exact_tail recomputes from there)
    int lite_miss; // 1: stopped before iteration it+1, whose residual lower bound (a
                   // lite pass, SweepParams::lite) did not prove the loop goes on
    double res;    // residual of the last iteration
    double epssq;
    double nband = -1.0;  // |res - eps^2| <= nband: near the threshold (< 0: off, the
                          // default of every DevState the host builds)
    double sum[kMaxT];  // sum r^2 of each iteration of the last pass (this rank,
                        // then all-reduced)
};

struct SweepParams {
    long long pitch;
    int ni, nj;          // local interior size
    int rows_per_block;  // H (temporally blocked: block rows 0 .. nby_big-1 are H tall)
    int nby;             // temporally blocked: block rows; rows nby_big .. nby-2 are
                         // h_small tall, the last one takes the rest (tb_geometry)
    int nby_big, h_small;
    int parity;          // (ioff + joff) & 1 : global colour of local cell (0,0)
    int ghost_left, ghost_right, ghost_bottom, ghost_top;  // physical boundary -> Neumann copy
    int red_lo_i, red_hi_i, red_lo_j, red_hi_j;  // cells whose red value is computed
    int variant;         // index into kSweepVariants
    int nbx, nblocks;    // launch geometry (logical blocks nbx x nby)
    int xcd_remap;       // deal consecutive logical blocks to one XCD
    int part;            // 0: all blocks, 1: interior blocks only, 2: boundary blocks only
    int int_lo_i, int_hi_i, int_lo_j, int_hi_j;  // footprint bounds of an interior block
    int upd_lo_i, upd_hi_i, upd_lo_j, upd_hi_j;  // temporally blocked: cells updated
                                                 // (1..n on physical sides, all on
                                                 // neighbour sides)
    double idx2, idy2, coef;  // 1/dx^2, 1/dy^2, factor (RB) or omega*factor (RBA)
    int pow2;                 // idx2 == idy2 == 2^m, m >= 0: the default TB kernel's P2 form
    int reserve;              // persistent launch: leave this many workgroup slots free
                              // (host only; the comm / edge streams' kernels run there)
    // chained passes (sor_tb.h rb_tbc_kernel): vertical runs of blocks taken
    // from the launch's segment list, with work stealing
    int chain;                // 1: blocks are 4 ring lengths tall, runs chain them
    int nseg0;                // segments of the launch's initial list
    int seg_cap;              // dynamic segment slots (created by steals)
    int chain_blocks;         // blocks in the launch (its part)
    int chain_edge;           // the edge list (strips at a physical left / right side)
    int lite;                 // the split ring's steady chunks count the residual of the
                              // stages before the last one on one row in S (a lower
                              // bound; misor_solve.hip kLite)
    int chain_grid;           // edge list: its workgroups (the first of the launch)
    int seg_run[9];           // XCD x takes the initial segments [seg_run[x], seg_run[x+1])
    unsigned long long* trace;  // diagnostics (MISOR_CHAIN_TRACE): per block L, 3 words --
                                // start and end (wall clock, 100 MHz), workgroup | run start
    const unsigned long long* seg_tmpl;  // the initial list (device; copied per launch)
    // the split ring's edge kernel: once its own list is done, its workgroups
    // steal from the main list's work area (initialised before either kernel
    // starts: no_init on the main launch); nullptr: no second list
    int* alt_work = nullptr;
    int alt_nseg0 = 0;
    int no_init = 0;          // the work area is initialised already (misor_solve.hip)
};

// Chained passes: a segment word holds the next unclaimed block row (bits
// 0..25), the end block row, exclusive (26..51), and the column (52..63).
// Work area of a chained launch: int head[kChainHead] (0..7: per-XCD tickets
// of the initial segments, 8: dynamic segments created), then the words.
constexpr int kChainBits = 26;
constexpr unsigned long long kChainMask = (1ull << kChainBits) - 1;
constexpr int kChainHead = 16;
constexpr int kChainSegCap = 4096;       // dynamic slots per launch
constexpr int kChainRingsPerBlock = 4;   // block height of a chained pass, in ring lengths
// the chained split-ring pass (sor_tbh.h rb_tbhc_kernel): blocks of 8 ring
// lengths (144 rows at T = 10), a block of a column at a physical left / right
// side costing ~2.5 others (its strip's kSteadyEdge chunks run ~1.8x a steady
// strip's; profiles/r05_hrsweep2_*.txt)
constexpr int kHrChainRingsPerBlock = 8;
constexpr double kHrChainEdgeCost = 2.5;
// the same on a decomposed rank's block (its passes split in two parts around
// the halo exchange): 10 ring lengths (180 rows) and an edge-column block at 3
// others -- wall ms per iteration of the pipelined loop, alternated on one box
// (profiles/r05_rank_geometry_ab.txt): the 8-GPU rank block with physical
// left + bottom sides 0.121 against 0.139 at 8 / 2.5, bottom only 0.125 vs
// 0.127, the 4-GPU block 0.204 vs 0.230, the 2-GPU block unchanged (sweeps:
// r05_edge_rings_ab*.txt; a single rank, without the split, stays at 144 rows)
constexpr int kHrChainRingsDist = 10;
constexpr double kHrChainEdgeCostDist = 3.0;
// chained passes by default on local blocks below this many cells: there the
// unchained blocks are short and their 4T warm-up rows cost most (one 8-GPU
// rank's 8192 x 16384 of the 32768^2 bench: 0.106 vs 0.110-0.118 ms per
// iteration); on larger blocks the unchained 576-row blocks are ahead
// (32768^2: 0.661 vs 0.695-0.709; profiles/r03_chain_rows.txt)
constexpr long long kChainCells = 1LL << 28;
constexpr double kChainEdgeCost = 2.0;   // a block of a column at a physical left / right
                                         // side, in steady blocks (segment lengths): a
                                         // kSteadyEdge block measures ~1.5; the edge
                                         // kernel's workgroups cannot steal from the main
                                         // one's, so it is given a few more than its share
                                         // (profiles/r03_chain_edge_cost.txt)
__host__ __device__ inline unsigned long long chain_word(int col, int next, int end) {
    return ((unsigned long long)col << (2 * kChainBits)) |
           ((unsigned long long)end << kChainBits) | (unsigned long long)next;
}
// zero the head, copy the initial list, empty the dynamic slots
void launch_chain_init(hipStream_t s, int* work, const unsigned long long* tmpl, int nseg0,
                       int cap);

struct NsParams {
    double dx, dy, dt;
    double xlength, ylength;
    double re, gx, gy, gamma;
    int bc_left, bc_right, bc_bottom, bc_top, problem;
};

// kernel launchers (sor_kernels.hip, ns_kernels.hip)
void launch_sweep(hipStream_t s, const SweepParams& prm, const double* src, double* dst,
                  const double* rhs, double* partials, const DevState* st);
// the same sweep (default variant's geometry) storing r^2 of every counted cell into rsq
void launch_sweep_rsq(hipStream_t s, const SweepParams& prm, const double* src, double* dst,
                      const double* rhs, double* partials, const DevState* st, double* rsq);
// T iterations per pass: partials[t * nparts + block]
void launch_finish(hipStream_t s, const double* partials, int nparts, int T, DevState* st,
                   double cells, int decide);
void launch_decide(hipStream_t s, DevState* st, int T, double cells, int lite = 0);
// single-rank loop test in two levels (chunk sums, then the finish kernel over
// kFinishChunks values per stage); scratch holds kMaxT * kFinishChunks doubles
constexpr int kFinishChunks = 32;
// count: a zeroed device int -- the partial-sum launch's last workgroup then
// runs the loop test itself (one launch); nullptr: a second, finish launch.
// decide 0: only the sums into st->sum (decomposed: all-reduce, then decide)
void launch_finish2(hipStream_t s, const double* partials, int nparts, int T, DevState* st,
                    double cells, double* scratch, int* count, int decide, int lite = 0);
// queue: 8 device ints (zeroed by the launch) for a persistent launch whose
// workgroups take blocks from per-XCD queues; nullptr: one workgroup per block
void launch_tb(hipStream_t s, int T, const SweepParams& prm, const double* src, double* dst,
               const double* rhs, double* partials, const DevState* st, int force, int* queue);
// the same for one T (sor_tb_inst.hip, one unit per T)
#define MISOR_DECL_TB(N)                                                                      \
    void launch_tb_t##N(hipStream_t s, const SweepParams& prm, const double* src, double* dst, \
                        const double* rhs, double* partials, const DevState* st, int force,   \
                        int* queue);                                                          \
    int tb_resident_t##N(int variant);
MISOR_DECL_TB(1) MISOR_DECL_TB(2) MISOR_DECL_TB(3) MISOR_DECL_TB(4) MISOR_DECL_TB(5)
MISOR_DECL_TB(6) MISOR_DECL_TB(7) MISOR_DECL_TB(8) MISOR_DECL_TB(9) MISOR_DECL_TB(10)
#undef MISOR_DECL_TB
// lexicographic Gauss-Seidel SOR, whole solve in one workgroup (lex_kernels.hip)
void launch_solve_lex(hipStream_t s, double* p, const double* rhs, int ni, int nj,
                      long long pitch, double idx2, double idy2, double factor, double cells,
                      int xorder, DevState* st);
// whole-solve single-workgroup kernel for grids whose p fits in LDS
int small_solve_fits(int ni, int nj);
void launch_solve_small(hipStream_t s, double* p, const double* rhs, int ni, int nj,
                        long long pitch, double idx2, double idy2, double coef, double cells,
                        DevState* st);

// 8-neighbour halo exchange of one field (halo.hip): regions in local cell
// coordinates; direction order L, R, B, T, BL, BR, TL, TR
constexpr int kDirs = 8;
struct HaloRegion {
    int x0, y0, w, h;  // first cell and extent (local reference indices)
    long long off;     // offset in the packed buffer (doubles)
};
struct HaloPlan {
    HaloRegion send[kDirs], recv[kDirs];
    long long total;  // doubles in each of the send / recv buffers
};
void launch_pack(hipStream_t s, const double* field, long long pitch, const HaloPlan& plan,
                 double* sendbuf);
void launch_unpack(hipStream_t s, double* field, long long pitch, const HaloPlan& plan,
                   const double* recvbuf);
int sweep_partials(int ni, int nj, int rows_per_block, int waves, int* nbx, int* nby);
// in-process transport: out[k] = combination (sum / max, rank order) of
// gather[q * kMaxT + k] over q < nranks, k < n
void launch_local_combine(hipStream_t s, const double* gather, int nranks, int n, int is_max,
                          double* out);

void launch_fill(hipStream_t s, double* a, long long count, double v);
// the message misor_last_error() returns (thread-local, shared by the 2D and 3D ABI)
void set_last_error(const char* msg);
void launch_poisson_init(hipStream_t s, double* p, double* rhs, const double* sx,
                         const double* sy, const double* rx, int ni, int nj,
                         long long pitch, int problem);

struct NsLaunch {
    hipStream_t s;
    long long pitch;
    int ni, nj;
    NsParams prm;
    // physical-boundary flags (multi-GPU: only edge ranks apply wall BCs)
    int wall_left, wall_right, wall_bottom, wall_top;
    int ioff, joff;          // global index of local cell (0,0)
    int imax_g, jmax_g;      // global interior size
};
void launch_set_bc(const NsLaunch& L, double* u, double* v);
void launch_special_bc(const NsLaunch& L, double* u);
void launch_compute_fg(const NsLaunch& L, const double* u, const double* v, double* f,
                       double* g);
void launch_compute_rhs(const NsLaunch& L, const double* f, const double* g, double* rhs);
// computeFG + computeRHS in one column march (RHS of column 1 / row 1 next to a
// neighbour rank left to launch_rhs_edges after the f, g exchange)
void launch_compute_fg_rhs(const NsLaunch& L, const double* u, const double* v, double* f,
                           double* g, double* rhs);
void launch_rhs_edges(const NsLaunch& L, const double* f, const double* g, double* rhs);
void launch_adapt_uv(const NsLaunch& L, const double* f, const double* g, const double* p,
                     double* u, double* v);
// reductions over ALL (ni+2)(nj+2) cells: partial per block, then a finish
int reduce_blocks(int ni, int nj);
void launch_absmax2(const NsLaunch& L, const double* u, const double* v, double* partials);
// adaptUV + the partials of launch_absmax2 over the fields it leaves
void launch_adapt_absmax(const NsLaunch& L, const double* f, const double* g, const double* p,
                         double* u, double* v, double* partials);
// normalizePressure's sum, exact (order- and decomposition-independent):
// fixed-point terms at 2^(E - kSumFrac), E = exponent of the global max |p|;
// limbs[0..2] = the local sum as three 44-bit integer limbs (doubles, summed
// exactly by an all-reduce); exact_sum_value rounds the total once (host)
constexpr int kSumFrac = 72;
void launch_exact_sum(const NsLaunch& L, const double* p, int E, double* partials,
                      double* limbs);
double exact_sum_value(const double limbs[3], int E);
void launch_finish_reduce(hipStream_t s, const double* partials, int n, int op, int width,
                          double* out);
// p -= avg over the whole local array (normalizePressure)
void launch_sub_mean(const NsLaunch& L, double* p, double avg);
enum { kReduceSum = 0, kReduceMax = 1 };

// ---------------------------------------------------------------------------
// 3D (assignment-6): dense reference layout (imax+2)(jmax+2)(kmax+2), i fastest
// ---------------------------------------------------------------------------
struct G3 {
    int I, J, K;        // interior cells (K: this rank's planes)
    long long sx, sxy;  // strides of j and k: (I+2), (I+2)(J+2)
    int Kg = 0, koff = 0;            // global planes; global k of local plane 0
    int lo_phys = 1, hi_phys = 1;    // local planes 1 / K border the physical boundary
    __host__ __device__ long long ix(int i, int j, int k) const {
        return (long long)k * sxy + (long long)j * sx + i;
    }
};
struct Fg3 {  // computeFG's scalars (solver.c:620-629)
    double gamma, ix, iy, iz, iRe, dt, gx, gy, gz;
};
int ns3_partials(const G3& g);
void launch3_rhs(hipStream_t s, const G3& g, const double* f, const double* gg, const double* h,
                 double* rhs, double idx, double idy, double idz, double idt);
// one solve iteration: two colour-pass launches (the ghost copy fused in) and
// the loop test; returns the number of partials per pass
int launch3_rb_iteration(hipStream_t s, const G3& g, double* p, const double* rhs, double idx2,
                         double idy2, double idz2, double factor, double* partials, DevState* st,
                         double cells);
// one solve iteration as ONE sweep launch (red then black, src -> dst) plus
// the loop test; rows in {4, 8, 12}, kc planes per workgroup
int sweep3_blocks(const G3& g, int rows, int kc);
int launch3_sweep(hipStream_t s, const G3& g, const double* src, double* dst, const double* rhs,
                  double idx2, double idy2, double idz2, double factor, int rows, int kc,
                  double* partials, DevState* st, double cells, bool sum_only = false,
                  bool ra2 = false);
void launch3_fg(hipStream_t s, const G3& g, const double* u, const double* v, const double* w,
                double* f, double* gg, double* h, const Fg3& c);
void launch3_adapt(hipStream_t s, const G3& g, const double* f, const double* gg,
                   const double* h, const double* p, double* u, double* v, double* w, double fx,
                   double fy, double fz);
void launch3_wall(hipStream_t s, const G3& g, double* n, double* t1, double* t2, int axis,
                  int gh, int in, int on, int onin, int bc);
void launch3_special(hipStream_t s, const G3& g, double* u, int problem);
int absmax3_blocks();
void launch3_absmax(hipStream_t s, const double* u, const double* v, const double* w,
                    long long n, double* partials, double* out);
void launch3_normalize(hipStream_t s, const G3& g, double* p, double* partials, double* sum,
                       double cells);
// normalizePressure in two halves around a cross-rank all-reduce of *sum
void launch3_interior_sum(hipStream_t s, const G3& g, const double* p, double* partials,
                          double* sum);
void launch3_sub_mean(hipStream_t s, const G3& g, double* p, const double* sum, double cells);
// the loop test of a decomposed solve: st->sum[0] holds the all-reduced sum
// of r^2 of the iteration (written by launch3_sweep with sum_only)
void launch3_decide(hipStream_t s, DevState* st, double cells);
// single rank, the loop test folded into the sweep: the sweep first applies
// the test of the previous sweep (prev_partials; nullptr: none) to st_in,
// workgroup 0 writes the result to st_out, and the launch is a no-op once the
// loop is over; launch3_fold_decide applies the test of a batch's last sweep
void launch3_sweep_folded(hipStream_t s, const G3& g, const double* src, double* dst,
                          const double* rhs, double idx2, double idy2, double idz2,
                          double factor, int rows, int kc, double* partials,
                          const double* prev_partials, const DevState* st_in, DevState* st_out,
                          double cells, bool ra2 = false);
// the whole solve in one cooperative launch, p resident in LDS
// (ns3d_resident.hip): boxes for this grid (0: not possible here), the size of
// its barrier state, the launch (0 ok, 1 refused -> fall back, < 0 error) and
// whether a barrier wait timed out
int resident3_boxes(const G3& g);
size_t resident3_bar_bytes();
int launch3_resident(hipStream_t s, const G3& g, double* p, const double* rhs, double idx2,
                     double idy2, double idz2, double factor, double cells, double* partials,
                     DevState* st, void* bar, double* mbox);
int resident3_aborted(const void* bar, hipStream_t s, int* aborted);
void launch3_fold_decide(hipStream_t s, const G3& g, int rows, int kc,
                         const double* prev_partials, const DevState* st_in, DevState* st_out,
                         double cells);

}  // namespace misor
