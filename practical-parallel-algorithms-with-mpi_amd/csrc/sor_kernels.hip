// sor_kernels.hip -- fused red-black SOR sweep for gfx950 (MI355X).
//
// One launch = one full red+black iteration of solveRB
// (assignment-4/src/solver.c:197-229): both colour passes, the residual
// sum r^2 of both colours, and the Neumann ghost copy of :219-227, reading p
// from `src` and writing the new p to `dst` (ping-pong buffers).
//
// Why fused: two half-sweep kernels on the natural layout touch every cache
// line of p and rhs twice per iteration (~48 B per lattice update); this kernel
// reads p and rhs once and writes p once: 24 B/LUP, the algorithmic minimum.
//
// Work decomposition
//   wave      = one strip of 128 columns (lane l owns columns ia=c0+2l, ia+1;
//               one 16-byte load per lane per row = one 1 KiB wave access)
//   workgroup = 4 strips side by side x H rows (blockIdx.y)
// Each wave marches up its H rows keeping a 3-row window in registers:
//   step r: red update of row r   (needs old rows r-1, r, r+1)
//           black update of row r-1 (needs the new red values of rows r-2..r)
//           store row r-1 once.
// The red values one column left/right of the strip (needed by the strip's
// edge black cells) and one row below/above the block are recomputed
// redundantly from the same old values, so they are bit-identical to the
// values the owning wave computes.  Nothing is exchanged between waves or
// workgroups inside a launch.
//
// Bit-exactness: the update and residual use the reference expression order
// ((P(i+1)-2P)+P(i-1))*idx2 + ((P(j+1)-2P)+P(j-1))*idy2 with no FMA
// contraction (-ffp-contract=off), so every cell value equals the CPU's
// bit for bit.  Only the order in which r^2 is summed differs (deterministic:
// fixed lane tree, fixed wave order, fixed block order in the finish kernel).
//
// Colour: cell (i,j) is red iff (i+j) is even in GLOBAL indices (pass 0 of
// solveRB starts at i=1 on j=1); `parity` carries the offset of this rank's
// block so decomposed runs colour identically.

#include "misor_internal.h"

namespace misor {

namespace {

// lane l receives lane l-1's value (lane 0: its own, overridden by callers)
__device__ __forceinline__ double from_left(double v) { return __shfl_up(v, 1, 64); }
// lane l receives lane l+1's value (lane 63: its own, overridden by callers)
__device__ __forceinline__ double from_right(double v) { return __shfl_down(v, 1, 64); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT = false>
__device__ __forceinline__ d2 ldv(const double* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const d2*>(p));
    return *reinterpret_cast<const d2*>(p);
}

template <bool NT>
__device__ __forceinline__ void stv(double* p, d2 v) {
    if (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p));
    else
        *reinterpret_cast<d2*>(p) = v;
}

// WAVES: strips per workgroup; D: rows of p / rhs kept in flight ahead of the
// row being updated; NT: non-temporal stores of the new p (write-once stream)
// RSQ: also store r^2 of every cell this block counts into rsq (same layout as
// p) -- the exact, order-independent residual of misor_api.hip exact_tail
template <int WAVES, int D, bool NT, bool LNT, bool RSQ = false>
__global__ __launch_bounds__(kLanes* WAVES) void rb_sweep_kernel(
    SweepParams prm, const double* __restrict__ src, double* __restrict__ dst,
    const double* __restrict__ rhs, double* __restrict__ partials,
    const DevState* __restrict__ st, double* __restrict__ rsq = nullptr) {
    __shared__ double wsum[WAVES];
    if (st->done) return;  // converged or capped: the whole grid exits

    // logical block: with xcd_remap, blocks that the dispatcher deals to one XCD
    // (b, b+8, b+16, ...) get consecutive logical ids, so horizontally and
    // vertically adjacent blocks share that XCD's L2 for their halo lines
    int L = blockIdx.x;
    if (prm.xcd_remap) {
        const int nwg = prm.nblocks, q = nwg / 8, rr = nwg % 8, x = L % 8;
        L = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + L / 8;
    }
    const int bx = L % prm.nbx, by = L / prm.nbx;
    if (prm.part != 0) {  // overlapped decomposed sweep: interior / boundary split
        const int c0b = 1 + bx * WAVES * kStripCells;
        const int j0b = 1 + by * prm.rows_per_block;
        const int j1b = min(j0b + prm.rows_per_block, prm.nj + 1);
        const bool interior = (c0b - 2 >= prm.int_lo_i) &&
                              (c0b + WAVES * kStripCells + 1 <= prm.int_hi_i) &&
                              (j0b - 2 >= prm.int_lo_j) && (j1b + 1 <= prm.int_hi_j);
        if (interior != (prm.part == 1)) return;  // the other launch owns this block
    }

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int strip = bx * WAVES + wave;
    const int ni = prm.ni, nj = prm.nj;
    const int c0 = 1 + strip * kStripCells;
    const int ia = c0 + 2 * lane;  // odd local column
    const int ib = ia + 1;
    const long long pitch = prm.pitch;
    const double idx2 = prm.idx2, idy2 = prm.idy2, coef = prm.coef;

    const bool hl = (lane == 0);   // holds the left halo pair  (c0-2, c0-1)
    const bool hr = (lane == 63);  // holds the right halo pair (c0+128, c0+129)
    const bool in_a = ia <= ni;    // owned: black update + residual
    const bool in_b = ib <= ni;
    // red is also recomputed on the 1-deep halo ring where a neighbour rank
    // owns it (red_lo/hi = 0 / n+1 there), from the 2-deep halo of p
    const bool red_a = ia <= prm.red_hi_i;
    const bool red_b = ib <= prm.red_hi_i;
    const int hcol = hl ? c0 - 1 : c0 + kStripCells;  // halo column that can be red
    const bool in_h = (hcol >= prm.red_lo_i) && (hcol <= prm.red_hi_i);
    const int hoff = hl ? -2 : 2;  // halo pair address relative to ia (lanes 0 / 63)

    double acc = 0.0;

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

    if (c0 <= ni) {  // wave-uniform: strips past the domain only join the reduction
        const int j0 = 1 + by * prm.rows_per_block;
        const int j1 = min(j0 + prm.rows_per_block, nj + 1);

        // element (ia, j) of the three arrays: base + j*pitch
        const double* sp = src + (long long)kYOff * pitch + kXOff + ia;
        const double* rp = rhs + (long long)kYOff * pitch + kXOff + ia;
        double* dp = dst + (long long)kYOff * pitch + kXOff + ia;
        double* qp = RSQ ? rsq + (long long)kYOff * pitch + kXOff + ia : nullptr;

        auto ldp = [&](int j) { return ldv<LNT>(sp + (long long)j * pitch); };
        auto ldr = [&](int j) { return ldv<LNT>(rp + (long long)j * pitch); };
        auto ldph = [&](int j) {
            d2 v = {0.0, 0.0};
            if (hl | hr) v = ldv(sp + (long long)j * pitch + hoff);
            return v;
        };
        auto ldrh = [&](int j) {
            d2 v = {0.0, 0.0};
            if (hl | hr) v = ldv(rp + (long long)j * pitch + hoff);
            return v;
        };

        // window: Mm2 = M(r-2), Mm1 = M(r-1) (red new, black old), Oc = O(r);
        // rings Pq = O(r+1 .. r+D), Rq = rhs(r .. r+D-1) (+ halo pairs) in flight
        d2 Mm1 = ldp(j0 - 2), Hm1 = ldph(j0 - 2);
        d2 Oc = ldp(j0 - 1), Hc = ldph(j0 - 1);
        d2 Pq[D], Hq[D], Rq[D], RHq[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            Pq[k] = ldp(j0 + k);
            Hq[k] = ldph(j0 + k);
            Rq[k] = ldr(j0 - 1 + k);
            RHq[k] = ldrh(j0 - 1 + k);
        }
        d2 Mm2 = {0.0, 0.0}, Rm1 = {0.0, 0.0};
        double HRm1 = 0.0;

        for (int r = j0 - 1; r <= j1; ++r) {
            // issue the loads D rows ahead
            const d2 nP = ldp(r + 1 + D), nH = ldph(r + 1 + D);
            const d2 nR = ldr(r + D), nRH = ldrh(r + D);
            const d2 Up = Pq[0], Hup = Hq[0], Rc = Rq[0], RHc = RHq[0];

            // ---------------- red pass on row r ----------------
            const int q = (prm.parity + 1 + r) & 1;  // 0: column ia red, 1: column ib red
            d2 Mr = Oc;
            double HRc = hl ? Hc.y : Hc.x;  // halo-column value after the red pass
            if (r >= prm.red_lo_j && r <= prm.red_hi_j) {
                const bool own = (r >= j0) && (r < j1);
                if (q == 0) {
                    // (ia, r) red; left neighbour from lane l-1 (lane 0: halo)
                    double Lf = from_left(Oc.y);
                    if (hl) Lf = Hc.y;
                    const double c = Oc.x;
                    const double rr = Rc.x - (((Oc.y - 2.0 * c) + Lf) * idx2 +
                                              ((Up.x - 2.0 * c) + Mm1.x) * idy2);
                    if (red_a) Mr.x = c - coef * rr;
                    if (in_a && own) acc += rr * rr;
                    if (RSQ && in_a && own) qp[(long long)r * pitch] = rr * rr;
                    // right halo column c0+128 is red too (same parity as ia)
                    if (hr && in_h) {
                        const double ch = Hc.x;
                        const double rh = RHc.x - (((Hc.y - 2.0 * ch) + Oc.y) * idx2 +
                                                   ((Hup.x - 2.0 * ch) + Hm1.x) * idy2);
                        HRc = ch - coef * rh;
                    }
                } else {
                    // (ib, r) red; right neighbour from lane l+1 (lane 63: halo)
                    double Rf = from_right(Oc.x);
                    if (hr) Rf = Hc.x;
                    const double c = Oc.y;
                    const double rr = Rc.y - (((Rf - 2.0 * c) + Oc.x) * idx2 +
                                              ((Up.y - 2.0 * c) + Mm1.y) * idy2);
                    if (red_b) Mr.y = c - coef * rr;
                    if (in_b && own) acc += rr * rr;
                    if (RSQ && in_b && own) qp[(long long)r * pitch + 1] = rr * rr;
                    // left halo column c0-1 is red (same parity as ib)
                    if (hl && in_h) {
                        const double ch = Hc.y;
                        const double rh = RHc.y - (((Oc.x - 2.0 * ch) + Hc.x) * idx2 +
                                                   ((Hup.y - 2.0 * ch) + Hm1.y) * idy2);
                        HRc = ch - coef * rh;
                    }
                }
            }

            // ---------------- black pass on row r-1, then store ----------------
            const int jw = r - 1;
            if (jw >= j0) {  // implies 1 <= jw <= nj
                d2 F = Mm1;
                if (q == 0) {
                    // row r-1 has q' = 1: column ia black, its right neighbour ib red
                    double Ln = from_left(Mm1.y);
                    if (hl) Ln = HRm1;
                    const double c = Mm1.x;
                    const double rr = Rm1.x - (((Mm1.y - 2.0 * c) + Ln) * idx2 +
                                               ((Mr.x - 2.0 * c) + Mm2.x) * idy2);
                    if (in_a) {
                        F.x = c - coef * rr;
                        acc += rr * rr;
                        if (RSQ) qp[(long long)jw * pitch] = rr * rr;
                    }
                } else {
                    // row r-1 has q' = 0: column ib black
                    double Rn = from_right(Mm1.x);
                    if (hr) Rn = HRm1;
                    const double c = Mm1.y;
                    const double rr = Rm1.y - (((Rn - 2.0 * c) + Mm1.x) * idx2 +
                                               ((Mr.y - 2.0 * c) + Mm2.y) * idy2);
                    if (in_b) {
                        F.y = c - coef * rr;
                        acc += rr * rr;
                        if (RSQ) qp[(long long)jw * pitch + 1] = rr * rr;
                    }
                }

                // Neumann ghost copy (assignment-4/src/solver.c:219-227), fused:
                // columns 0 / ni+1 of this row, rows 0 / nj+1 from rows 1 / nj.
                d2 out = F;
                if (prm.ghost_right) {
                    const double fb_left = from_left(F.y);  // final value at column ia-1
                    if (ia == ni + 1) out.x = fb_left;
                    if (ib == ni + 1) out.y = F.x;
                }
                double* drow = dp + (long long)jw * pitch;
                stv<NT>(drow, out);
                if (prm.ghost_left && strip == 0 && hl)  // (pad, P(0,jw) = P(1,jw))
                    stv<false>(drow - 2, d2{Hm1.x, F.x});
                if (prm.ghost_right && hr && c0 + kStripCells == ni + 1)
                    stv<false>(drow + 2, d2{F.y, Hm1.y});  // (P(ni+1)=P(ni), pad)
                if (prm.ghost_bottom && jw == 1) {
                    // row 0 <- row 1 for 1 <= i <= ni; corners keep their old value
                    const d2 o0 = Mm2;  // = old row 0 (ghost rows are never updated)
                    stv<false>(dp, d2{in_a ? F.x : o0.x, in_b ? F.y : o0.y});
                }
                if (prm.ghost_top && jw == nj) {
                    const d2 on = Mr;  // = old row nj+1
                    stv<false>(drow + pitch, d2{in_a ? F.x : on.x, in_b ? F.y : on.y});
                }
            }

            // rotate the window and the rings
            Mm2 = Mm1;
            Mm1 = Mr;
            Oc = Up;
            Hm1 = Hc;
            Hc = Hup;
            Rm1 = Rc;
            HRm1 = HRc;
#pragma unroll
            for (int k = 0; k + 1 < D; ++k) {
                Pq[k] = Pq[k + 1];
                Hq[k] = Hq[k + 1];
                Rq[k] = Rq[k + 1];
                RHq[k] = RHq[k + 1];
            }
            Pq[D - 1] = nP;
            Hq[D - 1] = nH;
            Rq[D - 1] = nR;
            RHq[D - 1] = nRH;
        }
    }

    // deterministic reduction: lane tree, then waves in order
    acc = wave_sum(acc);
    if (lane == 0) wsum[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += wsum[w];
        partials[L] = s;  // logical id: the sum order does not depend on the remap
    }
}

// Sum of the per-block partials in a fixed order, then the loop test of
// solveRB (assignment-4/src/solver.c:197,229,233):
//   res = sum / (imax*jmax); it++; continue while res >= eps^2 && it < itermax
// A temporally blocked pass leaves T groups of partials (one per iteration);
// they are decided in iteration order and the first failing test stops the
// count, exactly as the reference loop would have stopped.
// 256 threads: while a temporally blocked pass keeps every SIMD's registers
// full, a workgroup can only start where one of the sweep's workgroups has
// just left -- which frees one wave per SIMD, so a 1024-thread finish (4 waves
// per SIMD) could wait for a whole CU to drain; on the decomposed pipeline this
// kernel runs on the comm stream beside the next pass's sweep.
constexpr int kFinishThreads = 256;
// SC1: the partials were handed over by other workgroups of the same launch
// (rb_partsum_kernel's last workgroup): relaxed agent-scope loads (sc1)
template <bool SC1>
__device__ __forceinline__ void finish_body(const double* __restrict__ partials, int n, int T,
                                            DevState* st, double cells, int decide,
                                            double (&sh)[kMaxT][kFinishThreads],
                                            double (&tot)[kMaxT], int lite = 0) {
    constexpr int NT = kFinishThreads;
    const int t = threadIdx.x;
    auto ld = [&](const double* q) {
        return SC1 ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
    };
    // all T groups in one strided pass, four strides per trip with separate
    // accumulators (4T independent loads in flight per thread), combined in a
    // fixed order
    double s[kMaxT], s1[kMaxT], s2[kMaxT], s3[kMaxT];
#pragma unroll
    for (int g = 0; g < kMaxT; ++g) s[g] = s1[g] = s2[g] = s3[g] = 0.0;
    int k = t;
    for (; k + 3 * NT < n; k += 4 * NT) {
#pragma unroll
        for (int g = 0; g < kMaxT; ++g) {
            if (g < T) {
                const double* q = partials + (long long)g * n + k;
                s[g] += ld(q);
                s1[g] += ld(q + NT);
                s2[g] += ld(q + 2 * NT);
                s3[g] += ld(q + 3 * NT);
            }
        }
    }
    for (; k < n; k += NT) {
#pragma unroll
        for (int g = 0; g < kMaxT; ++g)
            if (g < T) s[g] += ld(partials + (long long)g * n + k);
    }
#pragma unroll
    for (int g = 0; g < kMaxT; ++g) s[g] = (s[g] + s1[g]) + (s2[g] + s3[g]);
#pragma unroll
    for (int g = 0; g < kMaxT; ++g)
        if (g < T) sh[g][t] = s[g];
    __syncthreads();
#pragma unroll
    for (int w = NT / 2; w >= 64; w >>= 1) {
        if (t < w) {
#pragma unroll
            for (int g = 0; g < kMaxT; ++g)
                if (g < T) sh[g][t] += sh[g][t + w];
        }
        __syncthreads();
    }
    if (t < 64) {
#pragma unroll
        for (int g = 0; g < kMaxT; ++g) {
            if (g < T) {
                const double v = wave_sum(sh[g][t]);
                if (t == 0) tot[g] = v;
            }
        }
    }
    if (t == 0) {
        for (int g = 0; g < T; ++g) {
            if (!decide) {
                st->sum[g] = tot[g];  // decomposed: all-reduce, then decide
            } else if (!st->done) {
                const double res = tot[g] / cells;
                if ((lite >> g) & 1) {
                    // a lower bound of the iteration's residual (the pass's steady
                    // chunks counted one row in S of this stage): it decides only
                    // where it proves the loop goes on -- not converged and not
                    // near the threshold, whatever the cells left out add
                    const int it = st->it + 1;
                    const bool on = st->nband >= 0.0 ? res > st->epssq + st->nband
                                                     : res >= st->epssq;
                    if (on && it < st->itermax) {
                        st->it = it;
                        st->res = res;  // (the pass's last stage is counted in full)
                    } else {
                        st->lite_miss = 1;  // the host redoes the pass counting every cell
                        st->done = 1;
                    }
                    continue;
                }
                if (fabs(res - st->epssq) <= st->nband) {  // near: stop before it
                    st->near = 1;
                    st->done = 1;
                    continue;
                }
                const int it = st->it + 1;
                st->res = res;
                st->it = it;
                st->done = !((res >= st->epssq) && (it < st->itermax));
            }
        }
    }
}

__global__ __launch_bounds__(kFinishThreads) void rb_finish_kernel(
    const double* __restrict__ partials, int n, int T, DevState* st, double cells, int decide) {
    __shared__ double sh[kMaxT][kFinishThreads];
    __shared__ double tot[kMaxT];
    if (st->done) return;
    finish_body<false>(partials, n, T, st, cells, decide, sh, tot);
}

// Single-rank loop test, first level: workgroup (c, g) sums chunk c of stage
// g's per-workgroup partials in a fixed order (strided by thread, then a
// tree), so the finish kernel reads kFinishChunks values per stage instead of
// one per sweep workgroup (14k at 32768^2: 65 -> ~10 us per pass)
// count != nullptr: the launch's last workgroup also runs the loop test
// (rb_finish_kernel, one launch per pass instead of two); T, cells: its
// arguments
__global__ __launch_bounds__(256) void rb_partsum_kernel(const double* __restrict__ partials,
                                                         int n, const DevState* __restrict__ st,
                                                         double* __restrict__ out, int* count,
                                                         int T, double cells, int decide,
                                                         int lite) {
    __shared__ double sh[256];
    __shared__ int is_last;
    // (st->done is the same for the whole launch: only its last workgroup
    // writes it, after every other one's add)
    if (st->done) return;
    const int c = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
    const int lo = (int)((long long)n * c / kFinishChunks);
    const int hi = (int)((long long)n * (c + 1) / kFinishChunks);
    const double* q = partials + (long long)g * n;
    double s0 = 0.0, s1 = 0.0;
    int k = lo + t;
    for (; k + 256 < hi; k += 512) {
        s0 += q[k];
        s1 += q[k + 256];
    }
    if (k < hi) s0 += q[k];
    sh[t] = s0 + s1;
    __syncthreads();
#pragma unroll
    for (int w = 128; w >= 64; w >>= 1) {
        if (t < w) sh[t] += sh[t + w];
        __syncthreads();
    }
    if (t < 64) {
        const double v = wave_sum(sh[t]);
        if (t == 0) {
            if (!count) {
                out[g * kFinishChunks + c] = v;
            } else {
                // hand-off to the launch's last workgroup (MISOR_MICROARCH.md
                // valid forms, row 1): an sc1 store, drained, then one lane's
                // agent-scope add to one counter; the workgroup whose add came
                // last reads every value with sc1 loads
                __hip_atomic_store(out + g * kFinishChunks + c, v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int k = __hip_atomic_fetch_add(count, 1, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                is_last = k == (int)(gridDim.x * gridDim.y) - 1;
            }
        }
    }
    if (!count) return;
    __syncthreads();
    if (!is_last) return;
    // the loop test of the pass (rb_finish_kernel), then the counter for the next
    {
        __shared__ double fsh[kMaxT][kFinishThreads];
        __shared__ double tot[kMaxT];
        finish_body<true>(out, kFinishChunks, T, const_cast<DevState*>(st), cells, decide, fsh,
                          tot, lite);
        if (t == 0) __hip_atomic_store(count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

void launch_finish2(hipStream_t s, const double* partials, int nparts, int T, DevState* st,
                    double cells, double* scratch, int* count, int decide, int lite) {
    // (lite: the stages whose sums are lower bounds -- only with the loop test
    // in the last workgroup, count != nullptr)
    hipLaunchKernelGGL(rb_partsum_kernel, dim3(kFinishChunks, T), dim3(256), 0, s, partials,
                       nparts, st, scratch, count, T, cells, decide, count ? lite : 0);
    if (!count)
        hipLaunchKernelGGL(rb_finish_kernel, dim3(1), dim3(kFinishThreads), 0, s, scratch,
                           kFinishChunks, T, st, cells, decide);
}

int sweep_waves(int variant) { return kSweepVariants[variant].waves; }

int sweep_partials(int ni, int nj, int rows_per_block, int waves, int* nbx, int* nby) {
    const int strips = (ni + kStripCells - 1) / kStripCells;
    *nbx = (strips + waves - 1) / waves;
    *nby = (nj + rows_per_block - 1) / rows_per_block;
    return (*nbx) * (*nby);
}

void launch_sweep(hipStream_t s, const SweepParams& prm, const double* src, double* dst,
                  const double* rhs, double* partials, const DevState* st) {
#define SWEEP(W, D, NT, LNT)                                                                \
    hipLaunchKernelGGL((rb_sweep_kernel<W, D, NT, LNT>), dim3(prm.nblocks), dim3(kLanes * W), \
                       0, s, prm, src, dst, rhs, partials, st)
    // must match kSweepVariants (misor_internal.h)
    switch (prm.variant) {
    case 0: SWEEP(4, 1, false, false); break;
    case 1: SWEEP(4, 2, false, false); break;
    case 2: SWEEP(4, 3, false, false); break;
    case 3: SWEEP(4, 1, true, false); break;
    case 4: SWEEP(4, 2, true, false); break;
    case 5: SWEEP(8, 1, false, false); break;
    case 6: SWEEP(8, 2, false, false); break;
    case 7: SWEEP(8, 2, true, false); break;
    case 8: SWEEP(8, 1, true, false); break;
    case 9: SWEEP(8, 3, true, false); break;
    case 10: SWEEP(16, 1, true, false); break;
    case 11: SWEEP(16, 2, true, false); break;
    case 12: SWEEP(4, 3, true, false); break;
    case 13: SWEEP(8, 2, true, true); break;
    case 14: SWEEP(16, 2, true, true); break;
    default: SWEEP(8, 2, true, false); break;
    }
#undef SWEEP
}

void launch_sweep_rsq(hipStream_t s, const SweepParams& prm, const double* src, double* dst,
                      const double* rhs, double* partials, const DevState* st, double* rsq) {
    // the default sweep variant's geometry (kDefaultSweepVariant: 8 strips, 2 rows
    // in flight, nt stores); the exact tail sets up prm with it
    hipLaunchKernelGGL((rb_sweep_kernel<8, 2, true, false, true>), dim3(prm.nblocks),
                       dim3(kLanes * 8), 0, s, prm, src, dst, rhs, partials, st, rsq);
}

void launch_finish(hipStream_t s, const double* partials, int nparts, int T, DevState* st,
                   double cells, int decide) {
    hipLaunchKernelGGL(rb_finish_kernel, dim3(1), dim3(kFinishThreads), 0, s, partials, nparts, T, st,
                       cells, decide);
}

// decomposed runs: st->sum[0..T-1] hold the all-reduced sums r^2 of every rank
// one thread; the state is read once and written once (it runs on the comm
// stream beside a full sweep, where every dependent memory round trip is slow)
// lite: the stages whose sums are lower bounds (finish_body)
__global__ void rb_decide_kernel(DevState* st, int T, double cells, int lite) {
    if (st->done) return;
    double sum[kMaxT];
#pragma unroll
    for (int g = 0; g < kMaxT; ++g) sum[g] = g < T ? st->sum[g] : 0.0;
    const double epssq = st->epssq, nband = st->nband;
    const int itermax = st->itermax;
    int it = st->it, done = 0, near = 0, miss = 0;
    double res = st->res;
    for (int g = 0; g < T && !done; ++g) {
        const double r = sum[g] / cells;
        if ((lite >> g) & 1) {  // a lower bound: proof that the loop goes on, or a miss
            const bool on = nband >= 0.0 ? r > epssq + nband : r >= epssq;
            if (on && it + 1 < itermax) {
                res = r;
                ++it;
                continue;
            }
            miss = done = 1;
            break;
        }
        if (fabs(r - epssq) <= nband) {  // near the threshold: stop before this iteration
            near = done = 1;
            break;
        }
        res = r;
        ++it;
        done = !((res >= epssq) && (it < itermax));
    }
    st->res = res;
    st->it = it;
    st->done = done;
    st->near = near;
    if (miss) st->lite_miss = 1;
}

void launch_decide(hipStream_t s, DevState* st, int T, double cells, int lite) {
    hipLaunchKernelGGL(rb_decide_kernel, dim3(1), dim3(1), 0, s, st, T, cells, lite);
}

// ---------------------------------------------------------------------------
// Small grids (the NS cases: 128^2 dcavity, 200x50 canal, 100^2 poisson.par):
// the whole solveRB loop in ONE workgroup, p resident in LDS.
//
// At these sizes a sweep moves ~0.4 MB and is pure launch/latency cost on
// the multi-block path (two launches per iteration); here an iteration is
// two LDS passes and a block reduction, with no launch and no host round
// trip until convergence.  In-place red then black pass, exactly solveRB's
// order of dependencies (assignment-4/src/solver.c:201-217), ghost copy rows
// then columns (:219-227), res = sum / (imax*jmax) and the same loop test.
// Each thread owns fixed (red, black) cell pairs, so its rhs values stay in
// registers for the whole solve.
// ---------------------------------------------------------------------------
constexpr int kSmallThreads = 1024;
constexpr int kSmallMaxPairs = 8;  // pairs per thread (128^2: exactly 8)

int small_solve_fits(int ni, int nj) {
    const long long cells = (long long)(ni + 2) * (nj + 2);
    const long long pairs = (long long)nj * ((ni + 1) / 2);
    return cells * 8 + 256 <= 160 * 1024 && pairs <= (long long)kSmallThreads * kSmallMaxPairs;
}

__global__ __launch_bounds__(kSmallThreads) void rb_solve_small_kernel(
    double* __restrict__ p_glob, const double* __restrict__ rhs_glob, int ni, int nj,
    long long pitch, double idx2, double idy2, double coef, double cells, DevState* st) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* red = lds;          // 16 wave partials + broadcast slot
    double* P = lds + 32;       // (ni+2) x (nj+2), row stride ni+2
    const int W = ni + 2;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const long long ncell = (long long)W * (nj + 2);

    for (long long k = t; k < ncell; k += kSmallThreads) {
        const int i = (int)(k % W), j = (int)(k / W);
        P[k] = p_glob[(long long)(j + kYOff) * pitch + (i + kXOff)];
    }
    // this thread's pairs: pair e covers columns 1+2m, 2+2m of row 1 + e / half
    const int half = (ni + 1) / 2;
    const int npairs = nj * half;
    int ci[kSmallMaxPairs][2];  // LDS index of (colour-0 cell, colour-1 cell), -1: none
    double rh[kSmallMaxPairs][2];
#pragma unroll
    for (int m = 0; m < kSmallMaxPairs; ++m) {
        const int e = t + m * kSmallThreads;
        ci[m][0] = ci[m][1] = -1;
        rh[m][0] = rh[m][1] = 0.0;
        if (e < npairs) {
            const int j = 1 + e / half, i0 = 1 + 2 * (e % half);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                // colour c cell of this pair: (i + j) & 1 == c
                const int i = ((i0 + j) & 1) == c ? i0 : i0 + 1;
                if (i <= ni) {
                    ci[m][c] = j * W + i;
                    rh[m][c] = rhs_glob[(long long)(j + kYOff) * pitch + (i + kXOff)];
                }
            }
        }
    }
    __syncthreads();

    const double epssq = st->epssq, nband = st->nband;
    const int itermax = st->itermax;
    double res = st->res;
    int it = st->it, near = 0;
    while ((res >= epssq) && (it < itermax)) {
        double acc = 0.0;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#pragma unroll
            for (int m = 0; m < kSmallMaxPairs; ++m) {
                const int k = ci[m][c];
                if (k >= 0) {
                    const double cc = P[k];
                    const double r = rh[m][c] - (((P[k + 1] - 2.0 * cc) + P[k - 1]) * idx2 +
                                                 ((P[k + W] - 2.0 * cc) + P[k - W]) * idy2);
                    P[k] = cc - coef * r;
                    acc += r * r;
                }
            }
            __syncthreads();
        }
        // Neumann ghost copy: rows, then columns (corners untouched)
        for (int i = 1 + t; i <= ni; i += kSmallThreads) {
            P[i] = P[W + i];
            P[(nj + 1) * W + i] = P[nj * W + i];
        }
        __syncthreads();
        for (int j = 1 + t; j <= nj; j += kSmallThreads) {
            P[j * W] = P[j * W + 1];
            P[j * W + ni + 1] = P[j * W + ni];
        }
        // fixed-order block sum of r^2
        acc = wave_sum(acc);
        if (lane == 0) red[wave] = acc;
        __syncthreads();
        if (t == 0) {
            double s = 0.0;
            for (int w = 0; w < kSmallThreads / 64; ++w) s += red[w];
            red[16] = s;
        }
        __syncthreads();
        const double rn = red[16] / cells;
        if (fabs(rn - epssq) <= nband) {  // near the threshold: p is left as it was;
            near = 1;                      // the host reruns up to it iterations
            break;
        }
        res = rn;
        ++it;
    }

    if (!near) {
        for (long long k = t; k < ncell; k += kSmallThreads) {
            const int i = (int)(k % W), j = (int)(k / W);
            p_glob[(long long)(j + kYOff) * pitch + (i + kXOff)] = P[k];
        }
    }
    if (t == 0) {
        st->it = it;
        st->res = res;
        st->done = 1;
        st->near = near;
    }
}

void launch_solve_small(hipStream_t s, double* p, const double* rhs, int ni, int nj,
                        long long pitch, double idx2, double idy2, double coef, double cells,
                        DevState* st) {
    const size_t lds = sizeof(double) * (32 + (size_t)(ni + 2) * (nj + 2));
    (void)hipFuncSetAttribute((const void*)rb_solve_small_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(rb_solve_small_kernel, dim3(1), dim3(kSmallThreads), lds, s, p, rhs, ni,
                       nj, pitch, idx2, idy2, coef, cells, st);
}

// ---------------------------------------------------------------------------
// Field initialisation
// ---------------------------------------------------------------------------

__global__ void fill_kernel(double* a, long long n, double v) {
    long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (; k < n; k += stride) a[k] = v;
}

void launch_fill(hipStream_t s, double* a, long long n, double v) {
    long long blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, n, v);
}

// assignment-4/src/solver.c:105-123: P(i,j) = sin(4 pi i dx) + sin(4 pi j dy),
// RHS(i,j) = sin(2 pi i dx) (problem 2) else 0, for all cells incl. ghosts.
// The sines come from host tables evaluated with libm exactly as the
// reference evaluates them; the sum of two doubles is correctly rounded on
// both sides, so the device field is bit-identical to the CPU's.
__global__ void poisson_init_kernel(double* p, double* rhs, const double* sx, const double* sy,
                                    const double* rx, int ni, int nj, long long pitch,
                                    int problem) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y;
    if (i > ni + 1 || j > nj + 1) return;
    const long long k = (long long)(j + kYOff) * pitch + (i + kXOff);
    p[k] = sx[i] + sy[j];
    rhs[k] = (problem == 2) ? rx[i] : 0.0;
}

void launch_poisson_init(hipStream_t s, double* p, double* rhs, const double* sx,
                         const double* sy, const double* rx, int ni, int nj, long long pitch,
                         int problem) {
    dim3 grid((ni + 2 + 255) / 256, nj + 2);
    hipLaunchKernelGGL(poisson_init_kernel, grid, dim3(256), 0, s, p, rhs, sx, sy, rx, ni, nj,
                       pitch, problem);
}

}  // namespace misor
