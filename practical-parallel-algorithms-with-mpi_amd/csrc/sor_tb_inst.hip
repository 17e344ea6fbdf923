// sor_tb_inst.hip -- the kernels of ONE pass length T = MISOR_TB_T (compiled
// once per T by the Makefile: build/sor_tb_t<T>.o).  Device code: sor_tb.h.
#include <algorithm>

#include "sor_tb.h"
#include "sor_tbh.h"

#ifndef MISOR_TB_T
#error "compile with -DMISOR_TB_T=<iterations per pass>"
#endif
#define MISOR_CAT2(a, b) a##b
#define MISOR_CAT(a, b) MISOR_CAT2(a, b)

namespace misor {

// workgroups of a persistent launch: as many as are resident at once
template <class K>
static int persistent_grid(K kernel, int threads) {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0);
    return std::max(8, per_cu * cus);
}

template <int T, int W, int D, bool B>
static int resident2() {
    static int n = 0;
    if (n == 0) n = persistent_grid(rb_tb_kernel<T, W, D, B, false>, kLanes * W);
    return n;
}

template <int T, int W, int D, bool P2, int E>
static int resident_chain() {
    static int n = 0;
    if (n == 0) n = persistent_grid(rb_tbc_kernel<T, W, D, P2, E>, kLanes * W);
    return n;
}

template <int T, int W, int D, bool P2, int SK>
static int residenthc() {
    static int n = 0;
    if (n == 0) n = persistent_grid(rb_tbhc_kernel<T, W, D, P2, SK, 0>, kLanes * W);
    return n;
}

constexpr int kT = MISOR_TB_T;
void MISOR_CAT(launch_tb_t, MISOR_TB_T)(hipStream_t s, const SweepParams& prm,
                                        const double* src, double* dst, const double* rhs,
                                        double* partials, const DevState* st, int force,
                                        int* queue) {
    auto go = [&](auto kernel, int threads, int resident) {
        int grid = prm.nblocks;
        // (queue: zero at creation, reset by the kernel's last workgroup)
        if (queue) grid = std::min(grid, std::max(8, resident - prm.reserve));
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, prm, src, dst, rhs, partials,
                           st, force, queue);
    };
    if (prm.variant == kHrTbVariant) {  // skewed (tb_ring_slots: T = 1 runs unskewed)
        constexpr int SK_ = kT >= 2 ? 1 : 0;
        {
            // the chained split-ring pass (sor_tbh.h rb_tbhc_kernel; configure_tb
            // keeps its passes chained and persistent): the work area gets the
            // launch's initial segment list (as the chained pass below), unless
            // the caller initialised it before the edge kernel (no_init)
            if (!prm.no_init) launch_chain_init(s, queue, prm.seg_tmpl, prm.nseg0, prm.seg_cap);
            auto gc = [&](auto kernel, int resident) {
                const int grid = std::min(prm.chain_blocks, std::max(8, resident - prm.reserve));
                hipLaunchKernelGGL(kernel, dim3(grid), dim3(kLanes * 4), 0, s, prm, src, dst, rhs,
                                   partials, st, force, queue);
            };
            // (one kernel for the main and the edge list: a strip at a physical
            // side marches block by block, the workgroup's other strips chain)
            const int res = residenthc<kT, 4, 2, false, SK_>();
            if constexpr (kT == kShortT) {  // (the residual lower bound: the short plan's T)
                if (prm.lite) {
                    if (prm.pow2) gc(rb_tbhc_kernel<kT, 4, 2, true, SK_, 0, true>, res);
                    else          gc(rb_tbhc_kernel<kT, 4, 2, false, SK_, 0, true>, res);
                    return;
                }
            }
            if (prm.pow2) gc(rb_tbhc_kernel<kT, 4, 2, true, SK_, 0>, res);
            else          gc(rb_tbhc_kernel<kT, 4, 2, false, SK_, 0>, res);
            return;
        }
    }
    // the 2- and 4-column register-ring kernels: T <= kMaxT2 (configure_tb)
    if constexpr (kT <= kMaxT2) {
        if (prm.chain && queue && prm.variant == 0) {
            // chained pass (sor_tb.h rb_tbc_kernel): the work area gets the launch's
            // initial segment list; as many workgroups as are resident (less the
            // reserve), at most one per block
            launch_chain_init(s, queue, prm.seg_tmpl, prm.nseg0, prm.seg_cap);
            auto gc = [&](auto kernel, int resident) {
                const int grid = std::min(prm.chain_blocks, std::max(8, resident - prm.reserve));
                hipLaunchKernelGGL(kernel, dim3(grid), dim3(kLanes * 4), 0, s, prm, src, dst, rhs,
                                   partials, st, force, queue);
            };
            // main kernel, or the edge kernel (columns at a physical left / right side)
            if (prm.chain_edge) {
                if (prm.pow2) gc(rb_tbc_kernel<kT, 4, 2, true, 1>, resident_chain<kT, 4, 2, true, 1>());
                else          gc(rb_tbc_kernel<kT, 4, 2, false, 1>, resident_chain<kT, 4, 2, false, 1>());
            } else {
                if (prm.pow2) gc(rb_tbc_kernel<kT, 4, 2, true, 0>, resident_chain<kT, 4, 2, true, 0>());
                else          gc(rb_tbc_kernel<kT, 4, 2, false, 0>, resident_chain<kT, 4, 2, false, 0>());
            }
            return;
        }
        if (prm.variant == 2) {  // 2 strips per workgroup (finer slots for small rank blocks)
            if (prm.pow2) go(rb_tb_kernel<kT, 2, 2, false, true>, kLanes * 2, resident2<kT, 2, 2, false>());
            else go(rb_tb_kernel<kT, 2, 2, false, false>, kLanes * 2, resident2<kT, 2, 2, false>());
        } else {  // the default (kTbVariants: every other built variant is 13, above)
            if (prm.pow2) go(rb_tb_kernel<kT, 4, 2, false, true>, kLanes * 4, resident2<kT, 4, 2, false>());
            else go(rb_tb_kernel<kT, 4, 2, false, false>, kLanes * 4, resident2<kT, 4, 2, false>());
        }
    }
}

int MISOR_CAT(tb_resident_t, MISOR_TB_T)(int variant) {
    if (variant == kHrTbVariant) return residenthc<kT, 4, 2, false, kT >= 2 ? 1 : 0>();
    if constexpr (kT <= kMaxT2)
        return variant == 2 ? resident2<kT, 2, 2, false>() : resident2<kT, 4, 2, false>();
    return 0;
}

}  // namespace misor
