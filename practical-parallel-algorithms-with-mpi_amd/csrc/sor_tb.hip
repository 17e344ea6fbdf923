// sor_tb.hip -- host side of the temporally blocked sweep: strip geometry and
// the launch dispatch over T (each T's kernels are instantiated in its own
// unit, sor_tb_inst.hip compiled with MISOR_TB_T = T, so the build runs in
// parallel).  Device code: sor_tb.h.
#include <algorithm>

#include "misor_internal.h"

namespace misor {

int tb_max_t(int variant) { return kTbVariants[variant].max_t; }

int tb_out_width(int T, int /*variant*/) { return kStripCells - 4 * T; }

int tb_waves(int variant) { return kTbVariants[variant].waves; }

int tb_ring_slots(int T, int variant) {
    const int D = kTbVariants[variant].ahead;
    if (kTbVariants[variant].hr) return hr_slots(T, D, kTbVariants[variant].skew && T >= 2 ? 1 : 0);
    return 2 * T + D + (D & 1);  // sor_tb.h ring_slots
}

int tb_nbx(int ni, int T, int variant) {
    const int ow = tb_out_width(T, variant);
    const int strips = (ni + ow - 1) / ow;
    const int waves = tb_waves(variant);
    return (strips + waves - 1) / waves;
}

__global__ void chain_init_kernel(int* work, const unsigned long long* tmpl, int nseg0,
                                  int cap) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long* seg = reinterpret_cast<unsigned long long*>(work + kChainHead);
    if (k < kChainHead) work[k] = 0;
    if (k < nseg0) seg[k] = tmpl[k];
    else if (k < nseg0 + cap) seg[k] = 0ull;
}

void launch_chain_init(hipStream_t s, int* work, const unsigned long long* tmpl, int nseg0,
                       int cap) {
    const int n = std::max(kChainHead, nseg0 + cap);
    hipLaunchKernelGGL(chain_init_kernel, dim3((n + 255) / 256), dim3(256), 0, s, work, tmpl,
                       nseg0, cap);
}

void launch_tb(hipStream_t s, int T, const SweepParams& prm, const double* src, double* dst,
               const double* rhs, double* partials, const DevState* st, int force, int* queue) {
    switch (T) {
#define C(N)                                                                \
    case N: launch_tb_t##N(s, prm, src, dst, rhs, partials, st, force, queue); break;
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9)
#undef C
    default: launch_tb_t10(s, prm, src, dst, rhs, partials, st, force, queue); break;
    }
}

int tb_resident(int T, int variant) {
    switch (T) {
#define C(N) \
    case N: return tb_resident_t##N(variant);
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9)
#undef C
    default: return tb_resident_t10(variant);
    }
}

}  // namespace misor
