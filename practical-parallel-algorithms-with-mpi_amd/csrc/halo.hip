// halo.hip -- pack / unpack of the 8-neighbour halo regions of one field into
// contiguous buffers for RCCL send/recv (columns are strided in HBM, so every
// region goes through the buffer; one launch packs all eight).
//
// Region sizes at the 32768^2, 8-GPU (4x2) configuration with the 2-deep p
// halo: left/right 2 x 16386 doubles (256 KiB), bottom/top 2 x 8194 (128 KiB),
// corners 2 x 2.  Bandwidth is irrelevant here; the launches are
// latency-bound (a few microseconds each).

#include "misor_internal.h"

namespace misor {

namespace {

template <bool PACK>
__global__ void halo_copy_kernel(double* field, long long pitch, HaloPlan plan, double* buf) {
    const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const HaloRegion* R = PACK ? plan.send : plan.recv;
    // find the region that holds packed element k (8 regions, in offset order)
#pragma unroll
    for (int d = 0; d < kDirs; ++d) {
        const HaloRegion r = R[d];
        const long long n = (long long)r.w * r.h;
        if (n > 0 && k >= r.off && k < r.off + n) {
            const long long e = k - r.off;
            const int i = r.x0 + (int)(e % r.w), j = r.y0 + (int)(e / r.w);
            double* cell = field + (long long)(j + kYOff) * pitch + (i + kXOff);
            if (PACK)
                buf[k] = *cell;
            else
                *cell = buf[k];
        }
    }
}

}  // namespace

void launch_pack(hipStream_t s, const double* field, long long pitch, const HaloPlan& plan,
                 double* sendbuf) {
    if (plan.total <= 0) return;
    const unsigned blocks = (unsigned)((plan.total + 255) / 256);
    hipLaunchKernelGGL(halo_copy_kernel<true>, dim3(blocks), dim3(256), 0, s,
                       const_cast<double*>(field), pitch, plan, sendbuf);
}

void launch_unpack(hipStream_t s, double* field, long long pitch, const HaloPlan& plan,
                   const double* recvbuf) {
    if (plan.total <= 0) return;
    const unsigned blocks = (unsigned)((plan.total + 255) / 256);
    hipLaunchKernelGGL(halo_copy_kernel<false>, dim3(blocks), dim3(256), 0, s, field, pitch,
                       plan, const_cast<double*>(recvbuf));
}

// in-process transport's all-reduce: gather[q * kMaxT + k] holds rank q's
// value k; every rank combines them in rank order (identical bits everywhere)
__global__ void local_combine_kernel(const double* gather, int nranks, int n, int is_max,
                                     double* out) {
    const int k = threadIdx.x;
    if (k >= n) return;
    double a = gather[k];
    for (int q = 1; q < nranks; ++q) {
        const double b = gather[q * kMaxT + k];
        a = is_max ? ((a > b) ? a : b) : a + b;
    }
    out[k] = a;
}

void launch_local_combine(hipStream_t s, const double* gather, int nranks, int n, int is_max,
                          double* out) {
    hipLaunchKernelGGL(local_combine_kernel, dim3(1), dim3(kMaxT), 0, s, gather, nranks, n,
                       is_max, out);
}

}  // namespace misor
