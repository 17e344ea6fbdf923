// fp64_lat.hip -- microbenchmark: issue cost and dependent latency of the FP64
// VALU instructions of the SOR stage (v_fma_f64, v_add_f64) and of the DPP
// lane shift (v_mov_b32_dpp), on gfx950, at 1 and 2 waves per SIMD.
//
// Each wave runs `iters` times a straight-line inline-asm block of 32
// instructions over K independent chains (instruction i writes chain i mod K
// and reads it: K = 1 is one dependent chain, K = 8 eight interleaved ones).
// Cycles come from s_memtime (the shader clock) around the loop in each
// wave; the clock from s_memtime / s_memrealtime (MI355X_MICROARCH.md 503).
// One workgroup per CU (LDS padding); 4 waves = 1 per SIMD, 8 = 2 per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o fp64_lat.bin fp64_lat.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            return 1;                                                          \
        }                                                                      \
    } while (0)

// 32 instructions on chains x0..x7 (k = i mod K)
#define R4(a, b, c, d) a b c d
#define FMA(k) "v_fma_f64 %" #k ", %" #k ", %8, %9\n"
#define ADD(k) "v_add_f64 %" #k ", %" #k ", %8\n"
// a lane shift of chain k = 1..4 (fixed registers v[1k0:1k1], both halves,
// wave_shr:1) folded back by an add; tmp v[1k2:1k3]
#define DPA(k)                                                                              \
    "v_mov_b32_dpp v1" #k "2, v1" #k "0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"   \
    "v_mov_b32_dpp v1" #k "3, v1" #k "1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"   \
    "v_add_f64 v[1" #k "0:1" #k "1], v[1" #k "0:1" #k "1], v[1" #k "2:1" #k "3]\n"
#define DCLOB "v110", "v111", "v112", "v113", "v120", "v121", "v122", "v123", "v130", \
              "v131", "v132", "v133", "v140", "v141", "v142", "v143"

template <int OP, int K>
__device__ __forceinline__ void block32(double (&x)[8], double a, double b, double& tmp) {
    // OP 0: fma, 1: add, 2: dpp pair + add (3 instructions per link, 10 links + 2 adds)
    if (OP == 0) {
        if (K == 1)
            asm volatile(R4(R4(FMA(0), FMA(0), FMA(0), FMA(0)), R4(FMA(0), FMA(0), FMA(0), FMA(0)),
                            R4(FMA(0), FMA(0), FMA(0), FMA(0)), R4(FMA(0), FMA(0), FMA(0), FMA(0)))
                             R4(R4(FMA(0), FMA(0), FMA(0), FMA(0)), R4(FMA(0), FMA(0), FMA(0), FMA(0)),
                                R4(FMA(0), FMA(0), FMA(0), FMA(0)), R4(FMA(0), FMA(0), FMA(0), FMA(0)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
        else if (K == 2)
            asm volatile(R4(R4(FMA(0), FMA(1), FMA(0), FMA(1)), R4(FMA(0), FMA(1), FMA(0), FMA(1)),
                            R4(FMA(0), FMA(1), FMA(0), FMA(1)), R4(FMA(0), FMA(1), FMA(0), FMA(1)))
                             R4(R4(FMA(0), FMA(1), FMA(0), FMA(1)), R4(FMA(0), FMA(1), FMA(0), FMA(1)),
                                R4(FMA(0), FMA(1), FMA(0), FMA(1)), R4(FMA(0), FMA(1), FMA(0), FMA(1)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
        else if (K == 4)
            asm volatile(R4(R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(0), FMA(1), FMA(2), FMA(3)),
                            R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(0), FMA(1), FMA(2), FMA(3)))
                             R4(R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(0), FMA(1), FMA(2), FMA(3)),
                                R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(0), FMA(1), FMA(2), FMA(3)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
        else
            asm volatile(R4(R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(4), FMA(5), FMA(6), FMA(7)),
                            R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(4), FMA(5), FMA(6), FMA(7)))
                             R4(R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(4), FMA(5), FMA(6), FMA(7)),
                                R4(FMA(0), FMA(1), FMA(2), FMA(3)), R4(FMA(4), FMA(5), FMA(6), FMA(7)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
    } else if (OP == 1) {
        if (K == 1)
            asm volatile(R4(R4(ADD(0), ADD(0), ADD(0), ADD(0)), R4(ADD(0), ADD(0), ADD(0), ADD(0)),
                            R4(ADD(0), ADD(0), ADD(0), ADD(0)), R4(ADD(0), ADD(0), ADD(0), ADD(0)))
                             R4(R4(ADD(0), ADD(0), ADD(0), ADD(0)), R4(ADD(0), ADD(0), ADD(0), ADD(0)),
                                R4(ADD(0), ADD(0), ADD(0), ADD(0)), R4(ADD(0), ADD(0), ADD(0), ADD(0)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
        else if (K == 2)
            asm volatile(R4(R4(ADD(0), ADD(1), ADD(0), ADD(1)), R4(ADD(0), ADD(1), ADD(0), ADD(1)),
                            R4(ADD(0), ADD(1), ADD(0), ADD(1)), R4(ADD(0), ADD(1), ADD(0), ADD(1)))
                             R4(R4(ADD(0), ADD(1), ADD(0), ADD(1)), R4(ADD(0), ADD(1), ADD(0), ADD(1)),
                                R4(ADD(0), ADD(1), ADD(0), ADD(1)), R4(ADD(0), ADD(1), ADD(0), ADD(1)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
        else if (K == 4)
            asm volatile(R4(R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(0), ADD(1), ADD(2), ADD(3)),
                            R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(0), ADD(1), ADD(2), ADD(3)))
                             R4(R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(0), ADD(1), ADD(2), ADD(3)),
                                R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(0), ADD(1), ADD(2), ADD(3)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
        else
            asm volatile(R4(R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(4), ADD(5), ADD(6), ADD(7)),
                            R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(4), ADD(5), ADD(6), ADD(7)))
                             R4(R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(4), ADD(5), ADD(6), ADD(7)),
                                R4(ADD(0), ADD(1), ADD(2), ADD(3)), R4(ADD(4), ADD(5), ADD(6), ADD(7)))
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),
                           "+v"(x[6]), "+v"(x[7])
                         : "v"(a), "v"(b));
    } else {
        // 10 links of (2 dpp + add) + 2 dpp = 32 instructions, chains rotating over K
        // register groups 1..4 (v1x0.. / v2x0.. / ...)
        if (K == 1)
            asm volatile(R4(DPA(1), DPA(1), DPA(1), DPA(1)) R4(DPA(1), DPA(1), DPA(1), DPA(1))
                             DPA(1) DPA(1)
                         "v_mov_b32_dpp v112, v110 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_mov_b32_dpp v113, v111 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         ::: DCLOB);
        else if (K == 2)
            asm volatile(R4(DPA(1), DPA(2), DPA(1), DPA(2)) R4(DPA(1), DPA(2), DPA(1), DPA(2))
                             DPA(1) DPA(2)
                         "v_mov_b32_dpp v112, v110 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_mov_b32_dpp v113, v111 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         ::: DCLOB);
        else
            asm volatile(R4(DPA(1), DPA(2), DPA(3), DPA(4)) R4(DPA(1), DPA(2), DPA(3), DPA(4))
                             DPA(1) DPA(2)
                         "v_mov_b32_dpp v112, v110 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         "v_mov_b32_dpp v113, v111 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                         ::: DCLOB);
    }
}

template <int OP, int K>
__global__ void __launch_bounds__(1024) lat(double* out, long long* clk, int iters) {
    __shared__ double pad[12000];  // > 80 KB: one workgroup per CU
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = 0.3 + 0.01 * k + 1e-6 * threadIdx.x;
    const double a = 0.5, b = 0.25;
    double tmp = 0.0;
    __builtin_amdgcn_sched_barrier(0);
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long w0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    if (OP == 2)
        asm volatile("v_mov_b64 v[110:111], %0\nv_mov_b64 v[120:121], %0\n"
                     "v_mov_b64 v[130:131], %0\nv_mov_b64 v[140:141], %0\n" ::"v"(x[0])
                     : DCLOB);
    for (int it = 0; it < iters; ++it) block32<OP, K>(x, a, b, tmp);
    if (OP == 2) asm volatile("v_add_f64 %0, %0, v[110:111]" : "+v"(x[1])::DCLOB);
    __builtin_amdgcn_sched_barrier(0);
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long w1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
    if (s == 12345.0) pad[threadIdx.x] = s;  // never
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + pad[0] * 0;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = w1 - w0;
    }
}

template <int OP, int K>
int run(int waves, int iters, int ncu) {
    const int threads = 64 * waves, blocks = ncu, nw = blocks * waves;
    double* out;
    long long* clk;
    CK(hipMalloc(&out, sizeof(double) * blocks * threads));
    CK(hipMalloc(&clk, sizeof(long long) * 2 * nw));
    for (int rep = 0; rep < 20; ++rep) lat<OP, K><<<blocks, threads>>>(out, clk, iters);  // warm clock
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    lat<OP, K><<<blocks, threads>>>(out, clk, iters);
    CK(hipEventRecord(e1));
    CK(hipDeviceSynchronize());
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> h(2 * nw);
    CK(hipMemcpy(h.data(), clk, sizeof(long long) * 2 * nw, hipMemcpyDeviceToHost));
    std::vector<double> cyc, ghz;
    for (int i = 0; i < nw; ++i) {
        cyc.push_back((double)h[2 * i]);
        ghz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 0.1);
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(ghz.begin(), ghz.end());
    const double per = cyc[nw / 2] / ((double)iters * 32);
    const char* name = OP == 0 ? "v_fma_f64" : OP == 1 ? "v_add_f64" : "dpp2+add";
    // the launch as a whole: SIMD cycles (event time x median clock) per
    // wave-instruction issued on that SIMD
    const double simd = ms * 1e-3 * ghz[nw / 2] * 1e9 / ((double)(waves / 4) * iters * 32);
    printf("%-10s chains %d  waves/SIMD %d  cycles per instruction per wave %.2f  "
           "(SIMD: %.2f per instruction; launch %.3f ms -> %.2f)  clock %.3f GHz\n",
           name, K, waves / 4, per, per / (waves / 4), ms, simd, ghz[nw / 2]);
    fflush(stdout);
    CK(hipFree(out));
    CK(hipFree(clk));
    return 0;
}

int main() {
    int ncu = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
    printf("CUs %d; 32 instructions per block; s_memtime cycles per wave, median over waves\n", ncu);
    const int iters = 20000;
    for (int w : {4, 8, 12, 16}) {
        run<0, 1>(w, iters, ncu);
        run<0, 2>(w, iters, ncu);
        run<0, 4>(w, iters, ncu);
        run<0, 8>(w, iters, ncu);
        run<1, 1>(w, iters, ncu);
        run<1, 2>(w, iters, ncu);
        run<1, 4>(w, iters, ncu);
        run<1, 8>(w, iters, ncu);
        if (w > 12) continue;  // the DPP form holds 144 VGPRs: at most 3 waves per SIMD
        run<2, 1>(w, iters, ncu);
        run<2, 2>(w, iters, ncu);
        run<2, 4>(w, iters, ncu);
    }
    return 0;
}
