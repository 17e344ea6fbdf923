// fp64_issue.hip -- microbenchmark: FP64 VALU issue rate and dependent latency
// on gfx950 at 1 / 2 waves per SIMD, with the in-kernel clock.  Each lane runs
// K independent chains of the logistic map (x = r * fma(-x, x, x): two
// dependent FP64 operations per link, chaotic so the operand bits toggle as in
// a real stencil).  One workgroup per CU (LDS padding), 4 or 8 waves.
// Build: hipcc --offload-arch=gfx950 -O3 -o fp64_issue fp64_issue.hip
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

template <int K, int DPP>
__global__ void __launch_bounds__(1024) chains(double* out, long long* clk, int iters, double r) {
    __shared__ double pad[18000];  // > 80 KB: one workgroup per CU
    double x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = 0.1 + 0.8 * ((threadIdx.x * 7 + k * 13 + blockIdx.x) % 97) / 97.0;
    long long t0 = __builtin_amdgcn_s_memtime();
    long long w0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (DPP == 2) {  // one FMA per link: x = x^2 - 1.9 (chaotic on [-2, 2])
                x[k] = __builtin_fma(x[k], x[k], -1.9);
                continue;
            }
            double t = __builtin_fma(-x[k], x[k], x[k]);
            if (DPP) {
                // a 64-bit lane shift (two v_mov_b32_dpp) mixed in every link
                const double s = __hiloint2double(
                    __builtin_amdgcn_mov_dpp(__double2hiint(t), 0x138, 0xf, 0xf, true),
                    __builtin_amdgcn_mov_dpp(__double2loint(t), 0x138, 0xf, 0xf, true));
                t = (t + s) * 0.5;
            }
            x[k] = r * t;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    long long w1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    if (s == 12345.0) pad[threadIdx.x] = s;  // never
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + pad[0] * 0;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = w1 - w0;
    }
}

template <int K, int DPP>
int run(int waves, int iters, int ncu) {
    const int threads = 64 * waves;
    const int blocks = ncu;
    double* out;
    long long* clk;
    CK(hipMalloc(&out, sizeof(double) * blocks * threads));
    CK(hipMalloc(&clk, sizeof(long long) * 2 * blocks));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep)
        chains<K, DPP><<<blocks, threads>>>(out, clk, iters / 4, 3.9);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    chains<K, DPP><<<blocks, threads>>>(out, clk, iters, 3.9);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<long long> h(2 * blocks);
    CK(hipMemcpy(h.data(), clk, sizeof(long long) * 2 * blocks, hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    for (int i = 0; i < blocks; ++i) ghz.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 0.1);
    std::sort(ghz.begin(), ghz.end());
    // FP64 wave-instructions per SIMD: waves/SIMD x iters x K x ops per link
    const int ops = DPP == 2 ? 1 : DPP ? 4 : 2;  // fma, mul (+ add, mul); dpp movs counted apart
    const double winst = (double)(waves / 4) * iters * K * ops;
    const double ghz_med = ghz[blocks / 2];
    const double cyc = ms * 1e-3 * ghz_med * 1e9;
    printf("K=%d dpp=%d waves/SIMD=%d  %.3f ms  clock %.3f GHz  FP64 wave-inst/SIMD %.3g  "
           "cycles per FP64 wave-inst %.2f  (%.2f at 2.4 GHz)\n",
           K, DPP, waves / 4, ms, ghz_med, winst, cyc / winst, ms * 1e-3 * 2.4e9 / winst);
    fflush(stdout);
    CK(hipFree(out));
    CK(hipFree(clk));
    return 0;
}

int main() {
    int ncu = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
    printf("CUs %d\n", ncu);
    const int iters = 100000;
    for (int w : {4, 8, 12, 16}) {
        run<4, 2>(w, iters, ncu);
        run<8, 2>(w, iters, ncu);
        run<16, 2>(w, iters, ncu);
        run<8, 0>(w, iters, ncu);
        run<16, 0>(w, iters, ncu);
        run<8, 1>(w, iters, ncu);
    }
    return 0;
}
