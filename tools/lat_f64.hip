// lat_f64.hip -- issue cost and dependent-chain latency of FP64 VALU ops on
// gfx950 (a diagnostic, not part of the library): every wave runs C
// independent chains of n dependent v_fma_f64 each; cycles per instruction
// per wave from s_memtime, for 1..4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/lat_f64.hip -o /tmp/lat_f64 && /tmp/lat_f64
#include <hip/hip_runtime.h>

#include <cstdio>

template <int C>
__global__ void chains(double* out, long long* cyc, int n, double a) {
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = threadIdx.x * 1e-3 + c;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = __builtin_fma(x[c], a, 1e-9);
        }
    }
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

// the tb stage's pattern: 2 v_mov_dpp + fma chain of depth 7 with one side branch
__global__ void dppchain(double* out, long long* cyc, int n, double a) {
    double v = threadIdx.x * 1e-3, w = 0.5;
    const long long t0 = clock64();
    for (int i = 0; i < n * 8; ++i) {
        const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
        const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
        const double f = __hiloint2double(hi, lo);
        v = __builtin_fma(-2.0, v, f) * a + w;
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <class K>
static void run(const char* name, K kern, int C, int waves_per_simd) {
    const int n = 4096, threads = 256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd;
    const int blocks = 256 * (256 * waves_per_simd / threads);
    double* out;
    long long* cyc;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, cyc, n, 0.999);
    hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    long long* h = new long long[nw];
    hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < nw; ++i) s += h[i];
    const double per_wave = s / nw / (8.0 * n * (C > 0 ? C : 1));
    printf("%-10s C=%d waves/SIMD=%d: %.2f cycles per instruction per wave, %.2f per SIMD\n", name, C,
           waves_per_simd, per_wave, per_wave / waves_per_simd);
    delete[] h;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 4; w *= 2) {
        run("fma_f64", chains<1>, 1, w);
        run("fma_f64", chains<2>, 2, w);
        run("fma_f64", chains<4>, 4, w);
        run("fma_f64", chains<8>, 8, w);
        run("dpp+fma", dppchain, 0, w);
    }
    return 0;
}
