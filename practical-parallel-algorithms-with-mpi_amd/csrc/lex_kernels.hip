// lex_kernels.hip -- the reference's lexicographic Gauss-Seidel SOR `solve`
// (assignment-4/src/solver.c:126-177; the NS version in
// assignment-5/sequential/src/solver.c:140-191) on the GPU, bit for bit.
//
// This is the ordering the reference's programs actually call (its committed
// p.dat / pressure.dat / velocity.dat come from it).  Cell (i,j) uses the NEW
// values of (i-1,j) and (i,j-1) and the OLD values of (i+1,j) and (i,j+1), so
// every cell of one anti-diagonal i+j = d can be updated at once once diagonal
// d-1 is done: one workgroup sweeps the diagonals 2 .. ni+nj with a barrier
// between them, with the reference's exact expression order per cell (two
// x/y orders: `xorder` 0 = assignment-4, 1 = assignment-5 sequential).  After
// the sweep: the Neumann ghost copy (rows, then columns), res = sum r^2 /
// (imax*jmax), the same loop test.  p lives in LDS when it fits (the NS and
// Poisson .par grids), in HBM otherwise.  Inherently sequential: this mode is
// for reproducing the reference's lexicographic results exactly, not for
// speed (the red-black kernels are the production path).

#include "misor_internal.h"

namespace misor {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace

// threads of the one workgroup: the longest anti-diagonal rounded up to whole
// waves (at most 1024): a barrier per diagonal costs less across fewer waves
// (the reference's 100 x 100 NS grid: 2 waves instead of 16)
constexpr int kLexThreads = 1024;

// W: row stride of P (LDS: ni+2; HBM: pitch); P points at cell (0,0)
template <bool XORDER>
__device__ __forceinline__ double lex_cell(double* P, const double* rhs_glob, long long rpitch,
                                           long long W, int i, int j, double idx2, double idy2,
                                           double factor) {
    const long long k = (long long)j * W + i;
    const double c = P[k];
    double xt, yt;
    if (XORDER) {  // assignment-5/sequential/src/solver.c:162-164
        xt = (P[k + 1] - 2.0 * c) + P[k - 1];
        yt = (P[k + W] - 2.0 * c) + P[k - W];
    } else {  // assignment-4/src/solver.c:149-151
        xt = (P[k - 1] - 2.0 * c) + P[k + 1];
        yt = (P[k - W] - 2.0 * c) + P[k + W];
    }
    const double r = rhs_glob[(long long)j * rpitch + i] - (xt * idx2 + yt * idy2);
    P[k] = c - (factor * r);
    return r;
}

template <bool XORDER>
__global__ __launch_bounds__(kLexThreads) void lex_solve_kernel(
    double* __restrict__ p_glob, const double* __restrict__ rhs_glob, int ni, int nj,
    long long pitch, double idx2, double idy2, double factor, double cells, int use_lds,
    DevState* st) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* red = lds;  // 16 wave partials + broadcast slot
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int nt = blockDim.x;
    double* const pg = p_glob + (long long)kYOff * pitch + kXOff;  // cell (0,0) in HBM
    const double* rg = rhs_glob + (long long)kYOff * pitch + kXOff;
    long long rpitch = pitch;
    double* P = pg;
    long long W = pitch;
    const long long Wl = ni + 2;
    if (use_lds) {
        P = lds + 32;
        W = Wl;
        const long long ncell = Wl * (nj + 2);
        for (long long k = t; k < ncell; k += nt) {
            const int i = (int)(k % Wl), j = (int)(k / Wl);
            P[k] = pg[(long long)j * pitch + i];
        }
        if (use_lds == 2) {
            // rhs too (its interior cells, row-major after p): every diagonal's
            // rhs loads are then LDS reads, not a global-memory round trip on
            // the diagonal's dependency chain (the reference's 100 x 100 grids)
            double* R = P + ncell;
            for (long long k = t; k < (long long)ni * nj; k += nt) {
                const int i = 1 + (int)(k % ni), j = 1 + (int)(k / ni);
                R[k] = rg[(long long)j * pitch + i];
            }
            rg = R - ni - 1;  // rg[j * ni + i] = R[(j - 1) ni + i - 1]
            rpitch = ni;
        }
        __syncthreads();
    }

    const double epssq = st->epssq;
    const int itermax = st->itermax;
    double res = 1.0;
    int it = 0;
    while ((res >= epssq) && (it < itermax)) {
        double acc = 0.0;
        for (int d = 2; d <= ni + nj; ++d) {
            const int ilo = max(1, d - nj), ihi = min(ni, d - 1);
            for (int i = ilo + t; i <= ihi; i += nt) {
                const double r = lex_cell<XORDER>(P, rg, rpitch, W, i, d - i, idx2, idy2, factor);
                acc += r * r;
            }
            __syncthreads();
        }
        // Neumann ghost copy: rows, then columns (corners untouched)
        for (int i = 1 + t; i <= ni; i += nt) {
            P[i] = P[W + i];
            P[(long long)(nj + 1) * W + i] = P[(long long)nj * W + i];
        }
        __syncthreads();
        for (int j = 1 + t; j <= nj; j += nt) {
            P[(long long)j * W] = P[(long long)j * W + 1];
            P[(long long)j * W + ni + 1] = P[(long long)j * W + ni];
        }
        // fixed-order block sum of r^2
        acc = wave_sum(acc);
        if (lane == 0) red[wave] = acc;
        __syncthreads();
        if (t == 0) {
            double s = 0.0;
            for (int w = 0; w < nt / 64; ++w) s += red[w];
            red[16] = s;
        }
        __syncthreads();
        res = red[16] / cells;
        ++it;
    }

    if (use_lds) {
        const long long ncell = Wl * (nj + 2);
        for (long long k = t; k < ncell; k += nt) {
            const int i = (int)(k % Wl), j = (int)(k / Wl);
            pg[(long long)j * pitch + i] = P[k];
        }
    }
    if (t == 0) {
        st->it = it;
        st->res = res;
        st->done = 1;
    }
}

void launch_solve_lex(hipStream_t s, double* p, const double* rhs, int ni, int nj,
                      long long pitch, double idx2, double idy2, double factor, double cells,
                      int xorder, DevState* st) {
    const size_t need = sizeof(double) * (32 + (size_t)(ni + 2) * (nj + 2));
    const size_t need_r = need + sizeof(double) * (size_t)ni * nj;  // + rhs
    // 2: p and rhs in LDS, 1: p in LDS, 0: both in HBM
    const int use_lds = need_r <= 160 * 1024 ? 2 : need <= 160 * 1024 ? 1 : 0;

    const int diag = ni < nj ? ni : nj;
    const int nt = std::min(kLexThreads, std::max(64, (diag + 63) / 64 * 64));
    const size_t lds = use_lds == 2 ? need_r : use_lds ? need : sizeof(double) * 32;
    if (xorder) {
        (void)hipFuncSetAttribute((const void*)lex_solve_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(lex_solve_kernel<true>, dim3(1), dim3(nt), lds, s, p, rhs, ni,
                           nj, pitch, idx2, idy2, factor, cells, use_lds, st);
    } else {
        (void)hipFuncSetAttribute((const void*)lex_solve_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(lex_solve_kernel<false>, dim3(1), dim3(nt), lds, s, p, rhs,
                           ni, nj, pitch, idx2, idy2, factor, cells, use_lds, st);
    }
}

}  // namespace misor
