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
    const double* const rg = rhs_glob + (long long)kYOff * pitch + kXOff;
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
                const double r = lex_cell<XORDER>(P, rg, pitch, W, i, d - i, idx2, idy2, factor);
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

// The same solve as ONE wave with no barriers (round 5), for grids whose p
// fits the LDS and has at most 64 * kLexWaveG rows (the reference's 100 x 100
// .par grids): lane L owns rows L + 1, L + 65, ... and row j trails row j - 1
// by one step -- cell (i, j) is updated at step (i - 1) + (j - 1) -- so at
// every step its NEW left neighbour is the lane's own result of the step
// before (a register), its NEW lower neighbour the result of lane L - 1 (lane
// 63 of the row group below, for lane 0) of the step before (a DPP lane
// rotation), and its right and upper neighbours are still OLD: exactly the
// lexicographic order, with no barrier and no LDS round trip on the step's
// dependency chain.  The old operands and rhs are loaded one step ahead; the
// new values go to LDS for the next sweep.  Per-cell expression: lex_cell's.
constexpr int kLexWaveG = 4;

template <bool XORDER, int GM>
__global__ __launch_bounds__(64) void lex_wave_kernel(double* __restrict__ p_glob,
                                                      const double* __restrict__ rhs_glob, int ni,
                                                      int nj, long long pitch, double idx2,
                                                      double idy2, double factor, double cells,
                                                      DevState* st) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x;
    double* const pg = p_glob + (long long)kYOff * pitch + kXOff;  // cell (0,0) in HBM
    const double* const rg = rhs_glob + (long long)kYOff * pitch + kXOff;
    const long long W = ni + 2;
    double* const P = lds;
    const long long ncell = W * (nj + 2);
    for (long long k = lane; k < ncell; k += 64) {
        const int i = (int)(k % W), j = (int)(k / W);
        P[k] = pg[(long long)j * pitch + i];
    }
    const double epssq = st->epssq;
    const int itermax = st->itermax;
    const int nsteps = ni + nj - 1;
    double res = 1.0;
    int it = 0;
    // the operands of a row's cell at one step: rhs and the OLD values of the
    // cell, its right and upper neighbours, and the ghosts a first column /
    // first row reads (left P(0, j), lower P(i, 0)); loaded one step ahead --
    // nothing this sweep writes before that step changes them
    struct Ops {
        double rh, c, r, u, gl, gd;
    };
    auto load_ops = [&](int i, int j) {
        Ops o{0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        if (j <= nj && i >= 1 && i <= ni) {
            const long long k = (long long)j * W + i;
            o.rh = rg[(long long)j * pitch + i];
            o.c = P[k];
            o.r = P[k + 1];
            o.u = P[k + W];
            o.gl = P[k - 1];  // (a ghost only where i == 1)
            o.gd = P[k - W];  // (a ghost only where j == 1)
        }
        return o;
    };
    while ((res >= epssq) && (it < itermax)) {
        double acc = 0.0;
        Ops nx[GM];
        double prev[GM];  // each row's result of the previous step: its NEW P(i-1, j)
#pragma unroll
        for (int g = 0; g < GM; ++g) {
            const int j = lane + 1 + 64 * g;
            nx[g] = load_ops(2 - j, j);
            prev[g] = 0.0;
        }
        for (int s = 0; s < nsteps; ++s) {
            Ops cur[GM];
#pragma unroll
            for (int g = 0; g < GM; ++g) {
                cur[g] = nx[g];
                const int j = lane + 1 + 64 * g;
                nx[g] = load_ops(s + 3 - j, j);  // next step's cell (i + 1, j)
            }
            // NEW P(i, j - 1): lane L - 1's result of the previous step (lane 63's
            // of the row group below for lane 0) -- a DPP lane rotation
            double rot[GM];
#pragma unroll
            for (int g = 0; g < GM; ++g)
                rot[g] = __hiloint2double(
                    __builtin_amdgcn_mov_dpp(__double2hiint(prev[g]), 0x13C, 0xf, 0xf, false),
                    __builtin_amdgcn_mov_dpp(__double2loint(prev[g]), 0x13C, 0xf, 0xf, false));
#pragma unroll
            for (int g = 0; g < GM; ++g) {
                const int j = lane + 1 + 64 * g, i = s + 2 - j;
                if (j <= nj && i >= 1 && i <= ni) {
                    const Ops& o = cur[g];
                    const double lft = i == 1 ? o.gl : prev[g];
                    const double dwn = j == 1 ? o.gd : (lane == 0 ? rot[g > 0 ? g - 1 : 0] : rot[g]);
                    const double c = o.c;
                    double xt, yt;
                    if (XORDER) {  // assignment-5/sequential/src/solver.c:162-164
                        xt = (o.r - 2.0 * c) + lft;
                        yt = (o.u - 2.0 * c) + dwn;
                    } else {  // assignment-4/src/solver.c:149-151
                        xt = (lft - 2.0 * c) + o.r;
                        yt = (dwn - 2.0 * c) + o.u;
                    }
                    const double r = o.rh - (xt * idx2 + yt * idy2);
                    const double v = c - (factor * r);
                    P[(long long)j * W + i] = v;
                    prev[g] = v;
                    acc += r * r;
                }
            }
        }
        asm volatile("" ::: "memory");
        // Neumann ghost copy: rows, then columns (corners untouched)
        for (int i = 1 + lane; i <= ni; i += 64) {
            P[i] = P[W + i];
            P[(long long)(nj + 1) * W + i] = P[(long long)nj * W + i];
        }
        asm volatile("" ::: "memory");
        for (int j = 1 + lane; j <= nj; j += 64) {
            P[(long long)j * W] = P[(long long)j * W + 1];
            P[(long long)j * W + ni + 1] = P[(long long)j * W + ni];
        }
        asm volatile("" ::: "memory");
        res = wave_sum(acc) / cells;
        ++it;
    }
    for (long long k = lane; k < ncell; k += 64) {
        const int i = (int)(k % W), j = (int)(k / W);
        pg[(long long)j * pitch + i] = P[k];
    }
    if (lane == 0) {
        st->it = it;
        st->res = res;
        st->done = 1;
    }
}

void launch_solve_lex(hipStream_t s, double* p, const double* rhs, int ni, int nj,
                      long long pitch, double idx2, double idy2, double factor, double cells,
                      int xorder, DevState* st) {
    const size_t need = sizeof(double) * (32 + (size_t)(ni + 2) * (nj + 2));
    const int use_lds = need <= 160 * 1024;
    static const bool wave = [] {  // MISOR_LEX_WAVE=0: the workgroup form (A/B)
        const char* e = getenv("MISOR_LEX_WAVE");
        return !(e && e[0] == '0');
    }();
    if (wave && use_lds && nj <= 64 * kLexWaveG) {
        const size_t lb = sizeof(double) * (size_t)(ni + 2) * (nj + 2);
        auto go = [&](auto kernel) {
            (void)hipFuncSetAttribute((const void*)kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb);
            hipLaunchKernelGGL(kernel, dim3(1), dim3(64), lb, s, p, rhs, ni, nj, pitch, idx2,
                               idy2, factor, cells, st);
        };
        const int G = (nj + 63) / 64;
        if (xorder) {
            if (G <= 1) go(lex_wave_kernel<true, 1>);
            else if (G <= 2) go(lex_wave_kernel<true, 2>);
            else go(lex_wave_kernel<true, kLexWaveG>);
        } else {
            if (G <= 1) go(lex_wave_kernel<false, 1>);
            else if (G <= 2) go(lex_wave_kernel<false, 2>);
            else go(lex_wave_kernel<false, kLexWaveG>);
        }
        return;
    }
    const int diag = ni < nj ? ni : nj;
    const int nt = std::min(kLexThreads, std::max(64, (diag + 63) / 64 * 64));
    const size_t lds = use_lds ? need : sizeof(double) * 32;
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
