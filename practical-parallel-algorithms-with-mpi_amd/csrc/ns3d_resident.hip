// ns3d_resident.hip -- the whole 3D red-black solve (assignment-6/src/
// solver.c:175-297) in ONE launch for grids whose pressure field fits in the
// GPU's combined LDS (256 CUs x 160 KB = 40 MB: p of the reference's 128^3 is
// 17 MB).
//
// Why: at 128^3 an iteration of the streaming sweep (k3_sweep, one launch per
// iteration) is a single resident round whose length is its k-march's latency
// chain, ~26 us for 2M cells.  Here every workgroup keeps one
// box of p (32 x 16 x 16 cells + a one-cell shell) in LDS and its rhs in
// registers for the whole solve, and the iterations are separated by grid
// barriers instead of kernel boundaries:
//
//   red pass (LDS)  -> its box-surface cells to p in HBM -> grid barrier ->
//   red shell cells from the neighbours' surfaces -> black pass -> black
//   surface cells + the workgroup's residual partial -> grid barrier ->
//   black shell cells; every workgroup sums all partials in the same fixed
//   order and applies the loop test (res = (res + sum)/N, solver.c:283-289),
//   so all stop after the same iteration.
//
// Semantics are solve()'s, cell by cell: red cells (i+j+k odd) only read
// black ones and vice versa, so the shell needs only the colour the next pass
// reads; the Neumann ghost-face copy of the iteration's end (solver.c:237-278,
// faces only, edges and corners never touched) is done by the owner of the
// face cell right after updating it -- the ghost is read by that cell alone.
// Launched cooperatively (hipLaunchCooperativeKernel refuses a grid that cannot
// be co-resident, and the host then falls back to k3_sweep); every barrier wait
// is bounded: on a timeout the kernel raises an abort flag that every
// workgroup checks, all of them exit, and the host reports the failure.
//
// Memory ordering across XCDs (their L2s are not coherent with each other).
// Default (mode 48): the box-surface cells and the partials -- the only global
// data the loop exchanges -- are written and read with relaxed agent-scope
// atomics (coherent across the L2s), each wave waits for its stores to be
// acknowledged before the workgroup arrives, and the barrier counts arrivals
// in two levels (per blockIdx % 8 group, then one global counter).  Measured
// at 128^3 (profiles/r03_res3d_modes.txt): agent-scope release/acquire fences
// in every wave (mode 0, L2 write-back + invalidate at each barrier) 69 us per
// iteration, in thread 0 only (mode 1) 41 us, atomics instead of fences (16)
// 24.4 us, + the two-level barrier (48) 20.9 us; of those, the two passes and
// the loop test take 9 us, the two barriers 4.6 us, the two exchanges 7.3 us.
// An uncached mailbox read with plain loads (mode 8) gave wrong results: the
// lines were still cached.

#include <cstdlib>
#include <type_traits>

#include "misor_internal.h"

namespace misor {

namespace {

constexpr int kRbx = 32, kRby = 16, kRbz = 16;  // box of cells per workgroup
constexpr int kRsx = kRbx + 2;                   // LDS strides (one-cell shell)
constexpr int kRsy = (kRby + 2) * kRsx;
constexpr int kRcells = (kRbz + 2) * kRsy;
constexpr int kRfaces = 2 * (kRby * kRbz + kRbx * kRbz + kRbx * kRby);  // shell face cells
constexpr int kRthreads = 256;
constexpr int kRg = 4;  // planes per group of a colour pass (its LDS reads issued together)
constexpr int kRq = kRfaces / kRthreads;  // shell cells per thread
static_assert(kRfaces % kRthreads == 0, "shell cells per thread");
static_assert(kRbx == 32 && kRby == 16 && kRthreads == 256,
              "thread t: column pair t & 15, row t >> 4, all planes of the box");
constexpr long long kSpinLimit = 1ll << 22;  // polls (~1 us each) before a barrier gives up

struct Bar3 {
    unsigned count;       // arrivals so far (zeroed before each launch)
    int abort;            // 1: a barrier timed out -- every workgroup leaves
    unsigned pad[14];
    unsigned xcd[8 * 16];  // mode bit 5: arrivals per group blockIdx % 8, one 64-B line each
};

__device__ __forceinline__ double rwave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// fixed-order sum over the workgroup (wave trees, then waves 0..NW-1 in
// order); every thread gets the result
template <int NW = 4>
__device__ __forceinline__ double rblock_sum(double v, double* sh) {
    v = rwave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = sh[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) s += sh[w];
    return s;
}

// grid barrier number n (1-based): returns false if the solve was aborted.
// mode (experiments, MISOR3_RESIDENT_MODE): bit 0 = the agent-scope fences by
// thread 0 only (after a workgroup-scope release by every wave)
//
// The default hand-off (mode bits 4 + 5, no agent-scope fence) is the
// "sc1 stores drained, sc1 loads" form of MI355X_MICROARCH.md (Workgroup
// dispatch ... Valid forms, table row 1), a gfx950 property measured there and
// not an architectural guarantee of the HIP memory model; the library is built
// for gfx950 only.  The conditions it rests on, all held here:
//  (1) every load of exchanged data (mailbox cells, partials) is a relaxed
//      agent-scope atomic load (global_load ... sc1), never a plain load
//      (mode 8 with plain loads read stale lines);
//  (2) every store of it is a relaxed agent-scope atomic store (sc1);
//  (3) every storing wave waits for its stores (s_waitcnt 0) before the
//      workgroup barrier, and only then does ONE lane (thread 0) add to the
//      arrival counter -- in the two-level form the group's last arriver,
//      told by the value its own add returned, adds to the global counter;
//  (4) the consumer polls the counter with sc1 loads (relaxed agent-scope
//      atomic loads) from one lane and the other waves load only after the
//      workgroup barrier that lane joins.
// Agent-scope release / acquire fences instead (mode 0 / 1) are correct by
// the memory model and cost an L2 write-back + invalidate per barrier: 41-69
// us per iteration against 16.4 (profiles/r03_res3d_modes.txt).
__device__ bool rgrid_sync(Bar3* bar, unsigned n, int* sh_flag, int mode) {
    if (mode & 24) {  // exchange data and partials by agent-scope atomics: no cache upkeep
        __builtin_amdgcn_s_waitcnt(0);  // this wave's stores acknowledged by memory
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
    } else if (mode & 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        unsigned target = n * gridDim.x;
        if (mode & 32) {  // two levels: the last of each group blockIdx % 8 arrives globally
            const unsigned x = blockIdx.x & 7, nb = gridDim.x;
            const unsigned cx = (nb - x + 7) / 8;
            const unsigned old = __hip_atomic_fetch_add(&bar->xcd[16 * x], 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == n * cx)
                __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            target = n * (nb < 8 ? nb : 8);
        } else {
            __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int ab = 0;
        long long polls = 0;
        while (__hip_atomic_load(&bar->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               target) {
            if (__hip_atomic_load(&bar->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                ab = 1;
                break;
            }
            if (++polls > kSpinLimit) {
                __hip_atomic_store(&bar->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ab = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *sh_flag = ab;
        if ((mode & 25) == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (mode & 24)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    else if (!(mode & 1))
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return *sh_flag == 0;
}

// rgrid_sync's arrival half (the exchange-by-atomics modes, bits 3 / 4: the
// workgroup may compute in between anything that reads no exchanged data and
// writes none) with the workgroup's residual partial folded in: every wave has
// put its wave sum in sh[]; after the arrival barrier thread 0 adds them in
// wave order (rblock_sum's order), stores the partial (relaxed agent-scope,
// acknowledged before the arrival counts) and arrives -- one workgroup
// barrier instead of rblock_sum's two plus the arrival's
template <int NW>
__device__ void rgrid_arrive_sum(Bar3* bar, unsigned n, int mode, const double* sh,
                                 double* part, bool count) {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = sh[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) s += sh[w];
        __hip_atomic_store(part, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0);
        if (!count) return;
        if (mode & 32) {
            const unsigned x = blockIdx.x & 7, nb = gridDim.x;
            const unsigned cx = (nb - x + 7) / 8;
            const unsigned old = __hip_atomic_fetch_add(&bar->xcd[16 * x], 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == n * cx)
                __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ bool rgrid_wait(Bar3* bar, unsigned n, int* sh_flag, int mode) {
    if (threadIdx.x == 0) {
        const unsigned nb = gridDim.x;
        const unsigned target = (mode & 32) ? n * (nb < 8 ? nb : 8) : n * nb;
        int ab = 0;
        long long polls = 0;
        while (__hip_atomic_load(&bar->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               target) {
            if (__hip_atomic_load(&bar->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                ab = 1;
                break;
            }
            if (++polls > kSpinLimit) {
                __hip_atomic_store(&bar->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ab = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *sh_flag = ab;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return *sh_flag == 0;
}

}  // namespace

__global__ __launch_bounds__(kRthreads, 1) void k3_resident(G3 g, double* __restrict__ p,
                                                            const double* __restrict__ rhs,
                                                            double idx2, double idy2, double idz2,
                                                            double factor, double cells,
                                                            double* __restrict__ partials,
                                                            DevState* __restrict__ st,
                                                            Bar3* __restrict__ bar, int nbx,
                                                            int nby, int mode,
                                                            double* __restrict__ mbox) {
    __shared__ double L[kRcells];
    __shared__ double sh[4];
    __shared__ int sh_flag;
    const int t = threadIdx.x;
    const int b = blockIdx.x;
    const int ox = 1 + (b % nbx) * kRbx;  // global coordinates of the box's first cell
    const int oy = 1 + (b / nbx % nby) * kRby;
    const int oz = 1 + b / (nbx * nby) * kRbz;
    const int I = g.I, J = g.J, K = g.K;
    const int sx = (int)g.sx, sxy = (int)g.sxy;  // resident grids are < 2^31 cells

    // p: the box and its shell (ghosts included; cells past a ragged edge: 0)
    for (int q = t; q < kRcells; q += kRthreads) {
        const int lz = q / kRsy, ly = q / kRsx % (kRby + 2), lx = q % kRsx;
        const int i = ox - 1 + lx, j = oy - 1 + ly, k = oz - 1 + lz;
        L[q] = (i <= I + 1 && j <= J + 1 && k <= K + 1) ? p[k * sxy + j * sx + i] : 0.0;
    }
    // this thread's cells: the column pair (i0, i0+1) of row j, planes oz .. oz+15
    const int px = t & 15, y = t >> 4;
    const int i0 = ox + 2 * px, j = oy + y;
    double rh[kRbz][2];
#pragma unroll
    for (int z = 0; z < kRbz; ++z) {
        const int k = oz + z;
#pragma unroll
        for (int e = 0; e < 2; ++e)
            rh[z][e] = (i0 + e <= I && j <= J && k <= K) ? rhs[k * sxy + j * sx + i0 + e] : 0.0;
    }
    // shell cells this thread refreshes: LDS position, global offset, colour
    // (bit 0: (i+j+k) & 1) and whether it is a neighbour's interior cell
    int sl[kRq], sg[kRq], sc[kRq];
#pragma unroll
    for (int m = 0; m < kRq; ++m) {
        const int f = t + kRthreads * m;
        int lx, ly, lz;
        if (f < 2 * kRby * kRbz) {  // x faces
            const int r = f % (kRby * kRbz);
            lx = f < kRby * kRbz ? 0 : kRbx + 1;
            ly = 1 + r % kRby;
            lz = 1 + r / kRby;
        } else if (f < 2 * kRby * kRbz + 2 * kRbx * kRbz) {  // y faces
            const int h = f - 2 * kRby * kRbz, r = h % (kRbx * kRbz);
            ly = h < kRbx * kRbz ? 0 : kRby + 1;
            lx = 1 + r % kRbx;
            lz = 1 + r / kRbx;
        } else {  // z faces
            const int h = f - 2 * kRby * kRbz - 2 * kRbx * kRbz, r = h % (kRbx * kRby);
            lz = h < kRbx * kRby ? 0 : kRbz + 1;
            lx = 1 + r % kRbx;
            ly = 1 + r / kRbx;
        }
        const int i = ox - 1 + lx, jj = oy - 1 + ly, k = oz - 1 + lz;
        const bool inner = i >= 1 && i <= I && jj >= 1 && jj <= J && k >= 1 && k <= K;
        sl[m] = (lz * (kRby + 2) + ly) * kRsx + lx;
        sg[m] = inner ? k * sxy + jj * sx + i : -1;
        sc[m] = (i + jj + k) & 1;
    }
    // where box-surface cells are exchanged: p itself, or (mode bit 3) a
    // mailbox of p's layout in uncached memory
    double* const xch = (mode & 8) ? mbox : p;
    // mode bit 3 or 4: exchanged cells and partials moved by relaxed agent-scope
    // atomics (coherent across the XCDs' L2s without write-backs / invalidations)
    const bool xa = (mode & 24) != 0;
    auto xload = [&](const double* a) {
        return xa ? __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *a;
    };
    auto xstore = [&](double* a, double v) {
        if (xa)
            __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            *a = v;
    };
    // the shell cells of colour `col` (0: black, i+j+k even; 1: red)
    auto refresh = [&](int col) {
        double v[kRq];
#pragma unroll
        for (int m = 0; m < kRq; ++m)
            v[m] = (sg[m] >= 0 && sc[m] == col) ? xload(xch + sg[m]) : 0.0;
#pragma unroll
        for (int m = 0; m < kRq; ++m)
            if (sg[m] >= 0 && sc[m] == col) L[sl[m]] = v[m];
    };
    // one colour pass: update, residual, ghost faces, box-surface cells to p
    double acc = 0.0;
    auto pass = [&](int col) {
        // groups of kRg planes: every LDS read of a group is issued before its
        // stores (a store may alias a later read as far as the compiler knows,
        // so one cell at a time would serialise on LDS latency)
        const int e0 = ((i0 + j + oz) & 1) == col ? 0 : 1;  // pair element of colour col, z = 0
#pragma unroll
        for (int z0 = 0; z0 < kRbz; z0 += kRg) {
            double c[kRg], xm[kRg], xp[kRg], ym[kRg], yp[kRg], zm[kRg], zp[kRg];
#pragma unroll
            for (int u = 0; u < kRg; ++u) {
                const int z = z0 + u, e = e0 ^ (z & 1);
                const int o = ((z + 1) * (kRby + 2) + (y + 1)) * kRsx + 2 * px + e + 1;
                c[u] = L[o];
                xm[u] = L[o - 1];
                xp[u] = L[o + 1];
                ym[u] = L[o - kRsx];
                yp[u] = L[o + kRsx];
                zm[u] = L[o - kRsy];
                zp[u] = L[o + kRsy];
            }
#pragma unroll
            for (int u = 0; u < kRg; ++u) {
                const int z = z0 + u, k = oz + z, e = e0 ^ (z & 1), i = i0 + e;
                if (i > I || j > J || k > K) continue;
                const int x = 2 * px + e;
                const int o = ((z + 1) * (kRby + 2) + (y + 1)) * kRsx + x + 1;
                const double cc = c[u];
                const double tx = (xp[u] - 2.0 * cc) + xm[u];
                const double ty = (yp[u] - 2.0 * cc) + ym[u];
                const double tz = (zp[u] - 2.0 * cc) + zm[u];
                const double r = (e ? rh[z][1] : rh[z][0]) - ((tx * idx2 + ty * idy2) + tz * idz2);
                const double v = cc - (factor * r);
                L[o] = v;
                acc += (r * r);
                // Neumann ghost faces (read by this cell only)
                if (i == 1) L[o - 1] = v;
                if (i == I) L[o + 1] = v;
                if (j == 1) L[o - kRsx] = v;
                if (j == J) L[o + kRsx] = v;
                if (k == 1) L[o - kRsy] = v;
                if (k == K) L[o + kRsy] = v;
                // box-surface cells: the neighbours' shells
                if (!(mode & 2) &&
                    (x == 0 || x == kRbx - 1 || y == 0 || y == kRby - 1 || z == 0 || z == kRbz - 1))
                    xstore(xch + (k * sxy + j * sx + i), v);
            }
        }
    };

    double res = st->res;
    int it = st->it, done = st->done;
    const double epssq = st->epssq;
    const int itermax = st->itermax;
    unsigned nbar = 0;
    bool ok = true;
    __syncthreads();
    // mode bit 1 / 2 (timing experiments only, results wrong): no shell
    // exchange / no grid barriers
    while (!done) {
        pass(1);  // red: i+j+k odd (solver.c: the sweep starts at (1,1,1))
        if (!(mode & 4) && !(ok = rgrid_sync(bar, ++nbar, &sh_flag, mode))) break;
        if (!(mode & 2)) refresh(1);
        __syncthreads();
        pass(0);
        const double s = rblock_sum(acc, sh);
        acc = 0.0;
        double* part = partials + (it & 1) * gridDim.x;
        if (t == 0) xstore(part + b, s);
        if (!(mode & 4) && !(ok = rgrid_sync(bar, ++nbar, &sh_flag, mode))) break;
        // every workgroup: the same fixed-order sum of all partials (loads
        // issued together with the shell's)
        double q = 0.0;
        for (int w = t; w < (int)gridDim.x; w += kRthreads) q += xload(part + w);
        if (!(mode & 2)) refresh(0);
        const double S = rblock_sum(q, sh);
        res = (res + S) / cells;
        ++it;
        done = !((res >= epssq) && (it < itermax));
        __syncthreads();
    }
    if (!ok) return;
    // the box and the ghost faces next to it, back to p
#pragma unroll
    for (int z = 0; z < kRbz; ++z) {
        const int k = oz + z;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int i = i0 + e;
            if (i > I || j > J || k > K) continue;
            const int o = ((z + 1) * (kRby + 2) + (y + 1)) * kRsx + 2 * px + e + 1;
            const int go = k * sxy + j * sx + i;
            p[go] = L[o];
            if (i == 1) p[go - 1] = L[o - 1];
            if (i == I) p[go + 1] = L[o + 1];
            if (j == 1) p[go - sx] = L[o - kRsx];
            if (j == J) p[go + sx] = L[o + kRsx];
            if (k == 1) p[go - sxy] = L[o - kRsy];
            if (k == K) p[go + sxy] = L[o + kRsy];
        }
    }
    if (b == 0 && t == 0) {
        st->it = it;
        st->res = res;
        st->done = done;
    }
}

// ---------------------------------------------------------------------------
// k3_resident1: ONE exchange and ONE grid barrier per iteration (mode bit 6).
// The LDS holds the box and a two-cell shell (36 x 20 x 20 doubles, 115 KB).
// Each iteration the workgroup also updates the red cells of the shell's
// inner layer (its face-neighbours' cells) with the same arithmetic as their
// owners, so the black pass finds every red neighbour locally; only black
// cells cross box boundaries: after the black pass a box writes its black
// cells within two of its surface to the mailbox of the iteration's parity,
// and after the barrier it reads the black cells of its shell (both face
// layers and the inner layer's edges).  Mailboxes alternate by iteration
// (a box may write iteration n+1's cells while a slower neighbour still reads
// iteration n's); p is only read at the start and written at the end.
constexpr int kTsx = kRbx + 4, kTsy = (kRby + 4) * kTsx, kTcells = (kRbz + 4) * kTsy;
constexpr int kTring = 2 * (kRby * kRbz + kRbx * kRbz + kRbx * kRby);  // inner-layer face cells
constexpr int kTshell = 2 * kTring + 4 * (kRbx + kRby + kRbz);  // received positions
constexpr int kTrx = kTshell / 2 + 128;  // black cells of the shell, at most

// shell position f (0 .. kTshell): face layers 0/1 and B+2/B+3, then the
// inner layer's 12 edges; LDS coordinates (shell offset 2)
__device__ __forceinline__ void shell_pos(int f, int& lx, int& ly, int& lz) {
    constexpr int FX = kRby * kRbz, FY = kRbx * kRbz, FZ = kRbx * kRby;
    if (f < 4 * FX) {
        const int l = f / FX, r = f % FX;
        lx = l < 2 ? l : kRbx + l;  // 0, 1, B+2, B+3
        ly = 2 + r % kRby;
        lz = 2 + r / kRby;
    } else if (f < 4 * (FX + FY)) {
        const int h = f - 4 * FX, l = h / FY, r = h % FY;
        ly = l < 2 ? l : kRby + l;
        lx = 2 + r % kRbx;
        lz = 2 + r / kRbx;
    } else if (f < 4 * (FX + FY + FZ)) {
        const int h = f - 4 * (FX + FY), l = h / FZ, r = h % FZ;
        lz = l < 2 ? l : kRbz + l;
        lx = 2 + r % kRbx;
        ly = 2 + r / kRbx;
    } else {  // edges of the inner layer: two coordinates in {1, B+2}
        const int h = f - 4 * (FX + FY + FZ);
        if (h < 4 * kRbx) {
            const int c = h / kRbx;
            lx = 2 + h % kRbx;
            ly = (c & 1) ? kRby + 2 : 1;
            lz = (c & 2) ? kRbz + 2 : 1;
        } else if (h < 4 * (kRbx + kRby)) {
            const int q = h - 4 * kRbx, c = q / kRby;
            ly = 2 + q % kRby;
            lx = (c & 1) ? kRbx + 2 : 1;
            lz = (c & 2) ? kRbz + 2 : 1;
        } else {
            const int q = h - 4 * (kRbx + kRby), c = q / kRbz;
            lz = 2 + q % kRbz;
            lx = (c & 1) ? kRbx + 2 : 1;
            ly = (c & 2) ? kRby + 2 : 1;
        }
    }
}

// inner-layer face position f (0 .. kTring)
__device__ __forceinline__ void ring_pos(int f, int& lx, int& ly, int& lz) {
    constexpr int FX = kRby * kRbz, FY = kRbx * kRbz, FZ = kRbx * kRby;
    if (f < 2 * FX) {
        const int r = f % FX;
        lx = f < FX ? 1 : kRbx + 2;
        ly = 2 + r % kRby;
        lz = 2 + r / kRby;
    } else if (f < 2 * (FX + FY)) {
        const int h = f - 2 * FX, r = h % FY;
        ly = h < FY ? 1 : kRby + 2;
        lx = 2 + r % kRbx;
        lz = 2 + r / kRbx;
    } else {
        const int h = f - 2 * (FX + FY), r = h % FZ;
        lz = h < FZ ? 1 : kRbz + 2;
        lx = 2 + r % kRbx;
        ly = 2 + r / kRbx;
    }
    (void)FZ;
}

// NT threads per box: thread t owns the column pair t & 15 of row (t >> 4) & 15
// in the PZ = 16 * 256 / NT planes from (t >> 8) * PZ (NT = 1024: four waves
// per SIMD to cover the LDS and FP64 latency of the passes)
// REG: every box lies wholly inside the domain (I, J, K multiples of the box:
// the reference's 128^3) -- the register form of the passes (below)
template <int NT, bool REG = false>
__global__ __launch_bounds__(NT, 1) void k3_resident1(G3 g, double* __restrict__ p,
                                                      const double* __restrict__ rhs, double idx2,
                                                      double idy2, double idz2, double factor,
                                                      double cells, double* __restrict__ partials,
                                                      DevState* __restrict__ st,
                                                      Bar3* __restrict__ bar, int nbx, int nby,
                                                      int mode, double* __restrict__ mbox,
                                                      int mstride) {
    constexpr int NW = NT / 64, PZ = kRbz * 256 / NT, G = NT >= 1024 ? 2 : (PZ < kRg ? PZ : kRg);
    static_assert(NT % 256 == 0 && PZ % 2 == 0 && PZ % G == 0 && G % 2 == 0, "thread layout");
    __shared__ double L[kTcells];
    __shared__ double sh[NW];
    __shared__ double sh_W[4];
    __shared__ int sh_flag;
    // built once: the shell's black cells to receive (LDS index | ghost-face bits
    // << 16, global offset) and the inner layer's red cells (LDS index | ghost
    // bits << 16, rhs) -- the loops below then touch only real cells
    __shared__ int2 rx_list[kTrx];
    __shared__ int ring_o[kTring / 2 + 64];
    __shared__ double ring_r[kTring / 2 + 64];
    __shared__ int n_rx, n_ring;
    const int t = threadIdx.x;
    const int b = blockIdx.x;
    const int ox = 1 + (b % nbx) * kRbx;
    const int oy = 1 + (b / nbx % nby) * kRby;
    const int oz = 1 + b / (nbx * nby) * kRbz;
    const int I = g.I, J = g.J, K = g.K;
    const int sx = (int)g.sx, sxy = (int)g.sxy;
    auto gof = [&](int i, int jj, int k) { return k * sxy + jj * sx + i; };
    auto inner = [&](int i, int jj, int k) {
        return i >= 1 && i <= I && jj >= 1 && jj <= J && k >= 1 && k <= K;
    };
    auto xload = [&](const double* a) {
        return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto xstore = [&](double* a, double v) {
        __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    // p: the box and its two-cell shell (ghosts included; outside the array: 0)
    for (int q = t; q < kTcells; q += NT) {
        const int lz = q / kTsy, ly = q / kTsx % (kRby + 4), lx = q % kTsx;
        const int i = ox - 2 + lx, jj = oy - 2 + ly, k = oz - 2 + lz;
        L[q] = (i >= 0 && jj >= 0 && k >= 0 && i <= I + 1 && jj <= J + 1 && k <= K + 1)
                   ? p[gof(i, jj, k)]
                   : 0.0;
    }
    const int px = t & 15, y = (t >> 4) & 15, zb = (t >> 8) * PZ;
    const int i0 = ox + 2 * px, j = oy + y;
    double rh[PZ][2];  // rh[z - zb]
#pragma unroll
    for (int z = 0; z < PZ; ++z) {
        const int k = oz + zb + z;
#pragma unroll
        for (int e = 0; e < 2; ++e)
            rh[z][e] = (i0 + e <= I && j <= J && k <= K) ? rhs[gof(i0 + e, j, k)] : 0.0;
    }
    auto gbits = [&](int i, int jj, int k) {
        return (i == 1 ? 1 : 0) | (i == I ? 2 : 0) | (jj == 1 ? 4 : 0) | (jj == J ? 8 : 0) |
               (k == 1 ? 16 : 0) | (k == K ? 32 : 0);
    };
    if (t == 0) n_rx = n_ring = 0;
    __syncthreads();
    for (int f = t; f < kTring; f += NT) {
        int lx, ly, lz;
        ring_pos(f, lx, ly, lz);
        const int i = ox - 2 + lx, jj = oy - 2 + ly, k = oz - 2 + lz;
        if (inner(i, jj, k) && ((i + jj + k) & 1)) {
            const int q = atomicAdd(&n_ring, 1);
            ring_o[q] = ((lz * (kRby + 4) + ly) * kTsx + lx) | (gbits(i, jj, k) << 16);
            ring_r[q] = rhs[gof(i, jj, k)];
        }
    }
    for (int f = t; f < kTshell; f += NT) {
        int lx, ly, lz;
        shell_pos(f, lx, ly, lz);
        const int i = ox - 2 + lx, jj = oy - 2 + ly, k = oz - 2 + lz;
        if (inner(i, jj, k) && !((i + jj + k) & 1)) {
            const int q = atomicAdd(&n_rx, 1);
            // ghost faces only for the inner layer's cells (the outer layer's are never read)
            const bool outer = lx == 0 || lx == kRbx + 3 || ly == 0 || ly == kRby + 3 || lz == 0 ||
                               lz == kRbz + 3;
            rx_list[q] = make_int2(((lz * (kRby + 4) + ly) * kTsx + lx) |
                                       ((outer ? 0 : gbits(i, jj, k)) << 16),
                                   gof(i, jj, k));
        }
    }
    __syncthreads();
    const int nring = n_ring, nrx = n_rx;
    auto ghosts = [&](int o, int gb, double v) {
        if (gb & 1) L[o - 1] = v;
        if (gb & 2) L[o + 1] = v;
        if (gb & 4) L[o - kTsx] = v;
        if (gb & 8) L[o + kTsx] = v;
        if (gb & 16) L[o - kTsy] = v;
        if (gb & 32) L[o + kTsy] = v;
    };
    // one update at LDS index o of cell (i, jj, k): returns r; ghost faces copied
    auto upd = [&](int o, int i, int jj, int k, double rv, double c, double xm, double xp,
                   double ym, double yp, double zm, double zp) {
        const double tx = (xp - 2.0 * c) + xm;
        const double ty = (yp - 2.0 * c) + ym;
        const double tz = (zp - 2.0 * c) + zm;
        const double r = rv - ((tx * idx2 + ty * idy2) + tz * idz2);
        const double v = c - (factor * r);
        L[o] = v;
        if (i == 1) L[o - 1] = v;
        if (i == I) L[o + 1] = v;
        if (jj == 1) L[o - kTsx] = v;
        if (jj == J) L[o + kTsx] = v;
        if (k == 1) L[o - kTsy] = v;
        if (k == K) L[o + kTsy] = v;
        return r;
    };
    double acc = 0.0;
    // (round 4 also tried computing the red cells deep inside the box during
    // the grid barrier's wait: ~1% with the separate residual sums, slower
    // once they were folded into the barrier -- profiles/r04_res3d_modes.txt)
    double own[PZ][2];
    // the box's cells of colour col (1: red, i+j+k odd); black cells within two
    // of the box surface go to the mailbox xm.  REG: the register form (full
    // boxes)
    auto pass = [&](int col, double* xm) {
        const int e0 = ((i0 + j + oz) & 1) == col ? 0 : 1;
#pragma unroll
        for (int z0 = 0; z0 < PZ; z0 += G) {
            double c[G], am[G], ap[G], bm[G], bp[G], cm[G], cp[G];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const int z = zb + z0 + u, e = e0 ^ (u & 1);  // zb, z0 even
                const int o = ((z + 2) * (kRby + 4) + (y + 2)) * kTsx + 2 * px + e + 2;
                if (REG) {
                    const int w = z0 + u;
                    // (the far x-neighbour from the next thread's register by a
                    // DPP row shift measured slower, 12.8-13.1 against 12.3-12.6
                    // us: profiles/r04_res3d_dpp.txt)
                    const double far = L[e ? o + 1 : o - 1];
                    const double mine = e ? own[w][1] : own[w][0];
                    const double part = e ? own[w][0] : own[w][1];
                    c[u] = mine;
                    am[u] = e ? part : far;
                    ap[u] = e ? far : part;
                    bm[u] = L[o - kTsx];
                    bp[u] = L[o + kTsx];
                    cm[u] = w > 0 ? (e ? own[w - 1][1] : own[w - 1][0]) : L[o - kTsy];
                    cp[u] = w < PZ - 1 ? (e ? own[w + 1][1] : own[w + 1][0]) : L[o + kTsy];
                } else {
                    c[u] = L[o];
                    am[u] = L[o - 1];
                    ap[u] = L[o + 1];
                    bm[u] = L[o - kTsx];
                    bp[u] = L[o + kTsx];
                    cm[u] = L[o - kTsy];
                    cp[u] = L[o + kTsy];
                }
            }
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const int z = zb + z0 + u, k = oz + z, e = e0 ^ (u & 1), i = i0 + e;
                if (i > I || j > J || k > K) continue;
                const int x = 2 * px + e;
                const int o = ((z + 2) * (kRby + 4) + (y + 2)) * kTsx + x + 2;
                const double r = upd(o, i, j, k, e ? rh[z0 + u][1] : rh[z0 + u][0], c[u], am[u], ap[u],
                                     bm[u], bp[u], cm[u], cp[u]);
                acc += (r * r);
                const double nv = c[u] - (factor * r);  // the value upd() stored
                if (REG) {
                    if (e) own[z0 + u][1] = nv;
                    else   own[z0 + u][0] = nv;
                }
                if (col == 0 && !(mode & 2) && (x < 2 || x >= kRbx - 2 || y < 2 || y >= kRby - 2 || z < 2 ||
                                 z >= kRbz - 2))
                    xstore(xm + gof(i, j, k), nv);
            }
        }
    };
    auto ring_red = [&]() {
        constexpr int RQ = (kTring / 2 + 64 + NT - 1) / NT;
        double c[RQ], am[RQ], ap[RQ], bm[RQ], bp[RQ], cm[RQ], cp[RQ];
        int oo[RQ];
#pragma unroll
        for (int m = 0; m < RQ; ++m) {
            const int q = t + NT * m;
            oo[m] = q < nring ? ring_o[q] : -1;
            const int o = oo[m] < 0 ? kTsy + kTsx + 1 : (oo[m] & 0xffff);
            c[m] = L[o];
            am[m] = L[o - 1];
            ap[m] = L[o + 1];
            bm[m] = L[o - kTsx];
            bp[m] = L[o + kTsx];
            cm[m] = L[o - kTsy];
            cp[m] = L[o + kTsy];
        }
#pragma unroll
        for (int m = 0; m < RQ; ++m) {
            if (oo[m] < 0) continue;
            const int o = oo[m] & 0xffff;
            const double tx = (ap[m] - 2.0 * c[m]) + am[m];
            const double ty = (bp[m] - 2.0 * c[m]) + bm[m];
            const double tz = (cp[m] - 2.0 * c[m]) + cm[m];
            const double r = ring_r[t + NT * m] - ((tx * idx2 + ty * idy2) + tz * idz2);
            const double v = c[m] - (factor * r);
            L[o] = v;
            ghosts(o, oo[m] >> 16, v);
        }
    };
    // the shell's black cells from mailbox xm, with their ghost faces
    auto receive = [&](const double* xm) {
        constexpr int RXQ = (kTrx + NT - 1) / NT;
        double v[RXQ];
        int2 e[RXQ];
#pragma unroll
        for (int m = 0; m < RXQ; ++m) {
            const int q = t + NT * m;
            e[m] = q < nrx ? rx_list[q] : make_int2(-1, 0);
            v[m] = e[m].x >= 0 ? xload(xm + e[m].y) : 0.0;
        }
#pragma unroll
        for (int m = 0; m < RXQ; ++m) {
            if (e[m].x < 0) continue;
            const int o = e[m].x & 0xffff;
            L[o] = v[m];
            ghosts(o, e[m].x >> 16, v[m]);
        }
    };

    double res = st->res;
    int it = st->it, done = st->done;
    const double epssq = st->epssq;
    const int itermax = st->itermax;
    unsigned nbar = 0;
    bool ok = true;
    __syncthreads();
    // mode bits 2 / 4 / 512 / 1024 (timing experiments only, results wrong):
    // no shell exchange / no grid barrier / no ring update / no partials read
    if (REG) {
#pragma unroll
        for (int u = 0; u < PZ; ++u) {
            const int o = ((zb + u + 2) * (kRby + 4) + (y + 2)) * kTsx + 2 * px + 2;
            own[u][0] = L[o];
            own[u][1] = L[o + 1];
        }
    }
    while (!done) {
        double* const xm = mbox + (it & 1) * (long long)mstride;
        if (!(mode & 512)) ring_red();  // the neighbours' red cells next to the box
        pass(1, xm);
        __syncthreads();
        pass(0, xm);
        // the workgroup's residual: wave sums to sh[], added and published
        // with the arrival (rgrid_arrive_sum)
        {
            const double ws = rwave_sum(acc);
            if ((t & 63) == 0) sh[t >> 6] = ws;
        }
        acc = 0.0;
        double* part = partials + (it & 1) * gridDim.x;
        ++nbar;
        rgrid_arrive_sum<NW>(bar, nbar, mode, sh, part + b, !(mode & 4));
        if (!(mode & 4) && !(ok = rgrid_wait(bar, nbar, &sh_flag, mode))) break;
        // the sum of all partials, by wave 0 in rblock_sum's order (the wave
        // tree of partials 64 w .. 64 w + 63, then w = 0, 1, ...): every
        // workgroup gets the same bits
        // (waves 0-3 one chunk of 64 partials each, lane 0's wave tree; the
        // chunks added in order after the barrier: the bits of wave 0 doing all
        // four in turn, without their four loads and trees in series on it)
        if (t < 256) {
            const double v = !(mode & 1024) && t < (int)gridDim.x ? xload(part + t) : 0.0;
            const double ws = rwave_sum(v);
            if ((t & 63) == 0) sh_W[t >> 6] = ws;
        }
        if (!(mode & 2)) receive(xm);
        __syncthreads();
        res = (res + (((sh_W[0] + sh_W[1]) + sh_W[2]) + sh_W[3])) / cells;
        ++it;
        done = !((res >= epssq) && (it < itermax));
    }
    if (!ok) return;
#pragma unroll
    for (int z = zb; z < zb + PZ; ++z) {
        const int k = oz + z;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int i = i0 + e;
            if (i > I || j > J || k > K) continue;
            const int o = ((z + 2) * (kRby + 4) + (y + 2)) * kTsx + 2 * px + e + 2;
            const int go = gof(i, j, k);
            p[go] = L[o];
            if (i == 1) p[go - 1] = L[o - 1];
            if (i == I) p[go + 1] = L[o + 1];
            if (j == 1) p[go - sx] = L[o - kTsx];
            if (j == J) p[go + sx] = L[o + kTsx];
            if (k == 1) p[go - sxy] = L[o - kTsy];
            if (k == K) p[go + sxy] = L[o + kTsy];
        }
    }
    if (b == 0 && t == 0) {
        st->it = it;
        st->res = res;
        st->done = done;
    }
}

// the resident solve's form (mode bits documented at rgrid_sync and the
// kernels) and its kernel and threads per box (bit 7: 1024, bit 8: 512, else
// 256; bit 12: no register form).  240: one barrier per iteration, atomics,
// the two-level barrier, 1024 threads per box -- 128^3: 12.7 us per iteration
// against 16.5 at 256 threads, same box (profiles/r04_res3d_modes.txt).
// Other forms: an experiment build, make ab XFLAGS=-DMISOR3_RESIDENT_MODE=<bits>
#ifndef MISOR3_RESIDENT_MODE
#define MISOR3_RESIDENT_MODE 240
#endif
static int resident_mode() { return MISOR3_RESIDENT_MODE; }

// full: every box lies wholly inside the domain -- then the register form
// (REG; mode bit 12 turns it off): 128^3 at 12.2-12.6 us per iteration against
// 12.7-13.2 for the LDS-only form, same box (profiles/r04_res3d_forms.txt)
static void resident_kernel(int md, bool full, const void** fn, int* nt) {
    const bool reg = full && !(md & 4096);
    if (!(md & 64)) {
        *fn = reinterpret_cast<const void*>(k3_resident);
        *nt = kRthreads;
    } else if (md & 128) {
        *fn = reg ? reinterpret_cast<const void*>(k3_resident1<1024, true>)
                  : reinterpret_cast<const void*>(k3_resident1<1024>);
        *nt = 1024;
    } else if (md & 256) {
        *fn = reg ? reinterpret_cast<const void*>(k3_resident1<512, true>)
                  : reinterpret_cast<const void*>(k3_resident1<512>);
        *nt = 512;
    } else {
        *fn = reinterpret_cast<const void*>(k3_resident1<256>);
        *nt = 256;
    }
}

static bool resident_full(const G3& g) {
    return g.I % kRbx == 0 && g.J % kRby == 0 && g.K % kRbz == 0;
}

// boxes of the resident solve for this grid, or 0 if it cannot run here
int resident3_boxes(const G3& g) {
    if (g.koff != 0 || !g.lo_phys || !g.hi_phys) return 0;  // single domain only
    if ((long long)(g.K + 2) * g.sxy >= (1ll << 31)) return 0;
    const int nbx = (g.I + kRbx - 1) / kRbx, nby = (g.J + kRby - 1) / kRby,
              nbz = (g.K + kRbz - 1) / kRbz;
    const long long nb = (long long)nbx * nby * nbz;
    // residency of the kernel launch3_resident launches with the mailboxes
    // (k3_resident1, ~154 KB of LDS) and of its fallback without them
    // (k3_resident, ~88 KB): the smaller answer, so the count reported here is
    // one the launched kernel is admitted with
    const void* fn = nullptr;
    int nt = 0, dev = 0, cus = 0, per0 = 0, per1 = 0;
    resident_kernel(resident_mode(), resident_full(g), &fn, &nt);
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per0, reinterpret_cast<const void*>(k3_resident),
                                                     kRthreads, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per1, fn, nt, 0) != hipSuccess)
        return 0;
    const int per = per0 < per1 ? per0 : per1;
    return nb <= (long long)cus * per && nb <= 256 ? (int)nb : 0;  // 256: partials slots
}

size_t resident3_bar_bytes() { return 1024; }
static_assert(sizeof(Bar3) <= 1024, "barrier state");

// 0: launched; 1: the device refused the cooperative grid (the caller falls
// back to the streaming sweep); < 0: error
int launch3_resident(hipStream_t s, const G3& g, double* p, const double* rhs, double idx2,
                     double idy2, double idz2, double factor, double cells, double* partials,
                     DevState* st, void* bar, double* mbox) {
    const int nb = resident3_boxes(g);
    if (nb == 0) return 1;
    int nbx = (g.I + kRbx - 1) / kRbx, nby = (g.J + kRby - 1) / kRby;
    if (hipMemsetAsync(bar, 0, sizeof(Bar3), s) != hipSuccess) return -1;
    G3 ga = g;
    Bar3* b = static_cast<Bar3*>(bar);
    int md = mbox ? resident_mode() : (resident_mode() & ~(8 | 64));
    const void* fn = nullptr;
    int nt = 0;
    resident_kernel(md, resident_full(g), &fn, &nt);
    void* args[] = {&ga, &p, const_cast<double**>(&rhs), &idx2, &idy2, &idz2, &factor, &cells,
                    &partials, &st, &b, &nbx, &nby, &md, &mbox};
    int mstride = (int)((g.K + 4) * g.sxy);  // the host's mailboxes: two buffers of p's size
    void* args1[] = {&ga, &p, const_cast<double**>(&rhs), &idx2, &idy2, &idz2, &factor, &cells,
                     &partials, &st, &b, &nbx, &nby, &md, &mbox, &mstride};
    const hipError_t e =
        hipLaunchCooperativeKernel(fn, dim3(nb), dim3(nt), (md & 64) ? args1 : args, 0, s);
    if (e == hipSuccess) return 0;
    (void)hipGetLastError();  // clear the refusal
    return 1;
}

int resident3_aborted(const void* bar, hipStream_t s, int* aborted) {
    Bar3 h{};
    if (hipMemcpyAsync(&h, bar, sizeof(Bar3), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    *aborted = h.abort;
    return 0;
}

}  // namespace misor
