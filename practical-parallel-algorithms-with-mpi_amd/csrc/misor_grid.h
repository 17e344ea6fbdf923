// misor_grid.h -- the host-side state of a grid (struct misor_grid) and what
// the C-ABI units share: misor_api.hip (lifecycle, transfers, gather, tuning,
// statistics), misor_comm.hip (halo exchange and all-reduce over RCCL or the
// in-process transport), misor_plan.hip (launch geometry, chained-pass
// plans), misor_solve.hip (the solve loop) and misor_ns.hip (the NS step).
// Internal: nothing here is part of include/misor.h.
#pragma once

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "misor_internal.h"

using namespace misor;

// helpers shared by the units: not exported from libmisor.so
#define MISOR_HIDDEN __attribute__((visibility("hidden")))

// record an error message for misor_last_error and return code
MISOR_HIDDEN int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess)                                                             \
            return fail(MISOR_EHIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                        \
    } while (0)

#define NCCLCHK(x)                                                                        \
    do {                                                                                  \
        ncclResult_t r_ = (x);                                                            \
        if (r_ != ncclSuccess)                                                            \
            return fail(MISOR_ECOMM, "%s: %s (%s:%d)", #x, ncclGetErrorString(r_),        \
                        __FILE__, __LINE__);                                              \
    } while (0)

// kP2: third pressure buffer of decomposed runs (the pipelined pass loop of
// misor_solve_rb_n writes pass k's result while pass k-1's source is kept)
enum { kP0 = 0, kP1 = 1, kRhs = 2, kU = 3, kV = 4, kF = 5, kG = 6, kP2 = 7, kNumFields = 8 };

// In-process transport: every rank of the group is a misor_grid owned by its
// own host thread of ONE process (any devices, including all on one GPU).
// Collectives are a host barrier plus device-to-device copies; the sum is
// combined in rank order.  It exists so the decomposed kernels can be run and
// checked on a single-GPU machine; across GPUs the RCCL path is used.
struct LocalGroup {
    int n = 0;
    std::vector<misor_grid*> members;
    std::vector<double> vals;  // n * kMaxT scratch for all-reduce
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    long long generation = 0;
    int joined = 0, left = 0;

    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        const long long gen = generation;
        if (++arrived == n) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};

struct misor_grid {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    misor_desc desc{};
    misor_local loc{};
    long long pitch = 0, rows = 0, elems = 0;
    double* fld[kNumFields] = {};
    int np = 2;   // pressure buffers: 2 (ping-pong), 3 on decomposed runs
    int cur = 0;  // which one (0 .. np-1, see pbuf) holds the current pressure
    int rhs_halo = 0;  // depth of rhs's exchanged halo still valid (0: rhs changed)
    // the current pressure buffer's halo (cells of the neighbours) predates the
    // last solve: a solve leaves it as the reference's solve loop does (its
    // exchange opens each iteration, assignment-5/skeleton/src/solver.c:607);
    // the next reader of it -- adaptUV, a download of p -- exchanges first
    // (p_halo), the next solve exchanges at its start anyway
    bool p_stale = false;
    // u, v versions: every entry point that writes u or v bumps uv_ver;
    // adaptUV leaves max |u|, |v| partials in max_partials (max_ver = uv_ver)
    unsigned uv_ver = 1, max_ver = 0;
    double* max_partials = nullptr;
    // f, g, rhs versions: every write of f, g or rhs from outside bumps fgr_ver;
    // the fused computeFG (ns_fuse) leaves rhs computed from its f, g with dt
    // fused_dt (fused_ver = fgr_ver), so computeRHS only completes the cells
    // next to a neighbour rank
    bool ns_fuse = true;
    unsigned fgr_ver = 1, fused_ver = 0;
    double fused_dt = 0.0;

    // sweep
    SweepParams sp{};
    int nbx = 0, nby = 0, nparts = 0, partials_cap = 0;
    double* partials = nullptr;  // two slots of partials_cap doubles (by pass parity)
    bool finish2 = true;  // single rank: two-level loop test (MISOR_TUNE_FINISH2 = 0: one kernel)
    DevState* st = nullptr;
    DevState* st_host = nullptr;  // pinned
    int last_iters = 0;
    // solveRB's loop test near its threshold (MISOR_TUNE_NEAR_BAND): relative
    // band of eps^2 whose iterations are re-summed exactly (exact_tail); 0: off
    double near_rel = 1e-10;
    int near_exp = 10;
    double* rsq = nullptr;  // exact_tail: r^2 per cell (allocated on first use)
    bool small_solve = true;  // whole-solve LDS kernel when p fits (single rank)
    // MISOR_TUNE_RES_LITE: single-rank 10-iteration split-ring passes count the
    // residual of their inner iterations on one row in S (misor_solve.hip)
    bool res_lite = true;
    bool lite_block = false;  // the rest of this solve counts in full (a lower bound missed)

    // temporally blocked sweep (sor_tb.hip): T iterations per pass over HBM
    int tsteps = kDefaultTsteps;  // requested T (1: single-iteration kernel)
    bool tsteps_set = false;      // T requested by MISOR_TUNE_TSTEPS (else the default rule)
    bool short_plan = false;      // capped solves may run as kShortT-iteration split-ring passes
    bool short_all = false;       // ... every solve of more than kDefaultTsteps iterations
    bool short_all_lite = false;  // ... the same while res_lite is on
    SweepParams tp{};             // its launch geometry (for T = tsteps)
    int tb_nparts = 0;
    int tb_rows_req = 0;          // MISOR_TUNE_TB_ROWS (0: automatic)
    bool tb_persistent = true;    // MISOR_TUNE_TB_PERSISTENT: work-queue launches
    int tb_reserve = kTbReserve;  // MISOR_TUNE_TB_RESERVE: slots a pipelined interior launch
                                  // leaves to the communication / edge-block streams
    int* tb_queue = nullptr;      // 8 per-XCD block counters of a persistent launch + its exit count
    // chained passes (sor_tb.h rb_tbc_kernel; MISOR_TUNE_TB_CHAIN): the initial
    // segment list of every pass length and part (0: whole pass, 1: interior
    // blocks, 2: edge blocks of a pipelined decomposed pass), and two work
    // areas (parts 0 / 1, part 2: they run concurrently on two streams)
    int tb_chain = -1;  // 1 on, 0 off, -1 automatic: on for local blocks below kChainCells
    // (each plan: the list of the main kernel and of the edge kernel --
    // columns at a physical left / right side, launched beside it on xstream)
    struct ChainList {
        unsigned long long* tmpl = nullptr;
        int nseg0 = 0, blocks = 0;
        int run[9] = {};  // XCD runs of the list
    };
    struct ChainPlan {
        ChainList main, edge;
        int reserve = -1;  // part 1 of a pipelined pass: the slots it leaves to part 2
        bool built = false;
    } chain_plan[2][kMaxT + 1][3];  // [the default variant's / the split ring's][T][part]
    int* tb_work[4] = {nullptr, nullptr, nullptr, nullptr};  // main / edge x parts 0-1 / 2
    long long tb_work_bytes[4] = {0, 0, 0, 0};
    hipStream_t xstream[2] = {nullptr, nullptr};  // edge kernels (parts 0-1 / 2)
    hipEvent_t ev_fork[2] = {}, ev_join[2] = {};
    // MISOR_CHAIN_TRACE=1: per-block timeline of the last chained pass (diagnostics)
    unsigned long long* chain_trace = nullptr;
    long long chain_trace_blocks = 0, chain_trace_last = 0;

    // reductions
    double* red_partials = nullptr;
    double* red_out = nullptr;   // 4 doubles on device
    double* red_host = nullptr;  // 4 doubles pinned

    // NS
    bool ns_ready = false;
    NsLaunch nl{};

    // multi-GPU
    bool dist = false;
    ncclComm_t comm = nullptr;
    int nbr[kDirs] = {-1, -1, -1, -1, -1, -1, -1, -1};  // L R B T BL BR TL TR
    HaloPlan plan[2 * kMaxT + 2] = {};                   // by halo depth 1 .. 2*kMaxT + 1
    int max_depth = 2;                                   // deepest plan built
    std::shared_ptr<LocalGroup> local;                   // in-process transport
    bool overlap = true;            // exchange on cstream while the interior sweeps
    hipStream_t cstream = nullptr;  // communication stream
    hipEvent_t ev_s = nullptr, ev_x = nullptr, ev_d = nullptr;
    hipEvent_t ev_i[2] = {}, ev_dk[2] = {};  // interior blocks / decide of pass k, by k & 1
    hipEvent_t ev_e2[2] = {};                // edge blocks of pass k on cstream, by k & 1
#ifdef MISOR_PROXY
    bool proxy = false;  // MISOR_PROXY_SIDES: a measurement proxy, fields meaningless
#endif
    double* sendbuf = nullptr;
    double* recvbuf = nullptr;
    double* gbuf = nullptr;  // misor_gather: this rank's owned block, packed
    long long gbuf_cap = 0;
    // in-process transport, event-driven: device work of different ranks is
    // ordered by HIP events only (no host-device synchronisation); the host
    // threads meet at barriers just to publish which event records to wait on
    hipEvent_t lx_pk = nullptr, lx_cp = nullptr;  // exchange: my send buffer packed / copies done
    hipEvent_t la_val[2] = {}, la_rd[2] = {}, la_cmb[2] = {};  // all-reduce, by parity
    double* la_stage = nullptr;   // 2 x kMaxT: my value, by all-reduce parity
    double* la_gather = nullptr;  // 2 x nranks x kMaxT: every rank's value, by parity
    long long la_gen = 0;
    bool comm_dead = false;       // the RCCL communicator was aborted (error / timeout)
    // communication timing inside a timed solve: start/stop event pairs of the
    // halo exchanges (0) and residual all-reduces (1) of the current batch
    bool comm_timing = false;
    std::vector<hipEvent_t> cev[2];
    size_t cev_used[2] = {0, 0};

    // stats
    bool timing = false;
    std::vector<hipEvent_t> ev;
    misor_stats stats{};
    // NS kernel timing (misor_stats.ns_ms): start/stop event pairs by kernel
    // group, resolved by misor_get_stats (or when a pool is full)
    std::vector<hipEvent_t> nev[3];
    size_t nev_used[3] = {0, 0, 0};
};

// pressure buffer x (mod np)
inline double* pbuf(misor_grid* g, long long x) {
    const int b = (int)(x % g->np);
    return g->fld[b == 2 ? kP2 : kP0 + b];
}

// ---- shared helpers (defined in the unit named beside each group) ----

// misor_comm.hip
MISOR_HIDDEN int allreduce(misor_grid* g, double* dev, int n, int is_max, hipStream_t s = nullptr);
MISOR_HIDDEN void build_plan(misor_grid* g, int d);
MISOR_HIDDEN int collect_comm_times(misor_grid* g);
MISOR_HIDDEN int exchange(misor_grid* g, double* field, int d, hipStream_t s = nullptr);
MISOR_HIDDEN int p_halo(misor_grid* g);
MISOR_HIDDEN int wait_stream(misor_grid* g, hipStream_t s);

// misor_plan.hip
MISOR_HIDDEN bool chain_on(const misor_grid* g, int variant);
MISOR_HIDDEN int chain_plan(misor_grid* g, int variant, int Tp, int part,
                      const misor_grid::ChainPlan** out);
MISOR_HIDDEN int configure_sweep(misor_grid* g, int variant, int rows, int remap);
MISOR_HIDDEN int configure_tb(misor_grid* g, int T, int variant, int rows);
MISOR_HIDDEN int default_tsteps(const misor_grid* g, int variant);
MISOR_HIDDEN void drop_chain_plans(misor_grid* g);
MISOR_HIDDEN int effective_tsteps(const misor_grid* g);
MISOR_HIDDEN int ensure_partials(misor_grid* g, int n);
MISOR_HIDDEN int pick_rows_per_block(int ni, int nj, int waves);
MISOR_HIDDEN void tb_geometry(const misor_grid* g, int T, SweepParams& tp);
MISOR_HIDDEN int tb_parts(const SweepParams& tp);

// misor_solve.hip
MISOR_HIDDEN int solve_rb_from(misor_grid* g, int itermax, int it0, double res0, int* iters,
                         double* res, bool* hand_off);

// misor_ns.hip
MISOR_HIDDEN int collect_ns_times(misor_grid* g);
