// misor_comm.hip -- communication of a decomposed grid: the 8-neighbour halo
// plans, the depth-d exchange and the all-reduce, over RCCL or the in-process
// transport (LOCAL: groups), with a progress timeout (misor_grid.h).

#include "misor_grid.h"

// Regions of the 8-neighbour exchange at halo depth d.  A rank sends the
// cells it owns (interior, plus ghost cells on its physical sides) next to each
// neighbour; ranks in one process row share nj and their physical top/bottom,
// ranks in one process column share ni, so send and receive extents match.
void build_plan(misor_grid* g, int d) {
    const int ni = g->loc.ni, nj = g->loc.nj;
    const int* nb = g->nbr;
    const int cl = nb[0] >= 0 ? 1 : 0, ch = nb[1] >= 0 ? ni : ni + 1;
    const int rl = nb[2] >= 0 ? 1 : 0, rh = nb[3] >= 0 ? nj : nj + 1;
    HaloRegion S[kDirs] = {
        {1, rl, d, rh - rl + 1, 0},      {ni - d + 1, rl, d, rh - rl + 1, 0},
        {cl, 1, ch - cl + 1, d, 0},      {cl, nj - d + 1, ch - cl + 1, d, 0},
        {1, 1, d, d, 0},                 {ni - d + 1, 1, d, d, 0},
        {1, nj - d + 1, d, d, 0},        {ni - d + 1, nj - d + 1, d, d, 0}};
    HaloRegion R[kDirs] = {
        {1 - d, rl, d, rh - rl + 1, 0},  {ni + 1, rl, d, rh - rl + 1, 0},
        {cl, 1 - d, ch - cl + 1, d, 0},  {cl, nj + 1, ch - cl + 1, d, 0},
        {1 - d, 1 - d, d, d, 0},         {ni + 1, 1 - d, d, d, 0},
        {1 - d, nj + 1, d, d, 0},        {ni + 1, nj + 1, d, d, 0}};
    HaloPlan& P = g->plan[d];
    long long so = 0, ro = 0;
    for (int k = 0; k < kDirs; ++k) {
        if (nb[k] < 0) S[k].w = S[k].h = R[k].w = R[k].h = 0;
        S[k].off = so;
        R[k].off = ro;
        so += (long long)S[k].w * S[k].h;
        ro += (long long)R[k].w * R[k].h;
        P.send[k] = S[k];
        P.recv[k] = R[k];
    }
    P.total = so > ro ? so : ro;
}

// a start/stop event pair for timing one communication step (kind 0: halo
// exchange, 1: all-reduce) of the current batch; false when not timing
static bool comm_pair(misor_grid* g, int kind, hipEvent_t* e0, hipEvent_t* e1) {
    if (!g->comm_timing) return false;
    std::vector<hipEvent_t>& v = g->cev[kind];
    size_t& u = g->cev_used[kind];
    while (v.size() < 2 * (u + 1)) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return false;
        v.push_back(e);
    }
    *e0 = v[2 * u];
    *e1 = v[2 * u + 1];
    ++u;
    return true;
}

// add the timed communication steps of the batch just synchronised to the stats
int collect_comm_times(misor_grid* g) {
    for (int kind = 0; kind < 2; ++kind) {
        for (size_t k = 0; k < g->cev_used[kind]; ++k) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, g->cev[kind][2 * k], g->cev[kind][2 * k + 1]));
            if (kind == 0) {
                g->stats.halo_ms += ms;
                g->stats.halos++;
            } else {
                g->stats.allreduce_ms += ms;
                g->stats.allreduces++;
            }
        }
        g->cev_used[kind] = 0;
    }
    return MISOR_OK;
}

static double comm_timeout_s() {
    const char* e = getenv("MISOR_COMM_TIMEOUT");
    const double v = e && *e ? atof(e) : 0.0;
    return v > 0 ? v : 600.0;
}

// Wait for stream s.  With an RCCL communicator, poll instead of blocking:
// an asynchronous communicator error (a peer died, a link failed:
// ncclCommGetAsyncError) or no progress for MISOR_COMM_TIMEOUT seconds
// (default 600) aborts the communicator and returns MISOR_ECOMM on this rank,
// where the reference's MPI default (MPI_ERRORS_ARE_FATAL) would end the job;
// a blocked hipStreamSynchronize would hang instead.
int wait_stream(misor_grid* g, hipStream_t s) {
    if (!g->comm) {
        HIPCHK(hipStreamSynchronize(s));
        return MISOR_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = comm_timeout_s();
    for (long spins = 0;; ++spins) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return MISOR_OK;
        if (e != hipErrorNotReady)
            return fail(MISOR_EHIP, "stream wait: %s", hipGetErrorString(e));
        ncclResult_t ar = ncclSuccess;
        const bool bad = ncclCommGetAsyncError(g->comm, &ar) == ncclSuccess &&
                         ar != ncclSuccess && ar != ncclInProgress;
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (bad || el > limit) {
            (void)ncclCommAbort(g->comm);
            g->comm = nullptr;
            g->comm_dead = true;
            if (bad)
                return fail(MISOR_ECOMM, "RCCL asynchronous error: %s", ncclGetErrorString(ar));
            return fail(MISOR_ECOMM, "communication made no progress for %.0f s "
                                     "(MISOR_COMM_TIMEOUT)", limit);
        }
        if (spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

#define COMMCHK(g)                                                                        \
    do {                                                                                  \
        if ((g)->comm_dead)                                                               \
            return fail(MISOR_ECOMM, "the communicator was aborted by an earlier error"); \
    } while (0)

// one 8-neighbour exchange of `field` at depth d on stream s (default: the
// grid stream): pack kernel, transport, unpack kernel
int exchange(misor_grid* g, double* field, int d, hipStream_t s) {
    if (!g->dist) return MISOR_OK;
    COMMCHK(g);
    if (!s) s = g->stream;
    const HaloPlan& P = g->plan[d];
    hipEvent_t t0 = nullptr, t1 = nullptr;
    const bool timed = comm_pair(g, 0, &t0, &t1);
    if (timed) HIPCHK(hipEventRecord(t0, s));
    if (g->local) {
        // In-process transport.  Rank q's copies of my send buffer and my own
        // unpack of the previous exchange must be done before I pack again;
        // my copies of q's buffer wait for q's pack.  Barrier 1: every rank has
        // recorded its pack event; barrier 2: every rank has recorded its copy
        // event (so the next exchange waits on this exchange's records).
        static const int opposite[kDirs] = {1, 0, 3, 2, 7, 6, 5, 4};
        LocalGroup& G = *g->local;
        HIPCHK(hipStreamWaitEvent(s, g->lx_cp, 0));
        for (int k = 0; k < kDirs; ++k)
            if (g->nbr[k] >= 0) HIPCHK(hipStreamWaitEvent(s, G.members[g->nbr[k]]->lx_cp, 0));
        launch_pack(s, field, g->pitch, P, g->sendbuf);
        HIPCHK(hipEventRecord(g->lx_pk, s));
        G.barrier();
        for (int k = 0; k < kDirs; ++k) {
            if (g->nbr[k] < 0) continue;
            const misor_grid* q = G.members[g->nbr[k]];
            const HaloRegion& sr = q->plan[d].send[opposite[k]];
            const HaloRegion& rr = P.recv[k];
            HIPCHK(hipStreamWaitEvent(s, q->lx_pk, 0));
            HIPCHK(hipMemcpyAsync(g->recvbuf + rr.off, q->sendbuf + sr.off,
                                  sizeof(double) * (size_t)rr.w * rr.h,
                                  hipMemcpyDeviceToDevice, s));
        }
        launch_unpack(s, field, g->pitch, P, g->recvbuf);
        HIPCHK(hipEventRecord(g->lx_cp, s));
        if (timed) HIPCHK(hipEventRecord(t1, s));
        HIPCHK(hipGetLastError());
        G.barrier();
        return MISOR_OK;
    }
    launch_pack(s, field, g->pitch, P, g->sendbuf);
    NCCLCHK(ncclGroupStart());
    for (int k = 0; k < kDirs; ++k) {
        if (g->nbr[k] < 0) continue;
        const size_t ns = (size_t)P.send[k].w * P.send[k].h;
        const size_t nr = (size_t)P.recv[k].w * P.recv[k].h;
        NCCLCHK(ncclSend(g->sendbuf + P.send[k].off, ns, ncclDouble, g->nbr[k], g->comm, s));
        NCCLCHK(ncclRecv(g->recvbuf + P.recv[k].off, nr, ncclDouble, g->nbr[k], g->comm, s));
    }
    NCCLCHK(ncclGroupEnd());
    launch_unpack(s, field, g->pitch, P, g->recvbuf);
    if (timed) HIPCHK(hipEventRecord(t1, s));
    HIPCHK(hipGetLastError());
    return MISOR_OK;
}

// the current pressure buffer's halo, exchanged 2 deep if a solve left it stale
int p_halo(misor_grid* g) {
    if (!g->dist || !g->p_stale) return MISOR_OK;
    int rc = exchange(g, pbuf(g, g->cur), 2);
    if (rc == MISOR_OK) g->p_stale = false;
    return rc;
}

// all-reduce of n <= kMaxT device doubles (sum or max) across the ranks, on
// stream s (default: the grid stream)
int allreduce(misor_grid* g, double* dev, int n, int is_max, hipStream_t s) {
    if (!g->dist) return MISOR_OK;
    COMMCHK(g);
    if (!s) s = g->stream;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    const bool timed = comm_pair(g, 1, &t0, &t1);
    if (timed) HIPCHK(hipEventRecord(t0, s));
    if (g->local) {
        // In-process transport: every rank stages its values (slot by parity,
        // reused two all-reduces later once every rank has read it), gathers
        // every rank's staged values after barrier 1 and combines them in rank
        // order on its device; barrier 2 publishes the read events.
        LocalGroup& G = *g->local;
        const int par = (int)(g->la_gen++ & 1);
        double* stage = g->la_stage + par * kMaxT;
        double* gather = g->la_gather + (size_t)par * G.n * kMaxT;
        HIPCHK(hipStreamWaitEvent(s, g->la_cmb[par], 0));
        for (int q = 0; q < G.n; ++q) HIPCHK(hipStreamWaitEvent(s, G.members[q]->la_rd[par], 0));
        HIPCHK(hipMemcpyAsync(stage, dev, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipEventRecord(g->la_val[par], s));
        G.barrier();
        for (int q = 0; q < G.n; ++q) {
            const misor_grid* o = G.members[q];
            HIPCHK(hipStreamWaitEvent(s, o->la_val[par], 0));
            HIPCHK(hipMemcpyAsync(gather + (size_t)q * kMaxT, o->la_stage + par * kMaxT,
                                  sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        }
        HIPCHK(hipEventRecord(g->la_rd[par], s));
        launch_local_combine(s, gather, G.n, n, is_max, dev);
        HIPCHK(hipEventRecord(g->la_cmb[par], s));
        if (timed) HIPCHK(hipEventRecord(t1, s));
        HIPCHK(hipGetLastError());
        G.barrier();
        return MISOR_OK;
    }
    NCCLCHK(ncclAllReduce(dev, dev, n, ncclDouble, is_max ? ncclMax : ncclSum, g->comm, s));
    if (timed) HIPCHK(hipEventRecord(t1, s));
    return MISOR_OK;
}
