/*
 * misor.h -- C ABI of libmisor: MI355X-native red-black SOR for the 2D
 * pressure Poisson equation and the 2D Navier-Stokes step kernels around it.
 *
 * This is the drop-in boundary for the reference's L4 solver layer.  The
 * reference has no FFI: its C `main` calls plain functions declared in
 * solver.h.  Each entry point below replaces one of them (cited per function);
 * the host programs in practical-parallel-algorithms-with-mpi_amd/host/ keep
 * the reference's own names (initSolver, solveRB, computeFG, ...) as thin
 * wrappers over these calls, see INTEGRATION.md.
 *
 * Conventions
 *  - Plain C: pointers, sizes, scalars.  No HIP/torch types in signatures.
 *  - Host arrays exchanged with the library use the reference layout:
 *    (ni+2) x (nj+2) doubles, row-major, i fastest, A(i,j) = a[j*(ni+2)+i]
 *    (assignment-4/src/solver.c:16), where (ni,nj) is the LOCAL block of this
 *    rank (= (imax,jmax) on one GPU).
 *  - Every function returns MISOR_OK (0) or a negative MISOR_E* code;
 *    misor_last_error() describes the last failure of the calling thread.
 *    The reference prints and exit(EXIT_FAILURE)s instead (allocate.c:18-35,
 *    parameter.c:32-35); the host wrappers map a non-zero return to exactly
 *    that.
 *  - Device fields live in HBM for the lifetime of the grid; nothing is
 *    copied across the boundary except by misor_upload / misor_download.
 */
#ifndef MISOR_H
#define MISOR_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MISOR_OK 0
#define MISOR_EINVAL (-1)   /* bad argument */
#define MISOR_EHIP (-2)     /* HIP runtime error */
#define MISOR_ENOMEM (-3)   /* device allocation failed */
#define MISOR_ECOMM (-4)    /* RCCL error */
#define MISOR_ESTATE (-5)   /* call not valid in this state */

/* field ids */
enum { MISOR_P = 0, MISOR_RHS = 1, MISOR_U = 2, MISOR_V = 3, MISOR_F = 4, MISOR_G = 5 };

/* boundary flags, assignment-5/sequential/src/solver.h:11 */
enum { MISOR_NOSLIP = 1, MISOR_SLIP = 2, MISOR_OUTFLOW = 3, MISOR_PERIODIC = 4 };

/* special boundary condition, selected in the reference by strcmp on the
 * problem name (assignment-5/sequential/src/solver.c:345,349) */
enum { MISOR_PROBLEM_NONE = 0, MISOR_PROBLEM_DCAVITY = 1, MISOR_PROBLEM_CANAL = 2 };

/* SOR update form: solveRB (P -= factor*r, factor includes omega,
 * assignment-4/src/solver.c:189,211) or solveRBA (P -= omega*factor*r,
 * :250,273) */
enum { MISOR_SOLVE_RB = 0, MISOR_SOLVE_RBA = 1 };

typedef struct misor_grid misor_grid;

typedef struct {
    /* global grid and the SOR parameters of Solver
     * (assignment-4/src/solver.h:11-22, assignment-5/sequential/src/solver.h:13-32) */
    int imax, jmax;     /* interior cells, whole domain */
    double dx, dy;      /* xlength/imax, ylength/jmax */
    double omega, eps;
    int itermax;
    int variant;        /* MISOR_SOLVE_RB or MISOR_SOLVE_RBA */
    int device;         /* HIP device ordinal; -1 = current device */
    /* 2D domain decomposition (assignment-5/skeleton/src/solver.c:445-473).
     * nranks = 1 for a single GPU; then the rest is ignored. */
    int nranks, rank;
    int dims[2];        /* process grid {x, y}; {0,0} = MPI_Dims_create rule */
    const void* comm_id; /* MISOR_COMM_ID_BYTES from misor_comm_unique_id() on rank 0:
                          * one process per GPU, halos and reductions over RCCL.
                          * Bytes starting with "LOCAL:<name>" select the in-process
                          * transport instead: the nranks grids of group <name> are
                          * created and driven by nranks host threads of ONE process
                          * (any devices, also all on one GPU); every member must make
                          * the same sequence of calls, as with RCCL. */
} misor_desc;

#define MISOR_COMM_ID_BYTES 128

/* NS physics parameters (assignment-5/sequential/src/solver.h:13-32) */
typedef struct {
    double xlength, ylength;
    double re, gx, gy, gamma, tau;
    int bcLeft, bcRight, bcBottom, bcTop;
    int problem;        /* MISOR_PROBLEM_* */
} misor_ns_desc;

/* what this rank owns (for uploads/downloads and tests) */
typedef struct {
    int ni, nj;         /* local interior cells */
    int ioff, joff;     /* global index of local cell (0,0) */
    int coords[2], dims[2];
    int neighbours[4];  /* left, right, bottom, top rank or -1 */
    long long pitch;    /* device row pitch in doubles */
} misor_local;

/* per-grid counters; sweep_ms is summed from HIP events recorded around
 * every sweep pass when timing is enabled (misor_enable_timing).  A pass is
 * one sweep kernel launch (two for an overlapped decomposed pass: interior
 * blocks, then boundary blocks) doing iters_per_pass red+black iterations
 * (MISOR_TUNE_TSTEPS). */
typedef struct {
    long long sweeps;       /* red+black iterations executed on the device */
    long long launches;     /* passes launched (incl. early-exited) */
    double sweep_ms;        /* total device time of timed passes (timing on) */
    long long timed_sweeps; /* iterations computed by the timed passes */
    long long timed_passes; /* passes covered by sweep_ms */
    int iters_per_pass;     /* T of the last multi-block solve (1: single sweep) */
    int tb_variant;         /* its TB variant (MISOR_TUNE_TB_VARIANT; -1: single sweep) */
    /* decomposed solves, timing on: HIP events around every halo exchange
     * (pack + transport + unpack) and every residual all-reduce (+ loop test)
     * on the stream that runs it (the communication stream when overlapped) */
    double halo_ms;         /* total device time of the solve's halo exchanges */
    long long halos;        /* exchanges covered by halo_ms */
    double allreduce_ms;    /* total device time of the residual all-reduces */
    long long allreduces;   /* all-reduces covered by allreduce_ms */
    int chained;            /* 1: the last multi-block solve's passes were chained runs
                             * (sor_tb.h rb_tbc_kernel / sor_tbh.h rb_tbhc_kernel) */
    /* NS step kernels, timing on: HIP events on the grid stream around each
     * launch.  [0] computeFG (+ the fused computeRHS, ns_kernels.hip
     * fg_rhs_kernel), [1] adaptUV (+ the next dt's max |u|, |v| partials,
     * adapt_absmax_kernel), [2] normalizePressure (max |p|, exact sum,
     * subtract: absmax2 + finish_reduce, exact_sum, sub_mean kernels) */
    double ns_ms[3];
    long long ns_calls[3];
    /* solves whose residual lower bounds (MISOR_TUNE_RES_LITE) missed once: the
     * pass redone counting every cell, the rest of the solve so */
    long long lite_misses;
} misor_stats;

const char* misor_last_error(void);
const char* misor_version(void);

/* decomposition rule of MPI_Dims_create(n, 2) + sizeOfRank
 * (assignment-5/skeleton/src/solver.c:30-32,445,472-473); host-only */
int misor_decompose(int nranks, int rank, int imax, int jmax, const int dims_in[2],
                    misor_local* out);

/* rank 0 calls this and ships the bytes to the other ranks out of band */
int misor_comm_unique_id(void* id_out /* MISOR_COMM_ID_BYTES */);

/* replaces the allocation half of initSolver (assignment-4/src/solver.c:83-97,
 * assignment-5/sequential/src/solver.c:59-91): all six fields, zeroed */
int misor_create(misor_grid** out, const misor_desc* desc);
void misor_destroy(misor_grid* g);
int misor_local_info(const misor_grid* g, misor_local* out);

/* stream the grid's kernels run on (hipStream_t as void*); NULL = own stream */
int misor_set_stream(misor_grid* g, void* hip_stream);
int misor_synchronize(misor_grid* g);

int misor_upload(misor_grid* g, int field, const double* host);
int misor_download(misor_grid* g, int field, double* host);
/* collectResult / assembleResult (assignment-5/skeleton/src/solver.c:234-359):
 * collective over the ranks of a decomposed grid.  Rank 0 receives the whole
 * field, (imax+2) x (jmax+2) doubles in the reference layout, in `host_global`;
 * every rank contributes its interior plus the ghost layer on its physical
 * sides; other ranks pass NULL.  With one rank it is misor_download. */
int misor_gather(misor_grid* g, int field, double* host_global);
/* exchange (assignment-5/skeleton/src/solver.c:137-165): collective over the
 * ranks of a decomposed grid.  The `depth`-deep halo of `field` (1 <= depth <=
 * the deepest halo the grid supports, >= 2) receives the neighbours' owned
 * cells, edges and corners, from all 8 neighbours; ghost cells on physical
 * sides are not touched.  MISOR_P is the current pressure buffer.  With one
 * rank it does nothing.  The solve and the NS steps exchange internally;
 * this entry point is the skeleton's own call (and its printExchange check). */
int misor_exchange(misor_grid* g, int field, int depth);
/* number of visible GPUs (host programs map rank -> device) */
int misor_device_count(int* n);
/* ranks of the grid's communicator as its transport counts them: ncclCommCount
 * of the RCCL communicator (MPI_Comm_size of the reference's solver->comm,
 * assignment-5/skeleton/src/solver.c:408,452), the member count of an
 * in-process group, 1 for a single-rank grid */
int misor_comm_ranks(const misor_grid* g, int* n);
/* fill a field (incl. ghosts) with a constant; initSolver of NS (solver.c:92-99) */
int misor_fill(misor_grid* g, int field, double value);

/* initSolver of assignment-4 (solver.c:99-123): p = sin(4 pi i dx) +
 * sin(4 pi j dy), rhs = sin(2 pi i dx) for problem 2 else 0, incl. ghosts.
 * The 1-D sine tables are evaluated on the host with libm exactly as the
 * reference does, so the fields are bit-identical to it. */
int misor_poisson_init(misor_grid* g, double xlength, double ylength, int problem);

/* solveRB / solveRBA (assignment-4/src/solver.c:179-299): red-black SOR
 * with Neumann ghost copy after each iteration, until res < eps^2 or itermax.
 * *iters = iterations done (the reference prints it, :237), *res = final
 * residual (sum r^2 / (imax*jmax)).  Either output may be NULL.
 * Decomposed: as the reference's MPI loop (assignment-5/skeleton/src/
 * solver.c:603-607, an exchange opens every iteration) the solve leaves the
 * final field's inter-rank halo to its next reader: misor_adapt_uv and a
 * misor_download of MISOR_P exchange it first (2 deep), the next solve at its
 * start; misor_gather reads owned cells only. */
int misor_solve_rb(misor_grid* g, int* iters, double* res);
/* the same with an explicit cap that overrides desc.itermax for this call */
int misor_solve_rb_n(misor_grid* g, int itermax, int* iters, double* res);
/* The reference's lexicographic Gauss-Seidel SOR `solve` (what its programs
 * call): assignment-4/src/solver.c:126-177 (xorder = MISOR_LEX_A4) and
 * assignment-5/sequential/src/solver.c:140-191 (xorder = MISOR_LEX_SEQ; the
 * two differ only in the order of the stencil terms), bit for bit, as an
 * anti-diagonal wavefront in one workgroup.  Single rank, variant RB only. */
enum { MISOR_LEX_A4 = 0, MISOR_LEX_SEQ = 1 };
int misor_solve_lex(misor_grid* g, int xorder, int* iters, double* res);

/* NS step kernels (assignment-5/sequential/src/solver.c) */
int misor_ns_setup(misor_grid* g, const misor_ns_desc* ns);
int misor_compute_timestep(misor_grid* g, double dt_bound, double tau, double* dt_out); /* :219-234 */
int misor_set_dt(misor_grid* g, double dt);
int misor_set_boundary_conditions(misor_grid* g);          /* :236-337 */
int misor_set_special_boundary_condition(misor_grid* g);   /* :339-358 */
int misor_compute_fg(misor_grid* g);                        /* :360-436 */
int misor_compute_rhs(misor_grid* g);                       /* :122-138 */
int misor_normalize_pressure(misor_grid* g);                /* :204-217 */
int misor_adapt_uv(misor_grid* g);                          /* :438-455 */
/* max |u| and max |v| over all cells incl. ghosts (maxElement, :193-202) */
int misor_max_uv(misor_grid* g, double* umax, double* vmax);

/* launch-geometry knobs of the sweep kernel (defaults chosen by measurement,
 * DESIGN.md); results are bit-identical for every setting */
enum {
    MISOR_TUNE_SWEEP_VARIANT = 1,  /* 0..7: strips per workgroup x rows in flight x nt stores */
    MISOR_TUNE_ROWS_PER_BLOCK = 2, /* rows one workgroup marches; <= 0: automatic */
    MISOR_TUNE_XCD_REMAP = 3,      /* 1: adjacent blocks on one XCD (shared L2 halos) */
    MISOR_TUNE_SMALL_SOLVE = 4,    /* 1 (default): whole solve in one workgroup, p in LDS,
                                    * when the grid fits (single rank, <= 128^2 cells) */
    MISOR_TUNE_OVERLAP = 5,        /* decomposed: 1 (default) = halo exchange and residual
                                    * all-reduce on a second stream, overlapped with the
                                    * interior blocks of the sweep; 0 = serial */
    MISOR_TUNE_TSTEPS = 6,         /* iterations per pass over HBM, 1..12: 1 = single-
                                    * iteration sweep kernel, T >= 2 = temporally blocked
                                    * kernel (T iterations per read of p and rhs); the
                                    * iteration count and every bit of p are unchanged.
                                    * A request binds every pass to T (no short pass
                                    * plan); <= 0 returns to the default rule */
    MISOR_TUNE_TB_VARIANT = 7,     /* temporally blocked kernel: 0..4 strips per workgroup x
                                    * rows in flight */
    MISOR_TUNE_TB_ROWS = 8,        /* temporally blocked kernel: rows per block; <= 0: auto
                                    * (a multiple of the kernel's rhs ring) */
    MISOR_TUNE_TB_PERSISTENT = 9,  /* temporally blocked kernel: 1 (default) = as many
                                    * workgroups as are resident, taking blocks from per-XCD
                                    * work queues; 0 = one workgroup per block */
    MISOR_TUNE_NS_FUSE = 10,       /* 1 (default): misor_compute_fg also computes RHS in the
                                    * same pass over u, v (computeRHS then only completes the
                                    * cells next to a neighbour rank); 0 = separate kernels */
    MISOR_TUNE_FINISH2 = 11,       /* single rank: 1 (default) = two-level loop test
                                    * (partial sums, then the test); 0 = one kernel */
    MISOR_TUNE_TB_RESERVE = 12,    /* decomposed, overlapped: workgroup slots the persistent
                                    * interior launch leaves to the exchange / all-reduce /
                                    * edge-block streams (default 16) */
    MISOR_TUNE_TB_CHAIN = 13,      /* temporally blocked kernel, persistent, default variant:
                                    * 1 = chained vertical runs of short blocks with work
                                    * stealing (no warm-up rows between the blocks of a
                                    * run); 0 = one block per work item; -1 (default) =
                                    * chained on local blocks below 2^28 cells.  Get: 1 if
                                    * chained passes are in effect */
    MISOR_TUNE_NEAR_BAND = 14      /* solveRB's loop test near its threshold: when an
                                    * iteration's res lies within a relative 10^-value of
                                    * eps^2, that iteration and the rest of the solve are
                                    * recomputed one sweep at a time with an exact
                                    * (order-independent) sum of r^2, so the iteration count
                                    * and res do not depend on the partition.  Default 10;
                                    * >= 300: off (set by tests to force the path: -30) */,
    MISOR_TUNE_RES_LITE = 15       /* single rank, 10-iteration split-ring passes: 1
                                    * (default) = the steady chunks count the residual of
                                    * a pass's iterations but its last on one row in S, a
                                    * lower bound that the loop test accepts only where it
                                    * proves the loop goes on (not converged, not near the
                                    * threshold); otherwise the pass is redone counting
                                    * every cell and the solve continues so.  The iteration
                                    * count, res and p are the same bits either way.
                                    * 0 = every iteration counted in full */
};
int misor_set_tuning(misor_grid* g, int key, int value);
int misor_get_tuning(const misor_grid* g, int key, int* value);

/* diagnostics: with MISOR_CHAIN_TRACE=1 in the environment when the grid is
 * configured, the per-block timeline of the last chained pass (3 words per
 * block L = by * nbx + bx: start and end on the 100 MHz wall clock, workgroup
 * | 1 << 32 for the first block of a run); *n = words available */
int misor_chain_trace(misor_grid* g, unsigned long long* out, long long cap, long long* n);

int misor_enable_timing(misor_grid* g, int on);
int misor_get_stats(const misor_grid* g, misor_stats* out);
int misor_reset_stats(misor_grid* g);

/* ------------------------------------------------------------------ 3D ---
 * assignment-6's 3D Navier-Stokes solver (assignment-6/src/solver.c) on one
 * GPU: the same step as solver.h's computeTimestep / setBoundaryConditions /
 * setSpecialBoundaryCondition / computeFG / computeRHS / solve / adaptUV, with
 * a 7-point red-black pressure solve.  Fields keep the reference layout:
 * (imax+2)(jmax+2)(kmax+2) doubles, i fastest, then j, then k (solver.c:19-34).
 * Every cell value is bit-identical to the reference's; the solve's residual
 * is summed in a fixed tree order (the reference sums sequentially). */
typedef struct misor_grid3 misor_grid3;

typedef struct {
    int imax, jmax, kmax;               /* interior cells */
    double xlength, ylength, zlength;   /* domain size */
    double re, gamma, tau, omega, eps;  /* Reynolds number, upwind factor, CFL
                                         * safety, SOR relaxation, tolerance */
    double gx, gy, gz;                  /* body force */
    int itermax;                        /* solve iteration cap */
    int bcTop, bcBottom, bcLeft, bcRight, bcFront, bcBack; /* MISOR_NOSLIP ... */
    int problem;                        /* MISOR_PROBLEM_* */
    int device;                         /* HIP device; < 0: the current one */
    /* decomposition: slabs of planes along k (misor3_decompose); nranks <= 1 =
     * one GPU.  comm_id as misor_desc.comm_id (RCCL id from
     * misor_comm_unique_id, or "LOCAL:<name>" for ranks as host threads) */
    int nranks, rank;
    const void* comm_id;
} misor3_desc;

/* field ids of misor3_upload / misor3_download / misor3_fill */
enum { MISOR3_P = 0, MISOR3_RHS = 1, MISOR3_U = 2, MISOR3_V = 3, MISOR3_W = 4,
       MISOR3_F = 5, MISOR3_G = 6, MISOR3_H = 7 };

/* the slab of `rank`: kloc planes from global plane koff+1 (sizeOfRank rule,
 * assignment-6/src/comm.c:24-101, along k only); at least 2 planes per rank.
 * The reference splits over a 3D process grid; see DESIGN.md 6b.  host-only */
int misor3_decompose(int nranks, int rank, int kmax, int* kloc, int* koff);
/* initSolver (solver.c:60-143): device fields, all zero; dx = xlength/imax ...
 * Decomposed grids hold their slab: local arrays (imax+2)(jmax+2)(kloc+2) */
int misor3_create(misor_grid3** out, const misor3_desc* d);
int misor3_local_info(const misor_grid3* g, int* kloc, int* koff);
void misor3_destroy(misor_grid3* g);
/* whole field incl. ghosts, (imax+2)(jmax+2)(kmax+2) doubles */
int misor3_upload(misor_grid3* g, int field, const double* host);
int misor3_download(misor_grid3* g, int field, double* host);
int misor3_fill(misor_grid3* g, int field, double value);
/* commCollectResult's gather (assignment-6/src/comm.c:246-384) of a whole
 * field, collective: rank 0 receives (imax+2)(jmax+2)(kmax+2) doubles, the
 * other ranks pass NULL.  One rank: misor3_download */
int misor3_gather(misor_grid3* g, int field, double* host_global);
int misor3_set_dt(misor_grid3* g, double dt);
/* computeTimestep (solver.c:340-362): dt = tau * min(dtBound, dx/umax, dy/vmax,
 * dz/wmax), dtBound = 0.5*re/(1/dx^2+1/dy^2+1/dz^2) (solver.c:136-139) */
int misor3_compute_timestep(misor_grid3* g, double* dt_out);
/* max |u|, |v|, |w| over every cell incl. ghosts (maxElement, solver.c:299-310) */
int misor3_max_uvw(misor_grid3* g, double* mx3);
int misor3_set_boundary_conditions(misor_grid3* g);       /* solver.c:364-577 */
int misor3_set_special_boundary_condition(misor_grid3* g); /* solver.c:579-604 */
int misor3_compute_fg(misor_grid3* g);                    /* solver.c:606-824 */
int misor3_compute_rhs(misor_grid3* g);                   /* solver.c:145-173 */
/* solve (solver.c:175-297): red-black SOR until res < eps^2 or itermax;
 * decomposed: halos and the residual sum cross the ranks, p and the
 * iteration count are those of the single-domain solve */
int misor3_solve(misor_grid3* g, int* iters, double* res);
int misor3_adapt_uvw(misor_grid3* g);                     /* solver.c:826-853 */
int misor3_normalize_pressure(misor_grid3* g);            /* solver.c:312-338 */
int misor3_synchronize(misor_grid3* g);
/* device time of the solves (HIP events on the grid's stream around each
 * misor3_solve: its colour-pass and loop-test kernels), accumulated while
 * timing is on; enabling resets the counters */
int misor3_enable_timing(misor_grid3* g, int on);
/* launch-geometry knobs of the 3D solve; results are bit-identical for every
 * setting */
enum {
    MISOR3_TUNE_SWEEP = 1,  /* 1 (default): one fused red+black sweep launch per iteration
                             * (k-march, LDS plane ring, ping-pong p); 0: two colour-pass
                             * launches, in place */
    MISOR3_TUNE_ROWS = 2,   /* fused sweep: rows per workgroup tile, 4 / 8 / 12 */
    MISOR3_TUNE_KCHUNK = 3, /* fused sweep: planes per workgroup (>= 4; 0: automatic) */
    MISOR3_TUNE_FOLD = 4,   /* single rank, fused sweep: 1 (default) = each sweep launch first
                             * applies the previous sweep's loop test (one launch per
                             * iteration); 0 = a finish kernel after every sweep */
    MISOR3_TUNE_RHS_AHEAD = 5, /* fused sweep: plane steps between an rhs load and its first
                                * use, 1 or 2; 0 (default) = 2 on marches of >= 16 planes */
    MISOR3_TUNE_RESIDENT = 6  /* single rank: the whole solve in one cooperative launch with
                               * p resident in LDS (boxes of 32x16x16 cells, grid barriers
                               * between the colour passes) when the grid fits the device
                               * (128^3 on 256 CUs); 1 / -1 (default) = when it fits, 0 = never.
                               * misor3_get_tuning returns whether the next solve uses it */
};
int misor3_set_tuning(misor_grid3* g, int key, int value);
int misor3_get_tuning(const misor_grid3* g, int key, int* value);
int misor3_get_solve_time(const misor_grid3* g, double* ms, long long* iters);

#ifdef __cplusplus
}
#endif
#endif
