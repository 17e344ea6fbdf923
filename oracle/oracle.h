/*
 * oracle.h -- CPU restatement of the reference's red-black SOR / 2D NS path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libmisor, the host
 * programs) links, loads or calls this code.  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() use it, and only as the
 * checker.
 *
 * Every function restates one reference function (file:line given at the
 * definition in oracle.c).  The arithmetic follows the reference expression
 * order exactly and is compiled with -O2 -ffp-contract=off, so it is
 * bit-identical to the reference C compiled the same way.  That equality is
 * pinned by tests/test_oracle.py against (a) oracle/_ref, the reference
 * sources compiled in this container, and (b) the fixtures under
 * tests/golden/ (the reference's own committed p.dat / init.dat and vectors
 * generated from oracle/_ref by tests/golden/make_golden.py).
 *
 * Arrays use the reference layout: (imax+2) x (jmax+2) doubles, row-major,
 * i fastest, P(i,j) = p[j*(imax+2)+i]  (assignment-4/src/solver.c:16).
 */
#ifndef ORACLE_H
#define ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* boundary flags, assignment-5/sequential/src/solver.h:11 */
enum { ORC_NOSLIP = 1, ORC_SLIP = 2, ORC_OUTFLOW = 3, ORC_PERIODIC = 4 };
/* setSpecialBoundaryCondition selector (strcmp on the problem name) */
enum { ORC_PROBLEM_NONE = 0, ORC_PROBLEM_DCAVITY = 1, ORC_PROBLEM_CANAL = 2 };

/* ---------------- Poisson (assignment-4) ---------------- */
void orc_poisson_init(int imax, int jmax, double xlength, double ylength,
                      int problem, double* p, double* rhs);
int orc_solve_rb(int imax, int jmax, double dx, double dy, double omega,
                 double eps, int itermax, double* p, const double* rhs,
                 double* res_out);
int orc_solve_rba(int imax, int jmax, double dx, double dy, double omega,
                  double eps, int itermax, double* p, const double* rhs,
                  double* res_out);
/* xorder 0: assignment-4 solve (P(i-1)-2P+P(i+1)); 1: NS solve (P(i+1)-2P+P(i-1)) */
int orc_solve_lex(int imax, int jmax, double dx, double dy, double omega,
                  double eps, int itermax, int xorder, double* p,
                  const double* rhs, double* res_out);

/* One red-black colour pass over a sub-block with GLOBAL colour parity.
 * Used by the multi-rank CPU model (tests/test_distributed_cpu.py).  The
 * block is (ni+2) x (nj+2) with its own ghost ring; local cell (li,lj) is
 * global cell (ioff+li, joff+lj).  colour 0 updates cells with (i+j) even
 * (solveRB's pass 0), colour 1 the odd ones.  Returns sum r^2 over the
 * updated cells. */
double orc_rb_pass_block(int ni, int nj, int ioff, int joff, int colour,
                         double idx2, double idy2, double factor, double* p,
                         const double* rhs);

/* Range form of the pass above for the 2-deep-halo model of the GPU
 * decomposition; see oracle.c. */
double orc_rb_pass_range(int stride, int org, int ilo, int ihi, int jlo, int jhi,
                         int oilo, int oihi, int ojlo, int ojhi, int ioff, int joff,
                         int colour, double idx2, double idy2, double factor, double* p,
                         const double* rhs);

/* ---------------- 2D Navier-Stokes (assignment-5/sequential) ---------------- */
typedef struct {
    int imax, jmax;
    double dx, dy;
    double xlength, ylength;
    double re, gx, gy, dt, te, tau, gamma, eps, omega, dtBound;
    int itermax;
    int bcLeft, bcRight, bcBottom, bcTop;
    int problem;
    double *p, *rhs, *f, *g, *u, *v;
} orc_ns;

void orc_ns_setup(orc_ns* s); /* dx, dy, dtBound from the other fields */
void orc_ns_compute_timestep(orc_ns* s);
void orc_ns_set_bc(orc_ns* s);
void orc_ns_set_special_bc(orc_ns* s);
void orc_ns_compute_fg(orc_ns* s);
void orc_ns_compute_rhs(orc_ns* s);
void orc_ns_normalize_pressure(orc_ns* s);
void orc_ns_adapt_uv(orc_ns* s);
double orc_ns_max_element(const orc_ns* s, const double* m);
/* Main loop of assignment-5/sequential/src/main.c:43-60.  solver: 0 =
 * lexicographic solve (the shipped NS), 1 = red-black solveRB (the composed
 * RB-NS oracle), 2 = that solveRB on 16 threads (orc_solve_rb_mt:
 * p bit-identical, the residual summed in another order).  Runs until t > te or max_steps steps (max_steps
 * < 0: unlimited).  iters[k] = pressure iterations of step k (if iters and
 * k < cap).  Returns the number of steps; *t_out = final t. */
int orc_ns_run(orc_ns* s, int solver, int max_steps, int* iters, int cap,
               double* t_out);

#ifdef __cplusplus
}
#endif
/* multi-core solveRB (oracle_mt.c): the bench's multi-core CPU baseline; p
 * bit-identical to orc_solve_rb, residual summed per thread band */
int orc_solve_rb_mt(int imax, int jmax, double dx, double dy, double omega, double eps,
                    int itermax, double* p, const double* rhs, double* res_out, int nthreads);

#endif
