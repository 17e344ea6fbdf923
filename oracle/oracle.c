/*
 * oracle.c -- CPU restatement of the reference algorithm (TEST INFRASTRUCTURE).
 *
 * Parity status: PINNED.  tests/test_oracle.py checks every function here
 * bit-for-bit against oracle/_ref (the reference sources compiled from
 * /root/reference by oracle/Makefile, same flags) and against the committed
 * fixtures in tests/golden/ (assignment-4/p.dat and init.dat from the
 * reference itself; RB vectors generated from oracle/_ref).
 *
 * Only tests/, bench.py (cpu_baseline) and __graft_entry__.smoke() may use
 * this file, and only as the checker.  Build: -O2 -std=c99 -ffp-contract=off.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stddef.h>
#include <stdlib.h>

#define ORC_PI 3.14159265358979323846 /* assignment-4/src/solver.c:15 */

#define AT(a, i, j) (a)[(size_t)(j) * (size_t)(imax + 2) + (size_t)(i)]

/* assignment-4/src/solver.c:83-124 (initSolver, problem selects rhs) */
void orc_poisson_init(int imax, int jmax, double xlength, double ylength,
                      int problem, double* p, double* rhs)
{
    double dx = xlength / imax;
    double dy = ylength / jmax;
    for (int j = 0; j < jmax + 2; j++)
        for (int i = 0; i < imax + 2; i++)
            AT(p, i, j) = sin(2.0 * ORC_PI * i * dx * 2.0) +
                          sin(2.0 * ORC_PI * j * dy * 2.0);
    for (int j = 0; j < jmax + 2; j++)
        for (int i = 0; i < imax + 2; i++)
            AT(rhs, i, j) = (problem == 2) ? sin(2.0 * ORC_PI * i * dx) : 0.0;
}

/* Neumann ghost copy after a full sweep: rows first, then columns, corners
 * untouched.  assignment-4/src/solver.c:219-227 (and :158-166). */
static void ghost_copy(int imax, int jmax, double* p)
{
    for (int i = 1; i < imax + 1; i++) {
        AT(p, i, 0)        = AT(p, i, 1);
        AT(p, i, jmax + 1) = AT(p, i, jmax);
    }
    for (int j = 1; j < jmax + 1; j++) {
        AT(p, 0, j)        = AT(p, 1, j);
        AT(p, imax + 1, j) = AT(p, imax, j);
    }
}

/* Shared body of solveRB / solveRBA.  `aform` selects the solveRBA update
 * P -= (omega*factor)*r with factor excluding omega
 * (assignment-4/src/solver.c:250,273) instead of P -= factor*r with
 * factor = omega*0.5*dx2*dy2/(dx2+dy2) (:189,:211). */
static int rb_core(int imax, int jmax, double dx, double dy, double omega,
                   double eps, int itermax, double* p, const double* rhs,
                   double* res_out, int aform)
{
    double dx2    = dx * dx;
    double dy2    = dy * dy;
    double idx2   = 1.0 / dx2;
    double idy2   = 1.0 / dy2;
    double factor = aform ? 0.5 * (dx2 * dy2) / (dx2 + dy2)
                          : omega * 0.5 * (dx2 * dy2) / (dx2 + dy2);
    double epssq  = eps * eps;
    double res    = 1.0;
    int it        = 0;

    /* assignment-4/src/solver.c:197-234 */
    while ((res >= epssq) && (it < itermax)) {
        res = 0.0;
        for (int colour = 0; colour < 2; colour++) {
            for (int j = 1; j < jmax + 1; j++) {
                /* pass 0 starts at i=1 on j=1 -> (i+j) even is pass 0 */
                int i0 = 1 + ((1 + j + colour) & 1);
                for (int i = i0; i < imax + 1; i += 2) {
                    double c = AT(p, i, j);
                    double r = AT(rhs, i, j) -
                               ((AT(p, i + 1, j) - 2.0 * c + AT(p, i - 1, j)) * idx2 +
                                (AT(p, i, j + 1) - 2.0 * c + AT(p, i, j - 1)) * idy2);
                    if (aform)
                        AT(p, i, j) = c - (omega * factor * r);
                    else
                        AT(p, i, j) = c - (factor * r);
                    res += (r * r);
                }
            }
        }
        ghost_copy(imax, jmax, p);
        res = res / ((double)imax * (double)jmax);
        it++;
    }
    if (res_out) *res_out = res;
    return it;
}

/* assignment-4/src/solver.c:179-238 */
int orc_solve_rb(int imax, int jmax, double dx, double dy, double omega,
                 double eps, int itermax, double* p, const double* rhs,
                 double* res_out)
{
    return rb_core(imax, jmax, dx, dy, omega, eps, itermax, p, rhs, res_out, 0);
}

/* assignment-4/src/solver.c:240-299 */
int orc_solve_rba(int imax, int jmax, double dx, double dy, double omega,
                  double eps, int itermax, double* p, const double* rhs,
                  double* res_out)
{
    return rb_core(imax, jmax, dx, dy, omega, eps, itermax, p, rhs, res_out, 1);
}

/* assignment-4/src/solver.c:126-177 (xorder 0) and
 * assignment-5/sequential/src/solver.c:140-191 (xorder 1). */
int orc_solve_lex(int imax, int jmax, double dx, double dy, double omega,
                  double eps, int itermax, int xorder, double* p,
                  const double* rhs, double* res_out)
{
    double dx2    = dx * dx;
    double dy2    = dy * dy;
    double idx2   = 1.0 / dx2;
    double idy2   = 1.0 / dy2;
    double factor = omega * 0.5 * (dx2 * dy2) / (dx2 + dy2);
    double epssq  = eps * eps;
    double res    = 1.0;
    int it        = 0;

    while ((res >= epssq) && (it < itermax)) {
        res = 0.0;
        for (int j = 1; j < jmax + 1; j++) {
            for (int i = 1; i < imax + 1; i++) {
                double c = AT(p, i, j);
                double xt = xorder ? (AT(p, i + 1, j) - 2.0 * c + AT(p, i - 1, j))
                                   : (AT(p, i - 1, j) - 2.0 * c + AT(p, i + 1, j));
                double r = AT(rhs, i, j) -
                           (xt * idx2 + (AT(p, i, j - 1 + 2 * xorder) - 2.0 * c +
                                         AT(p, i, j + 1 - 2 * xorder)) * idy2);
                AT(p, i, j) = c - (factor * r);
                res += (r * r);
            }
        }
        ghost_copy(imax, jmax, p);
        res = res / ((double)imax * (double)jmax);
        it++;
    }
    if (res_out) *res_out = res;
    return it;
}

/* One colour of solveRB's inner loop (assignment-4/src/solver.c:204-215)
 * on a decomposed block, colour taken from GLOBAL (i+j) parity. */
double orc_rb_pass_block(int ni, int nj, int ioff, int joff, int colour,
                         double idx2, double idy2, double factor, double* p,
                         const double* rhs)
{
    int imax   = ni; /* for AT() */
    double res = 0.0;
    for (int j = 1; j < nj + 1; j++) {
        int i0 = 1 + ((ioff + 1 + joff + j + colour) & 1);
        for (int i = i0; i < ni + 1; i += 2) {
            double c = AT(p, i, j);
            double r = AT(rhs, i, j) -
                       ((AT(p, i + 1, j) - 2.0 * c + AT(p, i - 1, j)) * idx2 +
                        (AT(p, i, j + 1) - 2.0 * c + AT(p, i, j - 1)) * idy2);
            AT(p, i, j) = c - (factor * r);
            res += (r * r);
        }
    }
    return res;
}

/* ------------------------------------------------------------------------ */
/* 2D Navier-Stokes, assignment-5/sequential/src/solver.c                    */
/* ------------------------------------------------------------------------ */

/* initSolver's derived quantities, assignment-5/sequential/src/solver.c:69-70,113-116 */
void orc_ns_setup(orc_ns* s)
{
    s->dx = s->xlength / s->imax;
    s->dy = s->ylength / s->jmax;
    double invSqrSum = 1.0 / (s->dx * s->dx) + 1.0 / (s->dy * s->dy);
    s->dtBound = 0.5 * s->re * 1.0 / invSqrSum;
}

/* :193-202 -- max |m| over ALL cells incl. ghosts, seeded with DBL_MIN */
double orc_ns_max_element(const orc_ns* s, const double* m)
{
    size_t n = (size_t)(s->imax + 2) * (size_t)(s->jmax + 2);
    double mx = DBL_MIN;
    for (size_t k = 0; k < n; k++) {
        double a = fabs(m[k]);
        mx = (mx > a) ? mx : a;
    }
    return mx;
}

/* :219-234 */
void orc_ns_compute_timestep(orc_ns* s)
{
    double dt   = s->dtBound;
    double umax = orc_ns_max_element(s, s->u);
    double vmax = orc_ns_max_element(s, s->v);
    if (umax > 0) dt = (dt > s->dx / umax) ? s->dx / umax : dt;
    if (vmax > 0) dt = (dt > s->dy / vmax) ? s->dy / vmax : dt;
    s->dt = dt * s->tau;
}

/* :236-337 */
void orc_ns_set_bc(orc_ns* s)
{
    int imax = s->imax, jmax = s->jmax;
    double *u = s->u, *v = s->v;

    switch (s->bcLeft) {
    case ORC_NOSLIP:
        for (int j = 1; j < jmax + 1; j++) { AT(u, 0, j) = 0.0; AT(v, 0, j) = -AT(v, 1, j); }
        break;
    case ORC_SLIP:
        for (int j = 1; j < jmax + 1; j++) { AT(u, 0, j) = 0.0; AT(v, 0, j) = AT(v, 1, j); }
        break;
    case ORC_OUTFLOW:
        for (int j = 1; j < jmax + 1; j++) { AT(u, 0, j) = AT(u, 1, j); AT(v, 0, j) = AT(v, 1, j); }
        break;
    default: break;
    }
    switch (s->bcRight) {
    case ORC_NOSLIP:
        for (int j = 1; j < jmax + 1; j++) { AT(u, imax, j) = 0.0; AT(v, imax + 1, j) = -AT(v, imax, j); }
        break;
    case ORC_SLIP:
        for (int j = 1; j < jmax + 1; j++) { AT(u, imax, j) = 0.0; AT(v, imax + 1, j) = AT(v, imax, j); }
        break;
    case ORC_OUTFLOW:
        for (int j = 1; j < jmax + 1; j++) { AT(u, imax, j) = AT(u, imax - 1, j); AT(v, imax + 1, j) = AT(v, imax, j); }
        break;
    default: break;
    }
    switch (s->bcBottom) {
    case ORC_NOSLIP:
        for (int i = 1; i < imax + 1; i++) { AT(v, i, 0) = 0.0; AT(u, i, 0) = -AT(u, i, 1); }
        break;
    case ORC_SLIP:
        for (int i = 1; i < imax + 1; i++) { AT(v, i, 0) = 0.0; AT(u, i, 0) = AT(u, i, 1); }
        break;
    case ORC_OUTFLOW:
        for (int i = 1; i < imax + 1; i++) { AT(u, i, 0) = AT(u, i, 1); AT(v, i, 0) = AT(v, i, 1); }
        break;
    default: break;
    }
    switch (s->bcTop) {
    case ORC_NOSLIP:
        for (int i = 1; i < imax + 1; i++) { AT(v, i, jmax) = 0.0; AT(u, i, jmax + 1) = -AT(u, i, jmax); }
        break;
    case ORC_SLIP:
        for (int i = 1; i < imax + 1; i++) { AT(v, i, jmax) = 0.0; AT(u, i, jmax + 1) = AT(u, i, jmax); }
        break;
    case ORC_OUTFLOW:
        for (int i = 1; i < imax + 1; i++) { AT(u, i, jmax + 1) = AT(u, i, jmax); AT(v, i, jmax) = AT(v, i, jmax - 1); }
        break;
    default: break;
    }
}

/* :339-358 */
void orc_ns_set_special_bc(orc_ns* s)
{
    int imax = s->imax, jmax = s->jmax;
    double* u = s->u;
    if (s->problem == ORC_PROBLEM_DCAVITY) {
        for (int i = 1; i < imax; i++) AT(u, i, jmax + 1) = 2.0 - AT(u, i, jmax);
    } else if (s->problem == ORC_PROBLEM_CANAL) {
        double ylength = s->ylength;
        for (int j = 1; j < jmax + 1; j++) {
            double y = s->dy * (j - 0.5);
            AT(u, 0, j) = y * (ylength - y) * 4.0 / (ylength * ylength);
        }
    }
}

/* :360-436 */
void orc_ns_compute_fg(orc_ns* s)
{
    int imax = s->imax, jmax = s->jmax;
    const double *u = s->u, *v = s->v;
    double *f = s->f, *g = s->g;
    double gx = s->gx, gy = s->gy, gamma = s->gamma, dt = s->dt;
    double inverseRe = 1.0 / s->re;
    double inverseDx = 1.0 / s->dx;
    double inverseDy = 1.0 / s->dy;

    for (int j = 1; j < jmax + 1; j++) {
        for (int i = 1; i < imax + 1; i++) {
            double uc = AT(u, i, j), ue = AT(u, i + 1, j), uw = AT(u, i - 1, j);
            double un = AT(u, i, j + 1), us = AT(u, i, j - 1), unw = AT(u, i - 1, j + 1);
            double vc = AT(v, i, j), ve = AT(v, i + 1, j), vw = AT(v, i - 1, j);
            double vn = AT(v, i, j + 1), vs = AT(v, i, j - 1), vse = AT(v, i + 1, j - 1);

            double du2dx = inverseDx * 0.25 * ((uc + ue) * (uc + ue) - (uc + uw) * (uc + uw)) +
                           gamma * inverseDx * 0.25 *
                               (fabs(uc + ue) * (uc - ue) + fabs(uc + uw) * (uc - uw));
            double duvdy = inverseDy * 0.25 * ((vc + ve) * (uc + un) - (vs + vse) * (uc + us)) +
                           gamma * inverseDy * 0.25 *
                               (fabs(vc + ve) * (uc - un) + fabs(vs + vse) * (uc - us));
            double du2dx2 = inverseDx * inverseDx * (ue - 2.0 * uc + uw);
            double du2dy2 = inverseDy * inverseDy * (un - 2.0 * uc + us);
            AT(f, i, j) = uc + dt * (inverseRe * (du2dx2 + du2dy2) - du2dx - duvdy + gx);

            double duvdx = inverseDx * 0.25 * ((uc + un) * (vc + ve) - (uw + unw) * (vc + vw)) +
                           gamma * inverseDx * 0.25 *
                               (fabs(uc + un) * (vc - ve) + fabs(uw + unw) * (vc - vw));
            double dv2dy = inverseDy * 0.25 * ((vc + vn) * (vc + vn) - (vc + vs) * (vc + vs)) +
                           gamma * inverseDy * 0.25 *
                               (fabs(vc + vn) * (vc - vn) + fabs(vc + vs) * (vc - vs));
            double dv2dx2 = inverseDx * inverseDx * (ve - 2.0 * vc + vw);
            double dv2dy2 = inverseDy * inverseDy * (vn - 2.0 * vc + vs);
            AT(g, i, j) = vc + dt * (inverseRe * (dv2dx2 + dv2dy2) - duvdx - dv2dy + gy);
        }
    }
    for (int j = 1; j < jmax + 1; j++) {
        AT(f, 0, j)    = AT(u, 0, j);
        AT(f, imax, j) = AT(u, imax, j);
    }
    for (int i = 1; i < imax + 1; i++) {
        AT(g, i, 0)    = AT(v, i, 0);
        AT(g, i, jmax) = AT(v, i, jmax);
    }
}

/* :122-138 */
void orc_ns_compute_rhs(orc_ns* s)
{
    int imax = s->imax, jmax = s->jmax;
    double idx = 1.0 / s->dx, idy = 1.0 / s->dy, idt = 1.0 / s->dt;
    for (int j = 1; j < jmax + 1; j++)
        for (int i = 1; i < imax + 1; i++)
            AT(s->rhs, i, j) = idt * ((AT(s->f, i, j) - AT(s->f, i - 1, j)) * idx +
                                      (AT(s->g, i, j) - AT(s->g, i, j - 1)) * idy);
}

/* :204-217 -- mean over ALL cells incl. ghosts, sequential sum */
void orc_ns_normalize_pressure(orc_ns* s)
{
    size_t n = (size_t)(s->imax + 2) * (size_t)(s->jmax + 2);
    double avg = 0.0;
    for (size_t k = 0; k < n; k++) avg += s->p[k];
    avg /= (double)n;
    for (size_t k = 0; k < n; k++) s->p[k] = s->p[k] - avg;
}

/* :438-455 */
void orc_ns_adapt_uv(orc_ns* s)
{
    int imax = s->imax, jmax = s->jmax;
    double fx = s->dt / s->dx, fy = s->dt / s->dy;
    for (int j = 1; j < jmax + 1; j++) {
        for (int i = 1; i < imax + 1; i++) {
            AT(s->u, i, j) = AT(s->f, i, j) - (AT(s->p, i + 1, j) - AT(s->p, i, j)) * fx;
            AT(s->v, i, j) = AT(s->g, i, j) - (AT(s->p, i, j + 1) - AT(s->p, i, j)) * fy;
        }
    }
}

/* assignment-5/sequential/src/main.c:37-60 */
int orc_ns_run(orc_ns* s, int solver, int max_steps, int* iters, int cap,
               double* t_out)
{
    double t = 0.0;
    int nt   = 0;
    while (t <= s->te && (max_steps < 0 || nt < max_steps)) {
        if (s->tau > 0.0) orc_ns_compute_timestep(s);
        orc_ns_set_bc(s);
        orc_ns_set_special_bc(s);
        orc_ns_compute_fg(s);
        orc_ns_compute_rhs(s);
        if (nt % 100 == 0) orc_ns_normalize_pressure(s);
        int it;
        if (solver == 1)
            it = orc_solve_rb(s->imax, s->jmax, s->dx, s->dy, s->omega, s->eps,
                              s->itermax, s->p, s->rhs, NULL);
        else if (solver == 2) /* the same solveRB on 16 threads over row bands
                               * (oracle_mt.c: p bit-identical, the residual summed
                               * in another order) -- large grids in the tests */
            it = orc_solve_rb_mt(s->imax, s->jmax, s->dx, s->dy, s->omega, s->eps,
                                 s->itermax, s->p, s->rhs, NULL, 16);
        else
            it = orc_solve_lex(s->imax, s->jmax, s->dx, s->dy, s->omega, s->eps,
                               s->itermax, 1, s->p, s->rhs, NULL);
        if (iters && nt < cap) iters[nt] = it;
        orc_ns_adapt_uv(s);
        t += s->dt;
        nt++;
    }
    if (t_out) *t_out = t;
    return nt;
}

/* Generalised colour pass for the multi-rank CPU model of the GPU algorithm
 * (tests/test_distributed_cpu.py): arrays with row stride `stride`, local
 * cell (li,lj) at p[(lj+org)*stride + li+org]; updates the cells of colour
 * `colour` (GLOBAL parity, global = (ioff+li, joff+lj)) in
 * [ilo..ihi] x [jlo..jhi] and returns sum r^2 over the updated cells that
 * also lie in [oilo..oihi] x [ojlo..ojhi] (the cells the rank owns).
 * Arithmetic as solveRB, assignment-4/src/solver.c:207-212. */
double orc_rb_pass_range(int stride, int org, int ilo, int ihi, int jlo, int jhi,
                         int oilo, int oihi, int ojlo, int ojhi, int ioff, int joff,
                         int colour, double idx2, double idy2, double factor, double* p,
                         const double* rhs)
{
#define RG(a, i, j) (a)[(size_t)((j) + org) * (size_t)stride + (size_t)((i) + org)]
    double res = 0.0;
    for (int j = jlo; j <= jhi; j++) {
        for (int i = ilo; i <= ihi; i++) {
            if (((ioff + i + joff + j) & 1) != colour) continue;
            double c = RG(p, i, j);
            double r = RG(rhs, i, j) -
                       ((RG(p, i + 1, j) - 2.0 * c + RG(p, i - 1, j)) * idx2 +
                        (RG(p, i, j + 1) - 2.0 * c + RG(p, i, j - 1)) * idy2);
            RG(p, i, j) = c - (factor * r);
            if (i >= oilo && i <= oihi && j >= ojlo && j <= ojhi) res += (r * r);
        }
    }
    return res;
#undef RG
}
