/*
 * solver_ns3d.c -- assignment-6/src/solver.c's functions as thin wrappers
 * over libmisor's 3D path (include/misor.h, misor3_*).  Every step runs on
 * the GPU; nothing is copied to the host until collectResult.
 */
#include "solver_ns3d.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ranks.h"
#include "util.h"

static int problemId(const char* name)
{
    /* setSpecialBoundaryCondition's strcmp (solver.c:581, 593) */
    if (name && strcmp(name, "dcavity") == 0) return MISOR_PROBLEM_DCAVITY;
    if (name && strcmp(name, "canal") == 0) return MISOR_PROBLEM_CANAL;
    return MISOR_PROBLEM_NONE;
}

/* initSolver, solver.c:75-143 */
void initSolver(Solver* s, Parameter* params)
{
    memset(s, 0, sizeof *s);
    s->problem = params->name;
    s->bcLeft = params->bcLeft;
    s->bcRight = params->bcRight;
    s->bcBottom = params->bcBottom;
    s->bcTop = params->bcTop;
    s->bcFront = params->bcFront;
    s->bcBack = params->bcBack;
    s->grid.imax = params->imax;
    s->grid.jmax = params->jmax;
    s->grid.kmax = params->kmax;
    s->grid.xlength = params->xlength;
    s->grid.ylength = params->ylength;
    s->grid.zlength = params->zlength;
    s->grid.dx = params->xlength / params->imax;
    s->grid.dy = params->ylength / params->jmax;
    s->grid.dz = params->zlength / params->kmax;
    s->eps = params->eps;
    s->omega = params->omg;
    s->itermax = params->itermax;
    s->re = params->re;
    s->gx = params->gx;
    s->gy = params->gy;
    s->gz = params->gz;
    s->dt = params->dt;
    s->te = params->te;
    s->tau = params->tau;
    s->gamma = params->gamma;

    misor3_desc d;
    memset(&d, 0, sizeof d);
    d.imax = s->grid.imax;
    d.jmax = s->grid.jmax;
    d.kmax = s->grid.kmax;
    d.xlength = s->grid.xlength;
    d.ylength = s->grid.ylength;
    d.zlength = s->grid.zlength;
    d.re = s->re;
    d.gamma = s->gamma;
    d.tau = s->tau;
    d.omega = s->omega;
    d.eps = s->eps;
    d.gx = s->gx;
    d.gy = s->gy;
    d.gz = s->gz;
    d.itermax = s->itermax;
    d.bcTop = s->bcTop;
    d.bcBottom = s->bcBottom;
    d.bcLeft = s->bcLeft;
    d.bcRight = s->bcRight;
    d.bcFront = s->bcFront;
    d.bcBack = s->bcBack;
    d.problem = problemId(s->problem);
    /* decomposed runs (host/ranks.h): slabs of planes, one rank per GPU */
    const RankCtx* rk = currentRank();
    d.device = rk->size > 1 ? rk->device : -1;
    d.nranks = rk->size;
    d.rank = rk->rank;
    d.comm_id = rk->comm_id;
    s->rank = rk->rank;
    s->size = rk->size;
    misorCheck(misor3_create(&s->dev, &d), "initSolver");
    misorCheck(misor3_fill(s->dev, MISOR3_U, params->u_init), "initSolver");
    misorCheck(misor3_fill(s->dev, MISOR3_V, params->v_init), "initSolver");
    misorCheck(misor3_fill(s->dev, MISOR3_W, params->w_init), "initSolver");
    misorCheck(misor3_fill(s->dev, MISOR3_P, params->p_init), "initSolver");
    misorCheck(misor3_set_dt(s->dev, s->dt), "initSolver");

    const double dx = s->grid.dx, dy = s->grid.dy, dz = s->grid.dz;
    double invSqrSum = 1.0 / (dx * dx) + 1.0 / (dy * dy) + 1.0 / (dz * dz);
    s->dtBound = 0.5 * s->re * 1.0 / invSqrSum;
}

void computeRHS(Solver* s) { misorCheck(misor3_compute_rhs(s->dev), "computeRHS"); }

void solve(Solver* s)
{
    misorCheck(misor3_solve(s->dev, &s->lastIterations, &s->lastRes), "solve");
#ifdef VERBOSE
    if (s->rank == 0)
        printf("Solver took %d iterations to reach %f\n", s->lastIterations, sqrt(s->lastRes));
#endif
}

void normalizePressure(Solver* s)
{
    misorCheck(misor3_normalize_pressure(s->dev), "normalizePressure");
}

void computeTimestep(Solver* s)
{
    misorCheck(misor3_compute_timestep(s->dev, &s->dt), "computeTimestep");
}

void setBoundaryConditions(Solver* s)
{
    misorCheck(misor3_set_boundary_conditions(s->dev), "setBoundaryConditions");
}

void setSpecialBoundaryCondition(Solver* s)
{
    misorCheck(misor3_set_special_boundary_condition(s->dev), "setSpecialBoundaryCondition");
}

void computeFG(Solver* s) { misorCheck(misor3_compute_fg(s->dev), "computeFG"); }

void adaptUV(Solver* s) { misorCheck(misor3_adapt_uvw(s->dev), "adaptUV"); }

void collectResult(Solver* s, double* pg, double* ug, double* vg, double* wg)
{
    const int imax = s->grid.imax, jmax = s->grid.jmax, kmax = s->grid.kmax;
    const int root = s->rank == 0;
    const size_t n = (size_t)(imax + 2) * (jmax + 2) * (kmax + 2);
    double *p = NULL, *u = NULL, *v = NULL, *w = NULL;
    if (root) {
        p = allocate(64, n * sizeof(double));
        u = allocate(64, n * sizeof(double));
        v = allocate(64, n * sizeof(double));
        w = allocate(64, n * sizeof(double));
    }
    misorCheck(misor3_gather(s->dev, MISOR3_P, p), "collectResult");
    misorCheck(misor3_gather(s->dev, MISOR3_U, u), "collectResult");
    misorCheck(misor3_gather(s->dev, MISOR3_V, v), "collectResult");
    misorCheck(misor3_gather(s->dev, MISOR3_W, w), "collectResult");
    if (!root) return;
#define L(a, i, j, k) (a)[((size_t)(k) * (jmax + 2) + (size_t)(j)) * (imax + 2) + (size_t)(i)]
    size_t q = 0;
    for (int k = 1; k <= kmax; k++)
        for (int j = 1; j <= jmax; j++)
            for (int i = 1; i <= imax; i++, q++) {
                pg[q] = L(p, i, j, k);
                ug[q] = (L(u, i, j, k) + L(u, i - 1, j, k)) / 2.0;
                vg[q] = (L(v, i, j, k) + L(v, i, j - 1, k)) / 2.0;
                wg[q] = (L(w, i, j, k) + L(w, i, j, k - 1)) / 2.0;
            }
#undef L
    free(p);
    free(u);
    free(v);
    free(w);
}

void freeSolver(Solver* s)
{
    misor3_destroy(s->dev);
    s->dev = NULL;
}
