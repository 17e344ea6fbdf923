/*
 * solver_ns.c -- assignment-5/sequential/src/solver.c's entry points as
 * wrappers over libmisor.  Semantics are the sequential solver's (SURVEY 8a
 * notes): dt from max|u|,|v| over all cells incl. ghosts, normalizePressure
 * over all cells, dcavity lid for i < imax, canal parabolic inflow.  The
 * pressure solve is red-black SOR (solveRB); `solve` maps to it unless
 * MISOR_SOLVER=lex selects the reference's lexicographic solve.
 * Decomposed runs (host/ranks.h): each rank owns a block of the 2D
 * decomposition; writeResult first assembles p, u, v on rank 0 (collectResult,
 * assignment-5/skeleton/src/solver.c:320-359) and only rank 0 writes.
 */
#include "solver_ns.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ranks.h"
#include "util.h"

void initSolver(Solver* solver, Parameter* params)
{
    memset(solver, 0, sizeof *solver);
    solver->problem = params->name;
    solver->bcLeft = params->bcLeft;
    solver->bcRight = params->bcRight;
    solver->bcBottom = params->bcBottom;
    solver->bcTop = params->bcTop;
    solver->imax = params->imax;
    solver->jmax = params->jmax;
    solver->xlength = params->xlength;
    solver->ylength = params->ylength;
    solver->dx = params->xlength / params->imax;
    solver->dy = params->ylength / params->jmax;
    solver->eps = params->eps;
    solver->omega = params->omg;
    solver->itermax = params->itermax;
    solver->re = params->re;
    solver->gx = params->gx;
    solver->gy = params->gy;
    solver->dt = params->dt;
    solver->te = params->te;
    solver->tau = params->tau;
    solver->gamma = params->gamma;

    double dx = solver->dx, dy = solver->dy;
    double invSqrSum = 1.0 / (dx * dx) + 1.0 / (dy * dy); /* solver.c:113-116 */
    solver->dtBound = 0.5 * solver->re * 1.0 / invSqrSum;

    misor_desc d = { 0 };
    d.imax = solver->imax;
    d.jmax = solver->jmax;
    d.dx = dx;
    d.dy = dy;
    d.omega = solver->omega;
    d.eps = solver->eps;
    d.itermax = solver->itermax;
    d.variant = MISOR_SOLVE_RB;
    const RankCtx* rk = currentRank();
    d.device = rk->device;
    d.nranks = rk->size;
    d.rank = rk->rank;
    d.comm_id = rk->comm_id;
    solver->rank = rk->rank;
    solver->size = rk->size;
    misorCheck(misor_create(&solver->dev, &d), "misor_create");

    misor_ns_desc n = { 0 };
    n.xlength = solver->xlength;
    n.ylength = solver->ylength;
    n.re = solver->re;
    n.gx = solver->gx;
    n.gy = solver->gy;
    n.gamma = solver->gamma;
    n.tau = solver->tau;
    n.bcLeft = solver->bcLeft;
    n.bcRight = solver->bcRight;
    n.bcBottom = solver->bcBottom;
    n.bcTop = solver->bcTop;
    n.problem = MISOR_PROBLEM_NONE;
    if (solver->problem && strcmp(solver->problem, "dcavity") == 0)
        n.problem = MISOR_PROBLEM_DCAVITY;
    else if (solver->problem && strcmp(solver->problem, "canal") == 0)
        n.problem = MISOR_PROBLEM_CANAL;
    misorCheck(misor_ns_setup(solver->dev, &n), "misor_ns_setup");

    /* solver.c:92-99: u, v, p = init values everywhere, rhs/f/g = 0 */
    misorCheck(misor_fill(solver->dev, MISOR_U, params->u_init), "misor_fill");
    misorCheck(misor_fill(solver->dev, MISOR_V, params->v_init), "misor_fill");
    misorCheck(misor_fill(solver->dev, MISOR_P, params->p_init), "misor_fill");
    misorCheck(misor_set_dt(solver->dev, solver->dt), "misor_set_dt");
}

void computeTimestep(Solver* solver)
{
    misorCheck(misor_compute_timestep(solver->dev, solver->dtBound, solver->tau, &solver->dt),
               "misor_compute_timestep");
}

void setBoundaryConditions(Solver* solver)
{
    misorCheck(misor_set_boundary_conditions(solver->dev), "misor_set_boundary_conditions");
}

void setSpecialBoundaryCondition(Solver* solver)
{
    misorCheck(misor_set_special_boundary_condition(solver->dev),
               "misor_set_special_boundary_condition");
}

void computeFG(Solver* solver)
{
    misorCheck(misor_set_dt(solver->dev, solver->dt), "misor_set_dt");
    misorCheck(misor_compute_fg(solver->dev), "misor_compute_fg");
}

void computeRHS(Solver* solver)
{
    misorCheck(misor_set_dt(solver->dev, solver->dt), "misor_set_dt");
    misorCheck(misor_compute_rhs(solver->dev), "misor_compute_rhs");
}

void normalizePressure(Solver* solver)
{
    misorCheck(misor_normalize_pressure(solver->dev), "misor_normalize_pressure");
}

void solveRB(Solver* solver)
{
    int it = 0;
    double res = 0.0;
    misorCheck(misor_solve_rb(solver->dev, &it, &res), "misor_solve_rb");
    solver->lastIterations = it;
#ifdef VERBOSE
    if (solver->rank == 0) printf("Solver took %d iterations to reach %f\n", it, sqrt(res));
#endif
}

/* red-black by default; MISOR_SOLVER=lex: the reference's own lexicographic
 * solve (assignment-5/sequential/src/solver.c:140-191), bit for bit */
void solve(Solver* solver)
{
    const char* s = getenv("MISOR_SOLVER");
    if (!(s && strcmp(s, "lex") == 0)) {
        solveRB(solver);
        return;
    }
    int it = 0;
    double res = 0.0;
    misorCheck(misor_solve_lex(solver->dev, MISOR_LEX_SEQ, &it, &res), "misor_solve_lex");
    solver->lastIterations = it;
#ifdef VERBOSE
    if (solver->rank == 0) printf("Solver took %d iterations to reach %f\n", it, sqrt(res));
#endif
}

void adaptUV(Solver* solver)
{
    misorCheck(misor_set_dt(solver->dev, solver->dt), "misor_set_dt");
    misorCheck(misor_adapt_uv(solver->dev), "misor_adapt_uv");
}

/* solver.c:457-505; collective in a decomposed run (collectResult) */
void writeResult(Solver* solver)
{
    int imax = solver->imax, jmax = solver->jmax;
    double dx = solver->dx, dy = solver->dy;
    size_t n = (size_t)(imax + 2) * (size_t)(jmax + 2);
    const int root = solver->rank == 0;
    if (root && !solver->p) solver->p = allocate(64, n * sizeof(double));
    if (root && !solver->u) solver->u = allocate(64, n * sizeof(double));
    if (root && !solver->v) solver->v = allocate(64, n * sizeof(double));
    misorCheck(misor_gather(solver->dev, MISOR_P, root ? solver->p : NULL), "misor_gather");
    misorCheck(misor_gather(solver->dev, MISOR_U, root ? solver->u : NULL), "misor_gather");
    misorCheck(misor_gather(solver->dev, MISOR_V, root ? solver->v : NULL), "misor_gather");
    if (!root) return;
#define AT(a, i, j) (a)[(size_t)(j) * (size_t)(imax + 2) + (size_t)(i)]
    FILE* fp = fopen("pressure.dat", "w");
    if (fp == NULL) {
        printf("Error!\n");
        exit(EXIT_FAILURE);
    }
    for (int j = 1; j < jmax + 1; j++) {
        double y = (double)(j - 0.5) * dy;
        for (int i = 1; i < imax + 1; i++) {
            double x = (double)(i - 0.5) * dx;
            fprintf(fp, "%.2f %.2f %f\n", x, y, AT(solver->p, i, j));
        }
        fprintf(fp, "\n");
    }
    fclose(fp);

    fp = fopen("velocity.dat", "w");
    if (fp == NULL) {
        printf("Error!\n");
        exit(EXIT_FAILURE);
    }
    for (int j = 1; j < jmax + 1; j++) {
        double y = dy * (j - 0.5);
        for (int i = 1; i < imax + 1; i++) {
            double x = dx * (i - 0.5);
            double vel_u = (AT(solver->u, i, j) + AT(solver->u, i - 1, j)) / 2.0;
            double vel_v = (AT(solver->v, i, j) + AT(solver->v, i, j - 1)) / 2.0;
            double len = sqrt((vel_u * vel_u) + (vel_v * vel_v));
            fprintf(fp, "%.2f %.2f %f %f %f\n", x, y, vel_u, vel_v, len);
        }
    }
    fclose(fp);
#undef AT
}
