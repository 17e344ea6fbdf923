/*
 * solver_poisson.c -- assignment-4's solver entry points (src/solver.c) as
 * wrappers over libmisor.  Behaviour kept from the reference:
 *   initSolver  : dx = xlength/imax, dy = ylength/jmax, p/rhs initial fields
 *                 (problem 2: rhs = sin(2 pi x)), solver.c:83-124
 *   solveRB     : red-black SOR until res < eps^2 or itermax, prints "%d "
 *                 (the iteration count), solver.c:179-238
 *   solveRBA    : the omega-outside variant, solver.c:240-299
 *   solve       : red-black SOR by default (the data-parallel production path,
 *                 DESIGN.md); MISOR_SOLVER=lex runs the reference's own
 *                 lexicographic SOR (solver.c:126-177) bit for bit instead
 *                 (single rank: misor_solve_lex)
 *   writeResult : "%f " for every cell incl. ghosts, '\n' per row, solver.c:301-323
 * Decomposed runs (host/ranks.h): every rank owns a block of the 2D
 * decomposition; getResult assembles p on rank 0 (the collectResult of
 * assignment-5/skeleton/src/solver.c:234-359), which alone prints and writes.
 */
#include "solver_poisson.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ranks.h"
#include "util.h"

static void fill_desc(misor_desc* d, const Solver* solver, int variant)
{
    const RankCtx* rk = currentRank();
    d->imax = solver->imax;
    d->jmax = solver->jmax;
    d->dx = solver->dx;
    d->dy = solver->dy;
    d->omega = solver->omega;
    d->eps = solver->eps;
    d->itermax = solver->itermax;
    d->variant = variant;
    d->device = rk->device;
    d->nranks = rk->size;
    d->rank = rk->rank;
    d->comm_id = rk->comm_id;
}

void initSolver(Solver* solver, Parameter* params, int problem)
{
    solver->imax = params->imax;
    solver->jmax = params->jmax;
    solver->dx = params->xlength / params->imax;
    solver->dy = params->ylength / params->jmax;
    solver->eps = params->eps;
    solver->omega = params->omg;
    solver->itermax = params->itermax;
    solver->rank = currentRank()->rank;
    solver->size = currentRank()->size;
    solver->ys = 0.0;
    solver->p = NULL;
    solver->rhs = NULL;

    misor_desc d = { 0 };
    fill_desc(&d, solver, MISOR_SOLVE_RB);
    misorCheck(misor_create(&solver->dev, &d), "misor_create");
    misor_local loc;
    misorCheck(misor_local_info(solver->dev, &loc), "misor_local_info");
    solver->jmaxLocal = loc.nj;
    misorCheck(misor_poisson_init(solver->dev, params->xlength, params->ylength, problem),
               "misor_poisson_init");
}

static void run(Solver* solver, int variant)
{
    int it = 0;
    double res = 0.0;
    (void)variant;
    misorCheck(misor_solve_rb(solver->dev, &it, &res), "misor_solve_rb");
    if (solver->rank == 0) printf("%d ", it);
}

void solveRB(Solver* solver) { run(solver, MISOR_SOLVE_RB); }

int useLexicographic(void)
{
    const char* s = getenv("MISOR_SOLVER");
    return s && strcmp(s, "lex") == 0;
}

void solve(Solver* solver)
{
    if (!useLexicographic()) {
        run(solver, MISOR_SOLVE_RB);
        return;
    }
    int it = 0;
    double res = 0.0;
    misorCheck(misor_solve_lex(solver->dev, MISOR_LEX_A4, &it, &res), "misor_solve_lex");
    if (solver->rank == 0) printf("%d ", it);
}

void solveRBA(Solver* solver)
{
    /* the update form is a property of the device grid: rebuild it as RBA,
     * carrying this rank's current p and rhs over */
    misor_local loc;
    misorCheck(misor_local_info(solver->dev, &loc), "misor_local_info");
    size_t n = (size_t)(loc.ni + 2) * (size_t)(loc.nj + 2);
    double* p = allocate(64, n * sizeof(double));
    double* rhs = allocate(64, n * sizeof(double));
    misorCheck(misor_download(solver->dev, MISOR_P, p), "misor_download");
    misorCheck(misor_download(solver->dev, MISOR_RHS, rhs), "misor_download");
    misor_destroy(solver->dev);
    misor_desc d = { 0 };
    fill_desc(&d, solver, MISOR_SOLVE_RBA);
    misorCheck(misor_create(&solver->dev, &d), "misor_create");
    misorCheck(misor_upload(solver->dev, MISOR_P, p), "misor_upload");
    misorCheck(misor_upload(solver->dev, MISOR_RHS, rhs), "misor_upload");
    free(p);
    free(rhs);
    run(solver, MISOR_SOLVE_RBA);
}

/* collective: rank 0 receives the whole p (assembled from every rank's block) */
void getResult(Solver* solver)
{
    size_t n = (size_t)(solver->imax + 2) * (size_t)(solver->jmax + 2);
    if (solver->rank == 0 && !solver->p) solver->p = allocate(64, n * sizeof(double));
    misorCheck(misor_gather(solver->dev, MISOR_P, solver->rank == 0 ? solver->p : NULL),
               "misor_gather");
}

void writeResult(Solver* solver, char* filename)
{
    int imax = solver->imax;
    int jmax = solver->jmax;
    getResult(solver);
    if (solver->rank != 0) return;
    double* p = solver->p;

    FILE* fp = fopen(filename, "w");
    if (fp == NULL) {
        printf("Error!\n");
        exit(EXIT_FAILURE);
    }
    for (int j = 0; j < jmax + 2; j++) {
        for (int i = 0; i < imax + 2; i++) fprintf(fp, "%f ", p[(size_t)j * (imax + 2) + i]);
        fprintf(fp, "\n");
    }
    fclose(fp);
}
