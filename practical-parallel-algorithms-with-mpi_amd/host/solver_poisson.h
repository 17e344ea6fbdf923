/*
 * solver_poisson.h -- drop-in for assignment-4/src/solver.h:11-27.  The
 * Solver struct keeps the reference fields; p/rhs are host mirrors that are
 * filled only for writeResult, the live fields are in HBM behind `dev`.
 */
#ifndef MISOR_HOST_SOLVER_POISSON_H
#define MISOR_HOST_SOLVER_POISSON_H
#include "misor.h"
#include "parameter.h"

typedef struct {
    double dx, dy;
    double ys;
    int imax, jmax;
    int jmaxLocal;
    int rank;
    int size;
    double *p, *rhs;
    double eps, omega;
    int itermax;
    misor_grid* dev; /* device-resident state (added) */
} Solver;

extern void initSolver(Solver*, Parameter*, int problem);
extern void getResult(Solver*);
extern void writeResult(Solver*, char*);
extern void solve(Solver*);
extern void solveRB(Solver*);
extern void solveRBA(Solver*);
/* MISOR_SOLVER=lex: solve() is the reference's lexicographic SOR (added) */
extern int useLexicographic(void);
#endif
