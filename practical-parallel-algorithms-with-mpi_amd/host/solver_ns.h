/*
 * solver_ns.h -- drop-in for assignment-5/sequential/src/solver.h:11-45.
 * Field pointers stay NULL until writeResult downloads them; the live fields
 * are in HBM behind `dev`.
 */
#ifndef MISOR_HOST_SOLVER_NS_H
#define MISOR_HOST_SOLVER_NS_H
#include "misor.h"
#include "parameter.h"

enum BC { NOSLIP = 1, SLIP, OUTFLOW, PERIODIC };

typedef struct {
    /* geometry and grid information */
    double dx, dy;
    int imax, jmax;
    double xlength, ylength;
    /* arrays (host mirrors, filled by writeResult) */
    double *p, *rhs;
    double *f, *g;
    double *u, *v;
    /* parameters */
    double eps, omega;
    double re, tau, gamma;
    double gx, gy;
    /* time stepping */
    int itermax;
    double dt, te;
    double dtBound;
    char* problem;
    int bcLeft, bcRight, bcBottom, bcTop;
    misor_grid* dev; /* device-resident state (added) */
    int lastIterations; /* iterations of the last pressure solve (added) */
    int rank, size;     /* this rank of a decomposed run (added; 0 of 1 on one GPU) */
} Solver;

extern void initSolver(Solver*, Parameter*);
extern void computeRHS(Solver*);
extern void solve(Solver*);
extern void solveRB(Solver*);
extern void normalizePressure(Solver*);
extern void computeTimestep(Solver*);
extern void setBoundaryConditions(Solver*);
extern void setSpecialBoundaryCondition(Solver*);
extern void computeFG(Solver*);
extern void adaptUV(Solver*);
extern void writeResult(Solver*);
#endif
