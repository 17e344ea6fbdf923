/*
 * solver_ns3d.h -- drop-in for assignment-6/src/solver.h (the 3D solver) on
 * libmisor's misor3_* entry points.  The live fields are in HBM behind
 * `dev`; collectResult downloads them once at the end.
 */
#ifndef MISOR_HOST_SOLVER_NS3D_H
#define MISOR_HOST_SOLVER_NS3D_H
#include "misor.h"
#include "parameter.h"

enum BC { NOSLIP = 1, SLIP, OUTFLOW, PERIODIC };

typedef struct {
    int imax, jmax, kmax;
    double xlength, ylength, zlength;
    double dx, dy, dz;
} Grid;

typedef struct {
    Grid grid;
    /* parameters */
    double eps, omega;
    double re, tau, gamma;
    double gx, gy, gz;
    /* time stepping */
    int itermax;
    double dt, te;
    double dtBound;
    char* problem;
    int bcLeft, bcRight, bcBottom, bcTop, bcFront, bcBack;
    misor_grid3* dev;   /* device-resident state (added) */
    int lastIterations; /* iterations of the last pressure solve (added) */
    double lastRes;     /* its final residual (added) */
    int rank, size;     /* this rank of a decomposed run (added; 0 of 1 on one GPU) */
} Solver;

extern void initSolver(Solver*, Parameter*);
extern void computeRHS(Solver*);
extern void solve(Solver*);
extern void normalizePressure(Solver*);
extern void computeTimestep(Solver*);
extern void setBoundaryConditions(Solver*);
extern void setSpecialBoundaryCondition(Solver*);
extern void computeFG(Solver*);
extern void adaptUV(Solver*);
/* commCollectResult (assignment-6/src/comm.c:246-426): interior p and
 * cell-centred u, v, w of the whole domain, imax*jmax*kmax each, i fastest,
 * on rank 0 (collective; the other ranks pass NULLs) */
extern void collectResult(Solver*, double* pg, double* ug, double* vg, double* wg);
extern void freeSolver(Solver*);
#endif
