/*
 * main_ns.c -- the assignment-5/sequential driver (src/main.c:18-66) on
 * libmisor:  exe-ns <file.par>  (dcavity.par / canal.par of assignment-5 or
 * assignment-6, the latter read as 2D).  Same loop, same progress bar, same
 * "Solution took %.2fs" line, same pressure.dat / velocity.dat.
 * MISOR_ITERLOG=<file> additionally writes one line per time step:
 * "nt t dt iterations".  MISOR_RANKS=N (or a launcher's WORLD_SIZE/RANK) runs
 * it decomposed over N ranks like the skeleton's mpirun -np N
 * (assignment-5/skeleton/src/main.c:18-66, host/ranks.h); rank 0 prints and
 * writes the assembled result.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parameter.h"
#include "progress.h"
#include "ranks.h"
#include "solver_ns.h"
#include "util.h"

static int rank_main(const RankCtx* rk, void* arg)
{
    Parameter params = *(Parameter*)arg;
    const int root = rk->rank == 0;
    double startTime, stopTime;
    Solver solver;
    initSolver(&solver, &params);
#ifndef VERBOSE
    if (root) initProgress(solver.te);
#endif
    const char* logname = getenv("MISOR_ITERLOG");
    FILE* ilog = (root && logname) ? fopen(logname, "w") : NULL;

    double tau = solver.tau;
    double te = solver.te;
    double t = 0.0;
    int nt = 0;

    startTime = getTimeStamp();
    while (t <= te) { /* dt is all-reduced: every rank takes the same steps */
        if (tau > 0.0) computeTimestep(&solver);
        setBoundaryConditions(&solver);
        setSpecialBoundaryCondition(&solver);
        computeFG(&solver);
        computeRHS(&solver);
        if (nt % 100 == 0) normalizePressure(&solver);
        solve(&solver);
        adaptUV(&solver);
        if (ilog) fprintf(ilog, "%d %.17g %.17g %d\n", nt, t, solver.dt, solver.lastIterations);
        t += solver.dt;
        nt++;
#ifdef VERBOSE
        if (root) printf("TIME %f , TIMESTEP %f\n", t, solver.dt);
#else
        if (root) printProgress(t);
#endif
    }
    stopTime = getTimeStamp();
    if (root) {
        printf("\n");
        printf("Solution took %.2fs\n", stopTime - startTime);
    }
    writeResult(&solver);
    if (ilog) fclose(ilog);
    misor_destroy(solver.dev);
    return 0;
}

int main(int argc, char** argv)
{
    Parameter params;
    initParameter(&params);

    if (argc != 2) {
        printf("Usage: %s <configFile>\n", argv[0]);
        exit(EXIT_SUCCESS);
    }
    readParameter(&params, argv[1]);
    const char* r = getenv("RANK");
    if (!r || atoi(r) == 0) printParameter(&params);
    fflush(stdout);
    return runRanks(rank_main, &params) ? EXIT_FAILURE : EXIT_SUCCESS;
}
