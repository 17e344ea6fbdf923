/*
 * main_ns.c -- the assignment-5/sequential driver (src/main.c:18-66) on
 * libmisor:  exe-ns <file.par>  (dcavity.par / canal.par of assignment-5 or
 * assignment-6, the latter read as 2D).  Same loop, same progress bar, same
 * "Solution took %.2fs" line, same pressure.dat / velocity.dat.
 * MISOR_ITERLOG=<file> additionally writes one line per time step:
 * "nt t dt iterations".
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parameter.h"
#include "solver_ns.h"
#include "util.h"

static double progEnd;
static int progCur;

static void initProgress(double end)
{
    progEnd = end;
    progCur = 0;
    printf("[          ]");
    fflush(stdout);
}

static void printProgress(double current)
{
    int now = (int)rint((current / progEnd) * 10.0);
    if (now > progCur) {
        char bar[11];
        progCur = now;
        for (int i = 0; i < 10; i++) bar[i] = (i < progCur) ? '#' : ' ';
        bar[10] = '\0';
        printf("\r[%s]", bar);
    }
    fflush(stdout);
}

int main(int argc, char** argv)
{
    double startTime, stopTime;
    Parameter params;
    Solver solver;
    initParameter(&params);

    if (argc != 2) {
        printf("Usage: %s <configFile>\n", argv[0]);
        exit(EXIT_SUCCESS);
    }
    readParameter(&params, argv[1]);
    printParameter(&params);
    initSolver(&solver, &params);
#ifndef VERBOSE
    initProgress(solver.te);
#endif
    const char* logname = getenv("MISOR_ITERLOG");
    FILE* ilog = logname ? fopen(logname, "w") : NULL;

    double tau = solver.tau;
    double te = solver.te;
    double t = 0.0;
    int nt = 0;

    startTime = getTimeStamp();
    while (t <= te) {
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
        printf("TIME %f , TIMESTEP %f\n", t, solver.dt);
#else
        printProgress(t);
#endif
    }
    stopTime = getTimeStamp();
    printf("\n");
    printf("Solution took %.2fs\n", stopTime - startTime);
    writeResult(&solver);
    if (ilog) fclose(ilog);
    misor_destroy(solver.dev);
    return EXIT_SUCCESS;
}
