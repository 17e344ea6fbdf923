/*
 * main_ns3d.c -- the assignment-6 driver (src/main.c:21-118) on libmisor's 3D
 * path:  exe-ns3d <file.par>  (assignment-6's dcavity.par / canal.par).
 * Same loop (no normalizePressure), same progress bar, same "Solution took
 * %.2fs" line, same <problem>.vtk output (ASCII, as the reference's
 * VtkOptions default; MISOR_VTK_FORMAT=binary selects the BINARY variant).
 * MISOR_ITERLOG=<file> additionally writes one line per time step:
 * "nt t dt iterations".  MISOR_RANKS=N (or a launcher's WORLD_SIZE/RANK,
 * host/ranks.h) runs it decomposed into N slabs of planes like the
 * reference's mpirun -np N; rank 0 prints and writes the collected result.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parameter.h"
#include "progress.h"
#include "ranks.h"
#include "solver_ns3d.h"
#include "util.h"
#include "vtk_writer.h"

static int rank_main(const RankCtx* rk, void* arg)
{
    Parameter p = *(Parameter*)arg;
    const int root = rk->rank == 0;
    double timeStart, timeStop;
    Solver s;
    initSolver(&s, &p);
#ifndef VERBOSE
    if (root) initProgress(s.te);
#endif
    const char* logname = getenv("MISOR_ITERLOG");
    FILE* ilog = (root && logname) ? fopen(logname, "w") : NULL;

    double tau = s.tau;
    double te = s.te;
    double t = 0.0;
    int nt = 0;

    timeStart = getTimeStamp();
    while (t <= te) { /* dt is all-reduced: every rank takes the same steps */
        if (tau > 0.0) computeTimestep(&s);
        setBoundaryConditions(&s);
        setSpecialBoundaryCondition(&s);
        computeFG(&s);
        computeRHS(&s);
        solve(&s);
        adaptUV(&s);
        if (ilog) fprintf(ilog, "%d %.17g %.17g %d\n", nt, t, s.dt, s.lastIterations);
        t += s.dt;
        nt++;
#ifdef VERBOSE
        if (root) printf("TIME %f , TIMESTEP %f\n", t, s.dt);
#else
        if (root) printProgress(t);
#endif
    }
    timeStop = getTimeStamp();
    if (root) {
#ifndef VERBOSE
        stopProgress();
#endif
        printf("Solution took %.2fs\n", timeStop - timeStart);
    }
    if (ilog) fclose(ilog);

    double *pg = NULL, *ug = NULL, *vg = NULL, *wg = NULL;
    if (root) {
        size_t bytesize = (size_t)s.grid.imax * s.grid.jmax * s.grid.kmax * sizeof(double);
        pg = allocate(64, bytesize);
        ug = allocate(64, bytesize);
        vg = allocate(64, bytesize);
        wg = allocate(64, bytesize);
    }
    collectResult(&s, pg, ug, vg, wg);
    if (root) {
        const char* fmt = getenv("MISOR_VTK_FORMAT");
        VtkOptions opts = { .grid = s.grid };
        if (fmt && strcmp(fmt, "binary") == 0) opts.fmt = BINARY;
        vtkOpen(&opts, s.problem);
        vtkScalar(&opts, "pressure", pg);
        vtkVector(&opts, "velocity", (VtkVector){ ug, vg, wg });
        vtkClose(&opts);
        free(pg);
        free(ug);
        free(vg);
        free(wg);
    }
    freeSolver(&s);
    return 0;
}

int main(int argc, char** argv)
{
    Parameter p;
    initParameter(&p);
    if (argc != 2) {
        printf("Usage: %s <configFile>\n", argv[0]);
        exit(EXIT_SUCCESS);
    }
    readParameter(&p, argv[1]);
    const char* r = getenv("RANK");
    if (!r || atoi(r) == 0) printParameter3D(&p);
    fflush(stdout);
    return runRanks(rank_main, &p) ? EXIT_FAILURE : EXIT_SUCCESS;
}
