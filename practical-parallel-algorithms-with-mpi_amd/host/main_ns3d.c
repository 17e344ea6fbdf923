/*
 * main_ns3d.c -- the assignment-6 driver (src/main.c:21-118) on libmisor's 3D
 * path:  exe-ns3d <file.par>  (assignment-6's dcavity.par / canal.par).
 * Same loop (no normalizePressure), same progress bar, same "Solution took
 * %.2fs" line, same <problem>.vtk output (ASCII, as the reference's
 * VtkOptions default; MISOR_VTK_FORMAT=binary selects the BINARY variant).
 * MISOR_ITERLOG=<file> additionally writes one line per time step:
 * "nt t dt iterations".  One GPU: the 3D path is not decomposed.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parameter.h"
#include "progress.h"
#include "solver_ns3d.h"
#include "util.h"
#include "vtk_writer.h"

int main(int argc, char** argv)
{
    double timeStart, timeStop;
    Parameter p;
    Solver s;

    initParameter(&p);
    if (argc != 2) {
        printf("Usage: %s <configFile>\n", argv[0]);
        exit(EXIT_SUCCESS);
    }
    readParameter(&p, argv[1]);
    printParameter3D(&p);
    initSolver(&s, &p);
#ifndef VERBOSE
    initProgress(s.te);
#endif
    const char* logname = getenv("MISOR_ITERLOG");
    FILE* ilog = logname ? fopen(logname, "w") : NULL;

    double tau = s.tau;
    double te = s.te;
    double t = 0.0;
    int nt = 0;

    timeStart = getTimeStamp();
    while (t <= te) {
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
        printf("TIME %f , TIMESTEP %f\n", t, s.dt);
#else
        printProgress(t);
#endif
    }
    timeStop = getTimeStamp();
#ifndef VERBOSE
    stopProgress();
#endif
    printf("Solution took %.2fs\n", timeStop - timeStart);
    if (ilog) fclose(ilog);

    size_t bytesize = (size_t)s.grid.imax * s.grid.jmax * s.grid.kmax * sizeof(double);
    double* pg = allocate(64, bytesize);
    double* ug = allocate(64, bytesize);
    double* vg = allocate(64, bytesize);
    double* wg = allocate(64, bytesize);
    collectResult(&s, pg, ug, vg, wg);

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
    freeSolver(&s);
    return EXIT_SUCCESS;
}
