/*
 * main_poisson.c -- the assignment-4 driver (src/main.c:18-41) on libmisor:
 *   exe-poisson <file.par>  ->  prints the parameters, the iteration count,
 *   writes p.dat and prints "Walltime %.2fs".  MISOR_RANKS=N (or a launcher's
 *   WORLD_SIZE/RANK) runs it decomposed over N ranks (host/ranks.h); rank 0
 *   prints and writes.
 */
#include <stdio.h>
#include <stdlib.h>

#include "parameter.h"
#include "ranks.h"
#include "solver_poisson.h"
#include "util.h"

static int rank_main(const RankCtx* rk, void* arg)
{
    Parameter params = *(Parameter*)arg;
    double startTime, endTime;
    Solver solver;

    initSolver(&solver, &params, 2);
    startTime = getTimeStamp();
    solve(&solver); /* assignment-4/src/main.c:34 */
    endTime = getTimeStamp();
    writeResult(&solver, "p.dat");

    if (rk->rank == 0) printf("Walltime %.2fs\n", endTime - startTime);
    misor_destroy(solver.dev);
    return 0;
}

int main(int argc, char** argv)
{
    Parameter params;
    initParameterPoisson(&params);

    if (argc < 2) {
        printf("Usage: %s <configFile>\n", argv[0]);
        exit(EXIT_SUCCESS);
    }
    readParameter(&params, argv[1]);
    const char* r = getenv("RANK");
    if (!r || atoi(r) == 0) printParameterPoisson(&params);
    fflush(stdout);
    return runRanks(rank_main, &params) ? EXIT_FAILURE : EXIT_SUCCESS;
}
