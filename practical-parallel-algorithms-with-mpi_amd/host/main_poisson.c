/*
 * main_poisson.c -- the assignment-4 driver (src/main.c:18-41) on libmisor:
 *   exe-poisson <file.par>  ->  prints the parameters, the iteration count,
 *   writes p.dat and prints "Walltime %.2fs".
 */
#include <stdio.h>
#include <stdlib.h>

#include "parameter.h"
#include "solver_poisson.h"
#include "util.h"

int main(int argc, char** argv)
{
    double startTime, endTime;
    Parameter params;
    Solver solver;
    initParameterPoisson(&params);

    if (argc < 2) {
        printf("Usage: %s <configFile>\n", argv[0]);
        exit(EXIT_SUCCESS);
    }
    readParameter(&params, argv[1]);
    printParameterPoisson(&params);

    initSolver(&solver, &params, 2);
    startTime = getTimeStamp();
    solveRB(&solver);
    endTime = getTimeStamp();
    writeResult(&solver, "p.dat");

    printf("Walltime %.2fs\n", endTime - startTime);
    misor_destroy(solver.dev);
    return EXIT_SUCCESS;
}
