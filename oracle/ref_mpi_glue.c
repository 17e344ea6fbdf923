/*
 * ref_mpi_glue.c -- TEST INFRASTRUCTURE (CPU baseline only; never linked into
 * the product).  A timing driver for the reference's MPI pressure solve,
 * assignment-5/skeleton/src/solver.c:586-661 (`solve`: an exchange of p per
 * iteration through MPI_Neighbor_alltoallw, solver.c:137-165, a
 * lexicographic sweep, and an MPI_Allreduce of the residual, :651), built
 * from the reference's own sources by oracle/Makefile (`make mpi`) with
 * MPICH's mpicc.  The reference's main (skeleton/src/main.c:19-80) runs the
 * whole NS loop; this driver calls its initSolver (solver.c:406-551: the
 * MPI_Dims_create / MPI_Cart_create topology, datatypes, per-rank arrays) and
 * then only `solve`, on assignment-4's problem-2 fields (p = sin(4 pi x) +
 * sin(4 pi y), rhs = sin(2 pi x), assignment-4/src/solver.c:99-123) set on
 * every rank's block, with eps so small that exactly `itermax` sweeps run.
 *
 * The skeleton's sweep is lexicographic and its NS physics is broken
 * (SURVEY.md 0.3); it is timed here only as the north star's communication-
 * pattern baseline: per-iteration halo exchange + residual all-reduce on the
 * host cores.
 *
 *   mpirun -np N ref-skel-solve IMAX JMAX SWEEPS RUNS
 * prints one JSON line on rank 0 (max over ranks of each run's solve time).
 */
#include <math.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parameter.h"
#include "solver.h"

/* sizeOfRank (skeleton/src/solver.c:30-32) restated */
static int block_size(int coord, int n_coords, int n) {
    return n / n_coords + ((n % n_coords > coord) ? 1 : 0);
}

static int cmp_double(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    if (argc != 5) {
        if (rank == 0) fprintf(stderr, "usage: %s IMAX JMAX SWEEPS RUNS\n", argv[0]);
        MPI_Finalize();
        return 1;
    }
    Parameter prm;
    initParameter(&prm);
    prm.imax = atoi(argv[1]);
    prm.jmax = atoi(argv[2]);
    prm.itermax = atoi(argv[3]);
    const int runs = atoi(argv[4]) > 0 ? atoi(argv[4]) : 1;
    prm.xlength = prm.ylength = 1.0;
    prm.eps = 1e-300; /* eps^2 = 0: res >= eps^2 always, itermax sweeps */
    prm.omg = 1.9;
    prm.name = "poisson";
    Solver s;
    initSolver(&s, &prm);

    /* problem-2 fields on this rank's block, global indices (ghosts included) */
    const int ni = s.imaxLocal, nj = s.jmaxLocal;
    int ioff = 0, joff = 0;
    for (int c = 0; c < s.coords[0]; ++c) ioff += block_size(c, s.dims[0], prm.imax);
    for (int c = 0; c < s.coords[1]; ++c) joff += block_size(c, s.dims[1], prm.jmax);
    const double PI = 3.14159265358979323846;
    const double dx = s.dx, dy = s.dy;
    for (int j = 0; j < nj + 2; ++j)
        for (int i = 0; i < ni + 2; ++i) {
            const size_t k = (size_t)j * (ni + 2) + i;
            s.p[k] = sin(2.0 * PI * (ioff + i) * dx * 2.0) + sin(2.0 * PI * (joff + j) * dy * 2.0);
            s.rhs[k] = sin(2.0 * PI * (ioff + i) * dx);
        }

    double* secs = (double*)malloc(sizeof(double) * runs);
    for (int r = 0; r < runs; ++r) {
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        solve(&s);
        const double el = MPI_Wtime() - t0;
        MPI_Reduce(&el, &secs[r], 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    }
    if (rank == 0) {
        qsort(secs, runs, sizeof(double), cmp_double);
        const double lup = (double)prm.imax * prm.jmax * prm.itermax;
        const double best = secs[0], med = runs % 2 ? secs[runs / 2]
                                                    : 0.5 * (secs[runs / 2 - 1] + secs[runs / 2]);
        printf("{\"ranks\": %d, \"dims\": [%d, %d], \"imax\": %d, \"jmax\": %d, \"sweeps\": %d, "
               "\"runs\": %d, \"best_s\": %.6f, \"median_s\": %.6f, \"mlups_best\": %.2f, "
               "\"mlups_median\": %.2f}\n",
               size, s.dims[0], s.dims[1], prm.imax, prm.jmax, prm.itermax, runs, best, med,
               lup / best / 1e6, lup / med / 1e6);
        fflush(stdout);
    }
    free(secs);
    MPI_Finalize();
    return 0;
}
