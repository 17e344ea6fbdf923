/*
 * oracle_mt.c -- multi-core CPU port of solveRB (assignment-4/src/solver.c:
 * 179-238), for the bench's CPU baseline on the GPU box's host cores
 * ("multi-core 2D-decomposed RB SOR ... pthreads with the same
 * decomposition" -- no MPI on the box).
 *
 * TEST/BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it and
 * tests/test_oracle.py checks it against the single-thread restatement; the
 * product never links it.
 *
 * Each thread owns a band of rows (the sizeOfRank rule over threads).  One
 * iteration: red pass over the band, barrier, black pass, barrier, Neumann
 * ghost copy (rows by the first/last band, columns by every band), barrier,
 * then thread 0 sums the per-thread r^2 in thread order.  The red-black
 * ordering makes p identical to the single-thread solve bit for bit; only the
 * residual's summation order differs.
 */
#include <pthread.h>
#include <stdlib.h>

#include "oracle.h"

#define AT(a, i, j) (a)[(size_t)(j) * (size_t)(imax + 2) + (size_t)(i)]

typedef struct {
    int imax, jmax, itermax, nthreads;
    double idx2, idy2, factor, epssq;
    double* p;
    const double* rhs;
    double* part;   /* per-thread r^2 */
    double res;
    int it, stop;
    pthread_barrier_t bar;
} Shared;

typedef struct {
    Shared* s;
    int t, j0, j1;  /* rows j0 .. j1-1 */
} Arg;

static double pass(const Shared* s, int j0, int j1, int colour)
{
    const int imax = s->imax;
    double* p = s->p;
    const double* rhs = s->rhs;
    double acc = 0.0;
    for (int j = j0; j < j1; j++) {
        int i0 = 1 + ((1 + j + colour) & 1);
        for (int i = i0; i < imax + 1; i += 2) {
            double c = AT(p, i, j);
            double r = AT(rhs, i, j) - ((AT(p, i + 1, j) - 2.0 * c + AT(p, i - 1, j)) * s->idx2 +
                                        (AT(p, i, j + 1) - 2.0 * c + AT(p, i, j - 1)) * s->idy2);
            AT(p, i, j) = c - (s->factor * r);
            acc += (r * r);
        }
    }
    return acc;
}

static void* worker(void* v)
{
    Arg* a = (Arg*)v;
    Shared* s = a->s;
    const int imax = s->imax, jmax = s->jmax;
    double* p = s->p;
    for (;;) {
        pthread_barrier_wait(&s->bar);
        if (s->stop) break;
        double acc = pass(s, a->j0, a->j1, 0);
        pthread_barrier_wait(&s->bar);
        acc += pass(s, a->j0, a->j1, 1);
        s->part[a->t] = acc;
        pthread_barrier_wait(&s->bar);
        /* ghost copy, assignment-4/src/solver.c:219-227 */
        if (a->j0 == 1)
            for (int i = 1; i < imax + 1; i++) AT(p, i, 0) = AT(p, i, 1);
        if (a->j1 == jmax + 1)
            for (int i = 1; i < imax + 1; i++) AT(p, i, jmax + 1) = AT(p, i, jmax);
        for (int j = a->j0; j < a->j1; j++) {
            AT(p, 0, j) = AT(p, 1, j);
            AT(p, imax + 1, j) = AT(p, imax, j);
        }
        pthread_barrier_wait(&s->bar);
        if (a->t == 0) {
            double res = 0.0;
            for (int q = 0; q < s->nthreads; q++) res += s->part[q];
            s->res = res / ((double)imax * (double)jmax);
            s->it++;
            s->stop = !((s->res >= s->epssq) && (s->it < s->itermax));
        }
    }
    return NULL;
}

int orc_solve_rb_mt(int imax, int jmax, double dx, double dy, double omega, double eps,
                    int itermax, double* p, const double* rhs, double* res_out, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > jmax) nthreads = jmax;
    Shared s;
    const double dx2 = dx * dx, dy2 = dy * dy;
    s.imax = imax;
    s.jmax = jmax;
    s.itermax = itermax;
    s.nthreads = nthreads;
    s.idx2 = 1.0 / dx2;
    s.idy2 = 1.0 / dy2;
    s.factor = omega * 0.5 * (dx2 * dy2) / (dx2 + dy2);
    s.epssq = eps * eps;
    s.p = p;
    s.rhs = rhs;
    s.part = calloc((size_t)nthreads, sizeof(double));
    s.res = 1.0;
    s.it = 0;
    s.stop = !((s.res >= s.epssq) && (s.it < itermax));
    pthread_barrier_init(&s.bar, NULL, (unsigned)nthreads);
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nthreads);
    Arg* args = malloc(sizeof(Arg) * (size_t)nthreads);
    int j = 1;
    for (int t = 0; t < nthreads; t++) {
        int rows = jmax / nthreads + (jmax % nthreads > t);
        args[t] = (Arg){ &s, t, j, j + rows };
        j += rows;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &args[t]);
    worker(&args[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&s.bar);
    free(th);
    free(args);
    free(s.part);
    if (res_out) *res_out = s.res;
    return s.it;
}
