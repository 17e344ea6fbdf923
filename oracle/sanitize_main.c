/*
 * sanitize_main.c -- TEST INFRASTRUCTURE: the oracle (oracle.c, oracle3d.c,
 * oracle_mt.c) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (make asan -> _asan/oracle-check; tests/test_sanitize_cpu.py).
 *
 * Runs every restated function on small, ragged grids and checks the results
 * that are known without a second implementation:
 *   * solveRB iteration counts of the reference's KATs
 *     (tests/golden/rb_kat.json: 50^2 686, 64x32 705, 33x75 877, generated
 *     from the reference's own assignment-4/src/solver.c:179-238),
 *   * the multi-threaded restatement bit-identical to the scalar one,
 *   * a few steps of the 2D NS main loop (assignment-5/sequential/src/main.c:43-60)
 *     with both solvers on dcavity and canal, and of the 3D one
 *     (assignment-6/src/main.c), for memory errors and UB only.
 * Exit 0 when every check passes.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "oracle3d.h"

static int fails = 0;
#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                             \
        }                                                                        \
    } while (0)

static double* field(int imax, int jmax, int kmax)
{
    return calloc((size_t)(imax + 2) * (jmax + 2) * (kmax + 2), sizeof(double));
}

static void poisson(void)
{
    const int kat[][3] = { { 50, 50, 686 }, { 64, 32, 705 }, { 33, 75, 877 } };
    for (int k = 0; k < 3; ++k) {
        const int ni = kat[k][0], nj = kat[k][1];
        double *p = field(ni, nj, 0), *rhs = field(ni, nj, 0);
        orc_poisson_init(ni, nj, 1.0, 1.0, 2, p, rhs);
        double res;
        const int it = orc_solve_rb(ni, nj, 1.0 / ni, 1.0 / nj, 1.9, 1e-6, 100000, p, rhs, &res);
        CHECK(it == kat[k][2]);
        free(p);
        free(rhs);
    }
    const int ni = 97, nj = 61;
    const size_t n = (size_t)(ni + 2) * (nj + 2);
    double *p0 = field(ni, nj, 0), *rhs = field(ni, nj, 0);
    double *a = field(ni, nj, 0), *b = field(ni, nj, 0);
    orc_poisson_init(ni, nj, 1.0, 1.0, 2, p0, rhs);
    for (int v = 0; v < 4; ++v) {
        memcpy(a, p0, n * sizeof(double));
        double r1 = 0, r2 = 0;
        if (v == 0) orc_solve_rb(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 9, a, rhs, &r1);
        if (v == 1) orc_solve_rba(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 9, a, rhs, &r1);
        if (v >= 2) orc_solve_lex(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 9, v - 2, a, rhs, &r1);
        if (v == 0) {
            memcpy(b, p0, n * sizeof(double));
            orc_solve_rb_mt(ni, nj, 1.0 / ni, 1.0 / nj, 1.7, 1e-300, 9, b, rhs, &r2, 4);
            CHECK(memcmp(a, b, n * sizeof(double)) == 0);
        }
    }
    /* the block-pass forms of the multi-rank CPU model */
    memcpy(a, p0, n * sizeof(double));
    const double f = 1.7 * 0.5 / (1.0 * ni * ni + 1.0 * nj * nj);
    for (int c = 0; c < 2; ++c) {
        orc_rb_pass_block(ni, nj, 0, 0, c, (double)ni * ni, (double)nj * nj, f, a, rhs);
        orc_rb_pass_range(ni + 2, 0, 1, ni, 1, nj, 1, ni, 1, nj, 0, 0, c, (double)ni * ni,
                          (double)nj * nj, f, a, rhs);
    }
    free(p0);
    free(rhs);
    free(a);
    free(b);
}

static void ns2d(int problem, int solver)
{
    orc_ns s;
    memset(&s, 0, sizeof s);
    s.imax = problem == ORC_PROBLEM_CANAL ? 60 : 33;
    s.jmax = problem == ORC_PROBLEM_CANAL ? 15 : 31;
    s.xlength = problem == ORC_PROBLEM_CANAL ? 30.0 : 1.0;
    s.ylength = problem == ORC_PROBLEM_CANAL ? 4.0 : 1.0;
    s.re = problem == ORC_PROBLEM_CANAL ? 100.0 : 10.0;
    s.dt = 0.02, s.te = 100.0, s.tau = 0.5, s.gamma = 0.9;
    s.eps = 1e-3, s.omega = 1.7, s.itermax = 500;
    if (problem == ORC_PROBLEM_CANAL) {
        s.bcLeft = ORC_NOSLIP, s.bcRight = ORC_OUTFLOW;
    } else {
        s.bcLeft = ORC_NOSLIP, s.bcRight = ORC_NOSLIP;
    }
    s.bcBottom = ORC_NOSLIP, s.bcTop = ORC_NOSLIP;
    s.problem = problem;
    double** fs[] = { &s.p, &s.rhs, &s.f, &s.g, &s.u, &s.v };
    for (int k = 0; k < 6; ++k) *fs[k] = field(s.imax, s.jmax, 0);
    orc_ns_setup(&s);
    int iters[8];
    double t;
    CHECK(orc_ns_run(&s, solver, 8, iters, 8, &t) == 8);
    for (int k = 0; k < 8; ++k) CHECK(iters[k] >= 0 && iters[k] <= s.itermax);
    (void)orc_ns_max_element(&s, s.u);
    for (int k = 0; k < 6; ++k) free(*fs[k]);
}

static void ns3d(int problem)
{
    orc3 s;
    memset(&s, 0, sizeof s);
    s.imax = 13, s.jmax = 9, s.kmax = 11;
    s.xlength = s.ylength = s.zlength = 1.0;
    s.re = 10.0, s.dt = 0.02, s.te = 100.0, s.tau = 0.5, s.gamma = 0.9;
    s.eps = 1e-3, s.omega = 1.7, s.itermax = 300;
    s.bcLeft = s.bcRight = s.bcBottom = s.bcTop = s.bcFront = s.bcBack = ORC_NOSLIP;
    if (problem == ORC_PROBLEM_CANAL) s.bcRight = ORC_OUTFLOW;
    s.problem = problem;
    double** fs[] = { &s.p, &s.rhs, &s.f, &s.g, &s.h, &s.u, &s.v, &s.w };
    for (int k = 0; k < 8; ++k) *fs[k] = field(s.imax, s.jmax, s.kmax);
    orc3_setup(&s);
    int iters[4];
    double t;
    CHECK(orc3_run(&s, 4, iters, 4, &t) == 4);
    orc3_normalize_pressure(&s);
    const size_t n = (size_t)s.imax * s.jmax * s.kmax;
    double *pg = malloc(n * 8), *ug = malloc(n * 8), *vg = malloc(n * 8), *wg = malloc(n * 8);
    orc3_collect(&s, pg, ug, vg, wg);
    free(pg);
    free(ug);
    free(vg);
    free(wg);
    for (int k = 0; k < 8; ++k) free(*fs[k]);
}

int main(void)
{
    poisson();
    for (int solver = 0; solver < 2; ++solver) {
        ns2d(ORC_PROBLEM_DCAVITY, solver);
        ns2d(ORC_PROBLEM_CANAL, solver);
    }
    ns3d(ORC_PROBLEM_DCAVITY);
    ns3d(ORC_PROBLEM_CANAL);
    if (fails) fprintf(stderr, "%d checks failed\n", fails);
    else printf("oracle-check: all checks passed\n");
    return fails ? 1 : 0;
}
