/*
 * ref_glue3d.c -- TEST INFRASTRUCTURE: entry points into the reference's own
 * 3D solver (assignment-6/src/{solver,comm,parameter,allocate}.c compiled in
 * place, single-domain branch of comm.c, -DVERBOSE so that solve() reports
 * its iteration count) for tests/test_oracle3d.py and the golden fixtures.
 * Nothing here restates the reference: it only drives it.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "comm.h"      /* assignment-6/src/comm.h      */
#include "parameter.h" /* assignment-6/src/parameter.h */
#include "solver.h"    /* assignment-6/src/solver.h    */

static FILE* cap_file;
static int saved_fd = -1;

static void capture_begin(void)
{
    fflush(stdout);
    cap_file = tmpfile();
    saved_fd = dup(1);
    dup2(fileno(cap_file), 1);
}

static char* capture_end(void)
{
    fflush(stdout);
    dup2(saved_fd, 1);
    close(saved_fd);
    long n = ftell(cap_file);
    if (n < 0) n = 0;
    rewind(cap_file);
    char* buf = (char*)malloc((size_t)n + 1);
    size_t got = fread(buf, 1, (size_t)n, cap_file);
    buf[got] = '\0';
    fclose(cap_file);
    return buf;
}

static size_t cells(const Solver* s)
{
    return (size_t)(s->comm.imaxLocal + 2) * (size_t)(s->comm.jmaxLocal + 2) *
           (size_t)(s->comm.kmaxLocal + 2);
}

/* initSolver exactly as assignment-6/src/main.c:27-40 does it; sizes > 0
 * override the .par, te >= 0 overrides te */
static void setup(Solver* s, Parameter* prm, const char* par, int imax, int jmax, int kmax,
                  double te)
{
    char* argv[1] = { (char*)"ref3d" };
    commInit(&s->comm, 1, argv);
    initParameter(prm);
    prm->name = NULL;
    readParameter(prm, par);
    if (imax > 0) prm->imax = imax;
    if (jmax > 0) prm->jmax = jmax;
    if (kmax > 0) prm->kmax = kmax;
    if (te >= 0.0) prm->te = te;
    commPartition(&s->comm, prm->kmax, prm->jmax, prm->imax);
    capture_begin();
    initSolver(s, prm); /* VERBOSE: prints its configuration */
    free(capture_end());
}

static void release(Solver* s, Parameter* prm)
{
    free(s->u); free(s->v); free(s->w); free(s->p);
    free(s->rhs); free(s->f); free(s->g); free(s->h);
    free(prm->name);
}

static int solve_counted(Solver* s)
{
    capture_begin();
    solve(s);
    char* out = capture_end();
    int it = -1;
    const char* q = strstr(out, "Solver took ");
    if (q) it = atoi(q + strlen("Solver took "));
    free(out);
    return it;
}

/* main loop of assignment-6/src/main.c:45-60.  Returns steps; iters[k] =
 * pressure iterations of step k; the final u, v, w, p (with ghosts) and t. */
int ref3_run(const char* par, int imax, int jmax, int kmax, double te, int max_steps,
             int* iters, int cap, double* p_out, double* u_out, double* v_out, double* w_out,
             double* t_out)
{
    Parameter prm;
    Solver s;
    setup(&s, &prm, par, imax, jmax, kmax, te);
    double t = 0.0;
    int nt = 0;
    while (t <= s.te && (max_steps < 0 || nt < max_steps)) {
        if (s.tau > 0.0) computeTimestep(&s);
        setBoundaryConditions(&s);
        setSpecialBoundaryCondition(&s);
        computeFG(&s);
        computeRHS(&s);
        int it = solve_counted(&s);
        if (iters && nt < cap) iters[nt] = it;
        adaptUV(&s);
        t += s.dt;
        nt++;
    }
    size_t n = cells(&s);
    if (p_out) memcpy(p_out, s.p, n * sizeof(double));
    if (u_out) memcpy(u_out, s.u, n * sizeof(double));
    if (v_out) memcpy(v_out, s.v, n * sizeof(double));
    if (w_out) memcpy(w_out, s.w, n * sizeof(double));
    if (t_out) *t_out = t;
    release(&s, &prm);
    return nt;
}

/* One reference function on a given state.  fields: 8 arrays in the order
 * u, v, w, p, rhs, f, g, h, each (imax+2)(jmax+2)(kmax+2), read and written
 * back.  which: 0 computeTimestep, 1 setBoundaryConditions,
 * 2 setSpecialBoundaryCondition, 3 computeFG, 4 computeRHS, 5 solve,
 * 6 adaptUV, 7 normalizePressure.  *dt is the dt used (in) / after (out).
 * Returns solve's iteration count for which == 5, else 0. */
int ref3_call(const char* par, int imax, int jmax, int kmax, int which, double* dt,
              double** fields)
{
    Parameter prm;
    Solver s;
    setup(&s, &prm, par, imax, jmax, kmax, -1.0);
    double* arr[8] = { s.u, s.v, s.w, s.p, s.rhs, s.f, s.g, s.h };
    size_t n = cells(&s);
    for (int q = 0; q < 8; q++) memcpy(arr[q], fields[q], n * sizeof(double));
    s.dt = *dt;
    int it = 0;
    switch (which) {
    case 0: computeTimestep(&s); break;
    case 1: setBoundaryConditions(&s); break;
    case 2: setSpecialBoundaryCondition(&s); break;
    case 3: computeFG(&s); break;
    case 4: computeRHS(&s); break;
    case 5: it = solve_counted(&s); break;
    case 6: adaptUV(&s); break;
    case 7: normalizePressure(&s); break;
    default: break;
    }
    for (int q = 0; q < 8; q++) memcpy(fields[q], arr[q], n * sizeof(double));
    *dt = s.dt;
    release(&s, &prm);
    return it;
}
