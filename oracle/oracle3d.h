/*
 * oracle3d.h -- CPU restatement of assignment-6's 3D NS step and red-black
 * pressure solve (assignment-6/src/solver.c), single domain.  TEST
 * INFRASTRUCTURE ONLY (see oracle.h); every function cites its reference
 * lines in oracle3d.c.
 * Layout: (imax+2)(jmax+2)(kmax+2) doubles, A(i,j,k) =
 * a[(k*(jmax+2) + j)*(imax+2) + i].
 */
#ifndef ORACLE3D_H
#define ORACLE3D_H

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC3_NOSLIP = 1, ORC3_SLIP = 2, ORC3_OUTFLOW = 3, ORC3_PERIODIC = 4 };
enum { ORC3_PROBLEM_NONE = 0, ORC3_PROBLEM_DCAVITY = 1, ORC3_PROBLEM_CANAL = 2 };

typedef struct {
    int imax, jmax, kmax;
    double xlength, ylength, zlength;
    double dx, dy, dz;
    double re, gx, gy, gz, dt, te, tau, gamma, eps, omega, dtBound;
    int itermax;
    int bcLeft, bcRight, bcBottom, bcTop, bcFront, bcBack;
    int problem;
    double *p, *rhs, *f, *g, *h, *u, *v, *w;
} orc3;

void orc3_setup(orc3* s); /* dx, dy, dz, dtBound */
void orc3_compute_rhs(orc3* s);
int orc3_solve(orc3* s, double* res_out);
double orc3_max_element(const orc3* s, const double* m);
void orc3_normalize_pressure(orc3* s);
void orc3_compute_timestep(orc3* s);
void orc3_set_bc(orc3* s);
void orc3_set_special_bc(orc3* s);
void orc3_compute_fg(orc3* s);
void orc3_adapt_uvw(orc3* s);
int orc3_run(orc3* s, int max_steps, int* iters, int cap, double* t_out);
void orc3_collect(const orc3* s, double* pg, double* ug, double* vg, double* wg);

#ifdef __cplusplus
}
#endif
#endif
