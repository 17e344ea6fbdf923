/*
 * oracle3d.c -- CPU restatement of assignment-6's 3D Navier-Stokes step and
 * its red-black pressure solve (assignment-6/src/solver.c), single domain.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker of the GPU 3D path.
 * Pinned bit for bit against the reference's own sources compiled in this
 * container (oracle/_ref/libref3d.so, oracle/Makefile `ref`) by
 * tests/test_oracle3d.py.
 *
 * Layout: (imax+2)(jmax+2)(kmax+2) doubles, i fastest, then j, then k:
 * A(i,j,k) = a[(k*(jmax+2) + j)*(imax+2) + i]  (solver.c:19-34 with the
 * local sizes of a single domain).  Expression order follows the reference
 * term by term; compiled -O2 -ffp-contract=off.
 */
#include <float.h>
#include <math.h>
#include <string.h>

#include "oracle3d.h"

#define IX(s, i, j, k) ((((size_t)(k) * (size_t)((s)->jmax + 2) + (size_t)(j)) * \
                         (size_t)((s)->imax + 2)) + (size_t)(i))
#define A3(a, i, j, k) (a)[IX(s, i, j, k)]

static size_t ncell(const orc3* s)
{
    return (size_t)(s->imax + 2) * (size_t)(s->jmax + 2) * (size_t)(s->kmax + 2);
}

/* initSolver's derived quantities (solver.c:86-95, 136-139) */
void orc3_setup(orc3* s)
{
    s->dx = s->xlength / s->imax;
    s->dy = s->ylength / s->jmax;
    s->dz = s->zlength / s->kmax;
    double inv = 1.0 / (s->dx * s->dx) + 1.0 / (s->dy * s->dy) + 1.0 / (s->dz * s->dz);
    s->dtBound = 0.5 * s->re * 1.0 / inv;
}

/* computeRHS, solver.c:145-173 */
void orc3_compute_rhs(orc3* s)
{
    const double idx = 1.0 / s->dx, idy = 1.0 / s->dy, idz = 1.0 / s->dz;
    const double idt = 1.0 / s->dt;
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++)
            for (int i = 1; i <= s->imax; i++) {
                double sx = (A3(s->f, i, j, k) - A3(s->f, i - 1, j, k)) * idx;
                double sy = (A3(s->g, i, j, k) - A3(s->g, i, j - 1, k)) * idy;
                double sz = (A3(s->h, i, j, k) - A3(s->h, i, j, k - 1)) * idz;
                A3(s->rhs, i, j, k) = ((sx + sy) + sz) * idt;
            }
}

/* Neumann ghost copy after each iteration, solver.c:237-278 (faces only,
 * interior index ranges; edges and corners are never touched) */
static void ghost_copy3(orc3* s, double* p)
{
    const int I = s->imax, J = s->jmax, K = s->kmax;
    for (int j = 1; j <= J; j++)
        for (int i = 1; i <= I; i++) {
            A3(p, i, j, 0) = A3(p, i, j, 1);
            A3(p, i, j, K + 1) = A3(p, i, j, K);
        }
    for (int k = 1; k <= K; k++)
        for (int i = 1; i <= I; i++) {
            A3(p, i, 0, k) = A3(p, i, 1, k);
            A3(p, i, J + 1, k) = A3(p, i, J, k);
        }
    for (int k = 1; k <= K; k++)
        for (int j = 1; j <= J; j++) {
            A3(p, 0, j, k) = A3(p, 1, j, k);
            A3(p, I + 1, j, k) = A3(p, I, j, k);
        }
}

/* solve, solver.c:175-297.  Red-black by (i+j+k) parity: pass 0 updates the
 * cells with i+j+k odd (the sweep starts at (1,1,1)), pass 1 the even ones.
 * As in the reference, `res` is carried over between iterations (it is set
 * to 1.0 once and never reset): res = (res + sum r^2) / (imax*jmax*kmax). */
int orc3_solve(orc3* s, double* res_out)
{
    const double dx2 = s->dx * s->dx, dy2 = s->dy * s->dy, dz2 = s->dz * s->dz;
    const double idx2 = 1.0 / dx2, idy2 = 1.0 / dy2, idz2 = 1.0 / dz2;
    const double factor = s->omega * 0.5 * (dx2 * dy2 * dz2) / (dy2 * dz2 + dx2 * dz2 + dx2 * dy2);
    const double epssq = s->eps * s->eps;
    double* p = s->p;
    const double* rhs = s->rhs;
    double res = 1.0;
    int it = 0;
    while ((res >= epssq) && (it < s->itermax)) {
        for (int pass = 0; pass < 2; pass++) {
            for (int k = 1; k <= s->kmax; k++)
                for (int j = 1; j <= s->jmax; j++) {
                    /* first i of this row with (i+j+k) odd (pass 0) / even (pass 1) */
                    int i0 = ((1 + j + k + pass) & 1) ? 1 : 2;
                    for (int i = i0; i <= s->imax; i += 2) {
                        double c = A3(p, i, j, k);
                        double tx = (A3(p, i + 1, j, k) - 2.0 * c) + A3(p, i - 1, j, k);
                        double ty = (A3(p, i, j + 1, k) - 2.0 * c) + A3(p, i, j - 1, k);
                        double tz = (A3(p, i, j, k + 1) - 2.0 * c) + A3(p, i, j, k - 1);
                        double r = A3(rhs, i, j, k) - ((tx * idx2 + ty * idy2) + tz * idz2);
                        A3(p, i, j, k) = c - (factor * r);
                        res += (r * r);
                    }
                }
        }
        ghost_copy3(s, p);
        res = res / (double)((long long)s->imax * s->jmax * s->kmax);
        it++;
    }
    if (res_out) *res_out = res;
    return it;
}

/* maxElement, solver.c:299-310: over every cell incl. ghosts, seeded DBL_MIN */
double orc3_max_element(const orc3* s, const double* m)
{
    double mx = DBL_MIN;
    size_t n = ncell(s);
    for (size_t q = 0; q < n; q++) {
        double a = fabs(m[q]);
        mx = (mx > a) ? mx : a;
    }
    return mx;
}

/* normalizePressure, solver.c:312-338 (interior cells only) */
void orc3_normalize_pressure(orc3* s)
{
    double avg = 0.0;
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++)
            for (int i = 1; i <= s->imax; i++) avg += A3(s->p, i, j, k);
    avg /= (s->imax * s->jmax * s->kmax);
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++)
            for (int i = 1; i <= s->imax; i++) A3(s->p, i, j, k) = A3(s->p, i, j, k) - avg;
}

/* computeTimestep, solver.c:340-362 */
void orc3_compute_timestep(orc3* s)
{
    double dt = s->dtBound;
    double um = orc3_max_element(s, s->u);
    double vm = orc3_max_element(s, s->v);
    double wm = orc3_max_element(s, s->w);
    if (um > 0) dt = (dt > s->dx / um) ? s->dx / um : dt;
    if (vm > 0) dt = (dt > s->dy / vm) ? s->dy / vm : dt;
    if (wm > 0) dt = (dt > s->dz / wm) ? s->dz / wm : dt;
    s->dt = dt * s->tau;
}

/* one wall of setBoundaryConditions (solver.c:364-577).  The wall's normal
 * velocity component `n` sits ON the wall (index `on`), the two tangential
 * ones `t1`, `t2` in the ghost layer (index `gh`) mirrored from the first
 * interior layer (index `in`).  NOSLIP: normal 0, tangential negated; SLIP:
 * normal 0, tangential copied; OUTFLOW: everything copied from the inside
 * (the normal one from the layer inside `on`); PERIODIC: nothing. */
typedef struct {
    int axis;   /* 0: x (left/right), 1: y (bottom/top), 2: z (front/back) */
    int gh, in; /* ghost layer, first interior layer */
    int on, onin; /* layer holding the wall-normal component, and the one inside it */
} Wall;

static void apply_wall(orc3* s, Wall w, int bc)
{
    if (bc != ORC3_NOSLIP && bc != ORC3_SLIP && bc != ORC3_OUTFLOW) return;
    double *n, *t1, *t2;
    int na, nb; /* extents of the two in-plane loops */
    if (w.axis == 0) {
        n = s->u; t1 = s->v; t2 = s->w; na = s->jmax; nb = s->kmax;
    } else if (w.axis == 1) {
        n = s->v; t1 = s->u; t2 = s->w; na = s->imax; nb = s->kmax;
    } else {
        n = s->w; t1 = s->u; t2 = s->v; na = s->imax; nb = s->jmax;
    }
    for (int b = 1; b <= nb; b++)
        for (int a = 1; a <= na; a++) {
            size_t g, in, on, onin;
            if (w.axis == 0) {
                g = IX(s, w.gh, a, b); in = IX(s, w.in, a, b);
                on = IX(s, w.on, a, b); onin = IX(s, w.onin, a, b);
            } else if (w.axis == 1) {
                g = IX(s, a, w.gh, b); in = IX(s, a, w.in, b);
                on = IX(s, a, w.on, b); onin = IX(s, a, w.onin, b);
            } else {
                g = IX(s, a, b, w.gh); in = IX(s, a, b, w.in);
                on = IX(s, a, b, w.on); onin = IX(s, a, b, w.onin);
            }
            /* the reference's statement order per wall: x-wall U,V,W;
             * y-wall U,V,W; z-wall U,V,W -- components are independent */
            if (bc == ORC3_NOSLIP) {
                n[on] = 0.0;
                t1[g] = -t1[in];
                t2[g] = -t2[in];
            } else if (bc == ORC3_SLIP) {
                n[on] = 0.0;
                t1[g] = t1[in];
                t2[g] = t2[in];
            } else {
                n[on] = n[onin];
                t1[g] = t1[in];
                t2[g] = t2[in];
            }
        }
}

/* setBoundaryConditions, solver.c:364-577: top, bottom, left, right, front,
 * back.  The normal component of the low walls lives in ghost layer 0
 * (U(0,j,k), V(i,0,k), W(i,j,0)), that of the high walls on the last interior
 * layer (U(imax,j,k), V(i,jmax,k), W(i,j,kmax)). */
void orc3_set_bc(orc3* s)
{
    const int I = s->imax, J = s->jmax, K = s->kmax;
    apply_wall(s, (Wall){ 1, J + 1, J, J, J - 1 }, s->bcTop);
    apply_wall(s, (Wall){ 1, 0, 1, 0, 1 }, s->bcBottom);
    apply_wall(s, (Wall){ 0, 0, 1, 0, 1 }, s->bcLeft);
    apply_wall(s, (Wall){ 0, I + 1, I, I, I - 1 }, s->bcRight);
    apply_wall(s, (Wall){ 2, 0, 1, 0, 1 }, s->bcFront);
    apply_wall(s, (Wall){ 2, K + 1, K, K, K - 1 }, s->bcBack);
}

/* setSpecialBoundaryCondition, solver.c:579-604: dcavity lid for
 * i = 1..imax-1, k = 1..kmax-1; canal inflow U(0,j,k) = 2.0 */
void orc3_set_special_bc(orc3* s)
{
    if (s->problem == ORC3_PROBLEM_DCAVITY) {
        for (int k = 1; k < s->kmax; k++)
            for (int i = 1; i < s->imax; i++)
                A3(s->u, i, s->jmax + 1, k) = 2.0 - A3(s->u, i, s->jmax, k);
    } else if (s->problem == ORC3_PROBLEM_CANAL) {
        for (int k = 1; k <= s->kmax; k++)
            for (int j = 1; j <= s->jmax; j++) A3(s->u, 0, j, k) = 2.0;
    }
}

/* donor-cell / gamma-upwind convective term of computeFG:
 *   ih*0.25*(ap*bp - am*bm) + gamma*ih*0.25*(|ap|*dp + |am|*dm)
 * ap, am: advecting sums at the + and - faces; bp, bm: advected sums;
 * dp, dm: advected differences */
static double conv(double ih, double gamma, double ap, double bp, double dp, double am,
                   double bm, double dm)
{
    return ih * 0.25 * (ap * bp - am * bm) + gamma * ih * 0.25 * (fabs(ap) * dp + fabs(am) * dm);
}

/* ih^2 * ((a+ - 2c) + a-) */
static double diff2(double ih, double ap, double c, double am)
{
    return ih * ih * (ap - 2.0 * c + am);
}

/* computeFG, solver.c:606-824 (incl. the boundary values of F, G, H) */
void orc3_compute_fg(orc3* s)
{
    const double gm = s->gamma, iRe = 1.0 / s->re;
    const double ix = 1.0 / s->dx, iy = 1.0 / s->dy, iz = 1.0 / s->dz;
    const double dt = s->dt;
    const double *u = s->u, *v = s->v, *w = s->w;
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++)
            for (int i = 1; i <= s->imax; i++) {
#define U_(a, b, c) A3(u, a, b, c)
#define V_(a, b, c) A3(v, a, b, c)
#define W_(a, b, c) A3(w, a, b, c)
                const double Uc = U_(i, j, k), Vc = V_(i, j, k), Wc = W_(i, j, k);
                /* F */
                double du2dx = conv(ix, gm, Uc + U_(i + 1, j, k), Uc + U_(i + 1, j, k),
                                    Uc - U_(i + 1, j, k), Uc + U_(i - 1, j, k),
                                    Uc + U_(i - 1, j, k), Uc - U_(i - 1, j, k));
                double duvdy = conv(iy, gm, Vc + V_(i + 1, j, k), Uc + U_(i, j + 1, k),
                                    Uc - U_(i, j + 1, k), V_(i, j - 1, k) + V_(i + 1, j - 1, k),
                                    Uc + U_(i, j - 1, k), Uc - U_(i, j - 1, k));
                double duwdz = conv(iz, gm, Wc + W_(i + 1, j, k), Uc + U_(i, j, k + 1),
                                    Uc - U_(i, j, k + 1), W_(i, j, k - 1) + W_(i + 1, j, k - 1),
                                    Uc + U_(i, j, k - 1), Uc - U_(i, j, k - 1));
                double lu = diff2(ix, U_(i + 1, j, k), Uc, U_(i - 1, j, k)) +
                            diff2(iy, U_(i, j + 1, k), Uc, U_(i, j - 1, k)) +
                            diff2(iz, U_(i, j, k + 1), Uc, U_(i, j, k - 1));
                A3(s->f, i, j, k) = Uc + dt * (iRe * lu - du2dx - duvdy - duwdz + s->gx);
                /* G */
                double duvdx = conv(ix, gm, Uc + U_(i, j + 1, k), Vc + V_(i + 1, j, k),
                                    Vc - V_(i + 1, j, k), U_(i - 1, j, k) + U_(i - 1, j + 1, k),
                                    Vc + V_(i - 1, j, k), Vc - V_(i - 1, j, k));
                double dv2dy = conv(iy, gm, Vc + V_(i, j + 1, k), Vc + V_(i, j + 1, k),
                                    Vc - V_(i, j + 1, k), Vc + V_(i, j - 1, k),
                                    Vc + V_(i, j - 1, k), Vc - V_(i, j - 1, k));
                /* as the reference (solver.c:719-727): the - side reuses V(k+1) */
                double dvwdz = conv(iz, gm, Wc + W_(i, j + 1, k), Vc + V_(i, j, k + 1),
                                    Vc - V_(i, j, k + 1), W_(i, j, k - 1) + W_(i, j + 1, k - 1),
                                    Vc + V_(i, j, k + 1), Vc - V_(i, j, k + 1));
                double lv = diff2(ix, V_(i + 1, j, k), Vc, V_(i - 1, j, k)) +
                            diff2(iy, V_(i, j + 1, k), Vc, V_(i, j - 1, k)) +
                            diff2(iz, V_(i, j, k + 1), Vc, V_(i, j, k - 1));
                A3(s->g, i, j, k) = Vc + dt * (iRe * lv - duvdx - dv2dy - dvwdz + s->gy);
                /* H */
                double duwdx = conv(ix, gm, Uc + U_(i, j, k + 1), Wc + W_(i + 1, j, k),
                                    Wc - W_(i + 1, j, k), U_(i - 1, j, k) + U_(i - 1, j, k + 1),
                                    Wc + W_(i - 1, j, k), Wc - W_(i - 1, j, k));
                double dvwdy = conv(iy, gm, Vc + V_(i, j, k + 1), Wc + W_(i, j + 1, k),
                                    Wc - W_(i, j + 1, k), V_(i, j - 1, k + 1) + V_(i, j - 1, k),
                                    Wc + W_(i, j - 1, k), Wc - W_(i, j - 1, k));
                double dw2dz = conv(iz, gm, Wc + W_(i, j, k + 1), Wc + W_(i, j, k + 1),
                                    Wc - W_(i, j, k + 1), Wc + W_(i, j, k - 1),
                                    Wc + W_(i, j, k - 1), Wc - W_(i, j, k - 1));
                double lw = diff2(ix, W_(i + 1, j, k), Wc, W_(i - 1, j, k)) +
                            diff2(iy, W_(i, j + 1, k), Wc, W_(i, j - 1, k)) +
                            diff2(iz, W_(i, j, k + 1), Wc, W_(i, j, k - 1));
                A3(s->h, i, j, k) = Wc + dt * (iRe * lw - duwdx - dvwdy - dw2dz + s->gz);
#undef U_
#undef V_
#undef W_
            }
    /* boundary values, solver.c:774-823 */
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++) {
            A3(s->f, 0, j, k) = A3(u, 0, j, k);
            A3(s->f, s->imax, j, k) = A3(u, s->imax, j, k);
        }
    for (int k = 1; k <= s->kmax; k++)
        for (int i = 1; i <= s->imax; i++) {
            A3(s->g, i, 0, k) = A3(v, i, 0, k);
            A3(s->g, i, s->jmax, k) = A3(v, i, s->jmax, k);
        }
    for (int j = 1; j <= s->jmax; j++)
        for (int i = 1; i <= s->imax; i++) {
            A3(s->h, i, j, 0) = A3(w, i, j, 0);
            A3(s->h, i, j, s->kmax) = A3(w, i, j, s->kmax);
        }
}

/* adaptUV, solver.c:826-853 */
void orc3_adapt_uvw(orc3* s)
{
    const double fx = s->dt / s->dx, fy = s->dt / s->dy, fz = s->dt / s->dz;
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++)
            for (int i = 1; i <= s->imax; i++) {
                const double pc = A3(s->p, i, j, k);
                A3(s->u, i, j, k) = A3(s->f, i, j, k) - (A3(s->p, i + 1, j, k) - pc) * fx;
                A3(s->v, i, j, k) = A3(s->g, i, j, k) - (A3(s->p, i, j + 1, k) - pc) * fy;
                A3(s->w, i, j, k) = A3(s->h, i, j, k) - (A3(s->p, i, j, k + 1) - pc) * fz;
            }
}

/* main loop of assignment-6/src/main.c:45-60 (no normalizePressure there) */
int orc3_run(orc3* s, int max_steps, int* iters, int cap, double* t_out)
{
    double t = 0.0;
    int nt = 0;
    while (t <= s->te && (max_steps < 0 || nt < max_steps)) {
        if (s->tau > 0.0) orc3_compute_timestep(s);
        orc3_set_bc(s);
        orc3_set_special_bc(s);
        orc3_compute_fg(s);
        orc3_compute_rhs(s);
        int it = orc3_solve(s, NULL);
        if (iters && nt < cap) iters[nt] = it;
        orc3_adapt_uvw(s);
        t += s->dt;
        nt++;
    }
    if (t_out) *t_out = t;
    return nt;
}

/* commCollectResult's single-domain branch (assignment-6/src/comm.c:386-426):
 * interior p and cell-centred velocities, imax*jmax*kmax each, i fastest */
void orc3_collect(const orc3* s, double* pg, double* ug, double* vg, double* wg)
{
    size_t q = 0;
    for (int k = 1; k <= s->kmax; k++)
        for (int j = 1; j <= s->jmax; j++)
            for (int i = 1; i <= s->imax; i++, q++) {
                pg[q] = A3(s->p, i, j, k);
                ug[q] = (A3(s->u, i, j, k) + A3(s->u, i - 1, j, k)) / 2.0;
                vg[q] = (A3(s->v, i, j, k) + A3(s->v, i, j - 1, k)) / 2.0;
                wg[q] = (A3(s->w, i, j, k) + A3(s->w, i, j, k - 1)) / 2.0;
            }
}
