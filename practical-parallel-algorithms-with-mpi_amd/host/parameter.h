/*
 * parameter.h -- the reference's .par configuration, one struct for both
 * drivers: the union of the keys read by assignment-4/src/parameter.c:55-63
 * (Poisson), assignment-5/sequential/src/parameter.c:55-82 (2D NS) and
 * assignment-6/src/parameter.c:60-89 (whose 3D-only keys kmax, zlength, gz,
 * w_init, bcFront, bcBack are accepted and ignored by the 2D solvers).
 */
#ifndef MISOR_HOST_PARAMETER_H
#define MISOR_HOST_PARAMETER_H

typedef struct {
    double xlength, ylength, zlength;
    int imax, jmax, kmax;
    int itermax;
    double eps, omg;
    double re, tau, gamma;
    double te, dt;
    double gx, gy, gz;
    char* name;
    int bcLeft, bcRight, bcBottom, bcTop, bcFront, bcBack;
    double u_init, v_init, w_init, p_init;
} Parameter;

/* defaults of assignment-4/src/parameter.c:15-24 */
void initParameterPoisson(Parameter*);
/* defaults of assignment-5/sequential/src/parameter.c:15-27 */
void initParameter(Parameter*);
/* same line syntax and key matching as the reference (parameter.c:26-67) */
void readParameter(Parameter*, const char* filename);
void printParameterPoisson(Parameter*);
void printParameter(Parameter*);
/* assignment-6/src/parameter.c:95-126 (the 3D solver) */
void printParameter3D(Parameter*);

#endif
