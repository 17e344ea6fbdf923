/*
 * parameter.c -- .par reader with the reference's exact line semantics
 * (assignment-4/src/parameter.c:26-67, assignment-5/sequential/src/parameter.c:29-85):
 *   - read line by line (4096 bytes max), cut at the first '#';
 *   - the key is the first space-separated token, the value the second
 *     (only ' ' separates tokens: "key\tvalue" is one token, as in the reference);
 *   - a key matches when the token STARTS WITH the key name (strncmp over the
 *     key's length), so "reynolds 5" sets re, exactly like the reference;
 *   - integers via atoi, reals via atof, name via strdup of the raw token
 *     (a trailing newline is kept when no comment follows, as in the reference).
 */
#include "parameter.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXLINE 4096

static void zero(Parameter* p) { memset(p, 0, sizeof *p); }

void initParameterPoisson(Parameter* p)
{
    zero(p);
    p->xlength = 1.0;
    p->ylength = 1.0;
    p->imax = 100;
    p->jmax = 100;
    p->itermax = 1000;
    p->eps = 0.0001;
    p->omg = 1.8;
}

void initParameter(Parameter* p)
{
    zero(p);
    p->xlength = 1.0;
    p->ylength = 1.0;
    p->zlength = 1.0;
    p->imax = 100;
    p->jmax = 100;
    p->kmax = 100;
    p->itermax = 1000;
    p->eps = 0.0001;
    p->omg = 1.7;
    p->re = 100.0;
    p->gamma = 0.9;
    p->tau = 0.5;
}

static int starts_with(const char* tok, const char* key)
{
    return strncmp(tok, key, strlen(key)) == 0;
}

void readParameter(Parameter* param, const char* filename)
{
    FILE* fp = fopen(filename, "r");
    char line[MAXLINE];

    if (!fp) {
        fprintf(stderr, "Could not open parameter file: %s\n", filename);
        exit(EXIT_FAILURE);
    }

    while (!feof(fp)) {
        line[0] = '\0';
        if (!fgets(line, MAXLINE, fp)) line[0] = '\0';
        char* hash = strchr(line, '#');
        if (hash) *hash = '\0';

        char* tok = strtok(line, " ");
        char* val = strtok(NULL, " ");
        if (tok == NULL || val == NULL) continue;

        /* every matching key is applied, in the reference's order */
        struct { const char* key; char kind; void* dst; } keys[] = {
            { "xlength", 'r', &param->xlength }, { "ylength", 'r', &param->ylength },
            { "zlength", 'r', &param->zlength }, { "imax", 'i', &param->imax },
            { "jmax", 'i', &param->jmax },       { "kmax", 'i', &param->kmax },
            { "itermax", 'i', &param->itermax }, { "eps", 'r', &param->eps },
            { "omg", 'r', &param->omg },         { "re", 'r', &param->re },
            { "tau", 'r', &param->tau },         { "gamma", 'r', &param->gamma },
            { "dt", 'r', &param->dt },           { "te", 'r', &param->te },
            { "gx", 'r', &param->gx },           { "gy", 'r', &param->gy },
            { "gz", 'r', &param->gz },           { "name", 's', &param->name },
            { "bcLeft", 'i', &param->bcLeft },   { "bcRight", 'i', &param->bcRight },
            { "bcBottom", 'i', &param->bcBottom }, { "bcTop", 'i', &param->bcTop },
            { "bcFront", 'i', &param->bcFront }, { "bcBack", 'i', &param->bcBack },
            { "u_init", 'r', &param->u_init },   { "v_init", 'r', &param->v_init },
            { "w_init", 'r', &param->w_init },   { "p_init", 'r', &param->p_init },
        };
        for (size_t k = 0; k < sizeof keys / sizeof keys[0]; k++) {
            if (!starts_with(tok, keys[k].key)) continue;
            switch (keys[k].kind) {
            case 'i': *(int*)keys[k].dst = atoi(val); break;
            case 'r': *(double*)keys[k].dst = atof(val); break;
            case 's':
                free(*(char**)keys[k].dst);
                *(char**)keys[k].dst = strdup(val);
                break;
            }
        }
    }
    fclose(fp);
}

/* assignment-4/src/parameter.c:69-79 */
void printParameterPoisson(Parameter* param)
{
    printf("Parameters:\n");
    printf("Geometry data:\n");
    printf("\tDomain box size (x, y): %e, %e\n", param->xlength, param->ylength);
    printf("\tCells (x, y): %d, %d\n", param->imax, param->jmax);
    printf("Iterative solver parameters:\n");
    printf("\tMax iterations: %d\n", param->itermax);
    printf("\tepsilon (stopping tolerance) : %e\n", param->eps);
    printf("\tomega (SOR relaxation): %e\n", param->omg);
}

/* assignment-5/sequential/src/parameter.c:87-111 */
void printParameter(Parameter* param)
{
    printf("Parameters for %s\n", param->name ? param->name : "(null)");
    printf("Boundary conditions Left:%d Right:%d Bottom:%d Top:%d\n", param->bcLeft,
           param->bcRight, param->bcBottom, param->bcTop);
    printf("\tReynolds number: %.2f\n", param->re);
    printf("\tInit arrays: U:%.2f V:%.2f P:%.2f\n", param->u_init, param->v_init,
           param->p_init);
    printf("Geometry data:\n");
    printf("\tDomain box size (x, y): %.2f, %.2f\n", param->xlength, param->ylength);
    printf("\tCells (x, y): %d, %d\n", param->imax, param->jmax);
    printf("Timestep parameters:\n");
    printf("\tDefault stepsize: %.2f, Final time %.2f\n", param->dt, param->te);
    printf("\tTau factor: %.2f\n", param->tau);
    printf("Iterative solver parameters:\n");
    printf("\tMax iterations: %d\n", param->itermax);
    printf("\tepsilon (stopping tolerance) : %f\n", param->eps);
    printf("\tgamma (stopping tolerance) : %f\n", param->gamma);
    printf("\tomega (SOR relaxation): %f\n", param->omg);
}

/* assignment-6/src/parameter.c:95-126 */
void printParameter3D(Parameter* param)
{
    printf("Parameters for %s\n", param->name ? param->name : "(null)");
    printf("Boundary conditions Left:%d Right:%d Bottom:%d Top:%d Front:%d "
           "Back:%d\n",
           param->bcLeft, param->bcRight, param->bcBottom, param->bcTop, param->bcFront,
           param->bcBack);
    printf("\tReynolds number: %.2f\n", param->re);
    printf("\tInit arrays: U:%.2f V:%.2f W:%.2f P:%.2f\n", param->u_init, param->v_init,
           param->w_init, param->p_init);
    printf("Geometry data:\n");
    printf("\tDomain box size (x, y, z): %.2f, %.2f, %.2f\n", param->xlength, param->ylength,
           param->zlength);
    printf("\tCells (x, y, z): %d, %d, %d\n", param->imax, param->jmax, param->kmax);
    printf("Timestep parameters:\n");
    printf("\tDefault stepsize: %.2f, Final time %.2f\n", param->dt, param->te);
    printf("\tTau factor: %.2f\n", param->tau);
    printf("Iterative solver parameters:\n");
    printf("\tMax iterations: %d\n", param->itermax);
    printf("\tepsilon (stopping tolerance) : %f\n", param->eps);
    printf("\tgamma (stopping tolerance) : %f\n", param->gamma);
    printf("\tomega (SOR relaxation): %f\n", param->omg);
}
