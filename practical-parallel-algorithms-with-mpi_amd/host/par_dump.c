/*
 * par_dump.c -- prints every field the host .par reader (parameter.c) produced,
 * one "key value" per line; tests/test_host_cpu.py compares it with the
 * reference's own readParameter (assignment-5/sequential/src/parameter.c)
 * run on the same files.
 *   par-dump <file.par> [poisson]
 */
#include <stdio.h>
#include <string.h>

#include "parameter.h"

int main(int argc, char** argv)
{
    Parameter p;
    if (argc < 2) {
        printf("Usage: %s <configFile> [poisson]\n", argv[0]);
        return 0;
    }
    if (argc > 2 && strcmp(argv[2], "poisson") == 0)
        initParameterPoisson(&p);
    else
        initParameter(&p);
    readParameter(&p, argv[1]);
    printf("xlength %.17g\nylength %.17g\nimax %d\njmax %d\nitermax %d\neps %.17g\nomg %.17g\n",
           p.xlength, p.ylength, p.imax, p.jmax, p.itermax, p.eps, p.omg);
    printf("re %.17g\ntau %.17g\ngamma %.17g\ndt %.17g\nte %.17g\ngx %.17g\ngy %.17g\n", p.re,
           p.tau, p.gamma, p.dt, p.te, p.gx, p.gy);
    printf("name %s\nbcLeft %d\nbcRight %d\nbcBottom %d\nbcTop %d\n", p.name ? p.name : "(null)",
           p.bcLeft, p.bcRight, p.bcBottom, p.bcTop);
    printf("u_init %.17g\nv_init %.17g\np_init %.17g\n", p.u_init, p.v_init, p.p_init);
    return 0;
}
