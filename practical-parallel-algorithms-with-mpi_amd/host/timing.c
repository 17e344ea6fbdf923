#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "misor.h"
#include "util.h"

double getTimeStamp(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1.e-9;
}

void misorCheck(int rc, const char* what)
{
    if (rc != MISOR_OK) {
        fprintf(stderr, "Error: %s failed (%d): %s\n", what, rc, misor_last_error());
        exit(EXIT_FAILURE);
    }
}
