/* progress.c -- "[####      ]" in tenths of the final time, redrawn in place */
#include "progress.h"

#include <math.h>
#include <stdio.h>

static double progEnd;
static int progCur;

void initProgress(double end)
{
    progEnd = end;
    progCur = 0;
    printf("[          ]");
    fflush(stdout);
}

void printProgress(double current)
{
    int now = (int)rint((current / progEnd) * 10.0);
    if (now > progCur) {
        char bar[11];
        progCur = now;
        for (int i = 0; i < 10; i++) bar[i] = (i < progCur) ? '#' : ' ';
        bar[10] = '\0';
        printf("\r[%s]", bar);
    }
    fflush(stdout);
}

void stopProgress(void)
{
    printf("\n");
    fflush(stdout);
}
