/*
 * vtk_writer.c -- legacy-VTK writer (format of assignment-6/src/vtkWriter.c).
 * Values are written from the collected global arrays (collectResult), in
 * blocks: ASCII through one formatted buffer per block, BINARY as byte-swapped
 * 64-bit words, so a 128^3 field is a few large fwrite calls.
 */
#include "vtk_writer.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { CHUNK = 1 << 16 }; /* values per write */

static double bigEndian(double x)
{
    uint64_t b;
    memcpy(&b, &x, sizeof b);
    b = __builtin_bswap64(b);
    memcpy(&x, &b, sizeof b);
    return x;
}

static void writeHeader(VtkOptions* o)
{
    fprintf(o->fh, "# vtk DataFile Version 3.0\n");
    fprintf(o->fh, "PAMPI cfd solver output\n");
    fprintf(o->fh, o->fmt == BINARY ? "BINARY\n" : "ASCII\n");
    fprintf(o->fh, "DATASET STRUCTURED_POINTS\n");
    fprintf(o->fh, "DIMENSIONS %d %d %d\n", o->grid.imax, o->grid.jmax, o->grid.kmax);
    fprintf(o->fh, "ORIGIN %f %f %f\n", o->grid.dx * 0.5, o->grid.dy * 0.5, o->grid.dz * 0.5);
    fprintf(o->fh, "SPACING %f %f %f\n", o->grid.dx, o->grid.dy, o->grid.dz);
    fprintf(o->fh, "POINT_DATA %d\n", o->grid.imax * o->grid.jmax * o->grid.kmax);
}

void vtkOpen(VtkOptions* o, char* problem)
{
    char filename[50];
    snprintf(filename, sizeof filename, "%s.vtk", problem);
    o->fh = fopen(filename, "w");
    if (!o->fh) {
        fprintf(stderr, "Could not open %s\n", filename);
        exit(EXIT_FAILURE);
    }
    writeHeader(o);
    printf("Writing VTK output for %s\n", problem);
}

/* ncomp interleaved components per point (1: scalar, 3: vector) */
static void writeBlock(VtkOptions* o, double* const* comp, int ncomp)
{
    const size_t n = (size_t)o->grid.imax * o->grid.jmax * o->grid.kmax;
    if (o->fmt == BINARY) {
        double* buf = malloc(sizeof(double) * CHUNK * ncomp);
        for (size_t q0 = 0; q0 < n; q0 += CHUNK) {
            size_t m = (n - q0 < CHUNK) ? n - q0 : CHUNK;
            for (size_t q = 0; q < m; q++)
                for (int c = 0; c < ncomp; c++) buf[q * ncomp + c] = bigEndian(comp[c][q0 + q]);
            fwrite(buf, sizeof(double), m * ncomp, o->fh);
        }
        free(buf);
        fprintf(o->fh, "\n");
        return;
    }
    /* ASCII: "%f\n" or "%f %f %f\n"; 3 * (%f of |x| < 1e300) fits 1024 bytes */
    char* buf = malloc((size_t)CHUNK * 1024);
    for (size_t q0 = 0; q0 < n; q0 += CHUNK) {
        size_t m = (n - q0 < CHUNK) ? n - q0 : CHUNK, len = 0;
        for (size_t q = 0; q < m; q++) {
            if (ncomp == 1)
                len += (size_t)sprintf(buf + len, "%f\n", comp[0][q0 + q]);
            else
                len += (size_t)sprintf(buf + len, "%f %f %f\n", comp[0][q0 + q],
                                       comp[1][q0 + q], comp[2][q0 + q]);
        }
        fwrite(buf, 1, len, o->fh);
    }
    free(buf);
}

void vtkScalar(VtkOptions* o, char* name, double* s)
{
    printf("Register scalar %s\n", name);
    if (!o->fh) {
        printf("vtkWriter not initialize! Call vtkOpen first!\n");
        return;
    }
    fprintf(o->fh, "SCALARS %s double 1\n", name);
    fprintf(o->fh, "LOOKUP_TABLE default\n");
    writeBlock(o, &s, 1);
}

void vtkVector(VtkOptions* o, char* name, VtkVector vec)
{
    printf("Register vector %s\n", name);
    if (!o->fh) {
        printf("vtkWriter not initialize! Call vtkOpen first!\n");
        return;
    }
    fprintf(o->fh, "VECTORS %s double\n", name);
    double* comp[3] = { vec.u, vec.v, vec.w };
    writeBlock(o, comp, 3);
}

void vtkClose(VtkOptions* o)
{
    fclose(o->fh);
    o->fh = NULL;
}
