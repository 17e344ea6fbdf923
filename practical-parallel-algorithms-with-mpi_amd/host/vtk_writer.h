/*
 * vtk_writer.h -- legacy-VTK output of the 3D solver, the interface of
 * assignment-6/src/vtkWriter.h (vtkOpen / vtkScalar / vtkVector / vtkClose).
 * The file is "<problem>.vtk": a STRUCTURED_POINTS dataset of the
 * imax*jmax*kmax interior cells, ORIGIN at the first cell centre, point data
 * in i-fastest order; ASCII ("%f" per value) or BINARY (big-endian doubles,
 * each data block closed by a newline), as vtkWriter.c:44-190 writes it.
 */
#ifndef MISOR_HOST_VTK_WRITER_H
#define MISOR_HOST_VTK_WRITER_H
#include <stdio.h>

#include "solver_ns3d.h"

typedef enum VtkFormat { ASCII = 0, BINARY } VtkFormat;

typedef struct VtkOptions {
    VtkFormat fmt;
    Grid grid;
    FILE* fh;
} VtkOptions;

typedef struct VtkVector {
    double *u, *v, *w;
} VtkVector;

extern void vtkOpen(VtkOptions* opts, char* problem);
extern void vtkVector(VtkOptions* opts, char* name, VtkVector vec);
extern void vtkScalar(VtkOptions* opts, char* name, double* p);
extern void vtkClose(VtkOptions* opts);
#endif
