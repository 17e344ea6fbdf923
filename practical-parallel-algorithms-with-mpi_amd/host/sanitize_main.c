/*
 * sanitize_main.c -- the host-only code of the drop-in programs under
 * AddressSanitizer + UndefinedBehaviorSanitizer (make asan -> bin/asan/host-check;
 * tests/test_sanitize_cpu.py).  GPU code is not sanitized (no GPU ASan on this
 * pool); everything here runs on the CPU:
 *   * the .par reader on each file named on the command line (every key of
 *     the reference's readParameter, assignment-5/sequential/src/parameter.c:29-85,
 *     plus the printParameter* formatting),
 *   * the RCCL-id hand-off file (comm_file.c): tag, path, publish, fetch of the
 *     right tag, refusal of a stale file of another launch,
 *   * the legacy-VTK writer (vtk_writer.c, assignment-6/src/vtkWriter.c) in
 *     ASCII and BINARY on a grid whose size is not a multiple of its chunk.
 *   host-check <dir for output files> <file.par>...
 * Exit 0 when every check passes; sanitizer reports abort with a non-zero code.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "comm_file.h"
#include "parameter.h"
#include "vtk_writer.h"

static int fails = 0;
#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                     \
        }                                                                \
    } while (0)

static void checkPar(const char* path)
{
    Parameter p;
    initParameter(&p);
    readParameter(&p, path);
    CHECK(p.imax > 0 && p.jmax > 0);
    printParameter(&p);
    printParameter3D(&p);
    free(p.name);
    Parameter q;
    initParameterPoisson(&q);
    readParameter(&q, path);
    printParameterPoisson(&q);
    free(q.name);
}

static void checkCommFile(const char* dir)
{
    char tag[COMM_TAG_BYTES], path[1024], other[1024];
    setenv("MISOR_RUN_TAG", "sanitize run/1 <tag>", 1);
    unsetenv("MISOR_COMM_FILE");
    CHECK(commFileTag(tag, sizeof tag) == 0);
    commFilePath(4, tag, path, sizeof path);
    CHECK(strchr(path + strlen("/tmp/"), '/') == NULL);  /* tag sanitised */
    snprintf(path, sizeof path, "%s/comm.id", dir);
    snprintf(other, sizeof other, "%s", "an earlier launch");
    unsigned char id[128], got[128];
    for (int k = 0; k < 128; ++k) id[k] = (unsigned char)(k * 37 + 1);
    /* a stale file of another launch is never taken for this one */
    CHECK(commFilePublish(path, other, id, sizeof id) == 0);
    CHECK(commFileFetch(path, tag, got, sizeof got, 0.05) == -1);
    CHECK(commFilePublish(path, tag, id, sizeof id) == 0);
    memset(got, 0, sizeof got);
    CHECK(commFileFetch(path, tag, got, sizeof got, 1.0) == 0);
    CHECK(memcmp(id, got, sizeof id) == 0);
    unlink(path);
    unsetenv("MISOR_RUN_TAG");
}

static void checkVtk(const char* dir)
{
    const Grid g = { 37, 29, 67, 1.0, 2.0, 3.0, 1.0 / 37, 2.0 / 29, 3.0 / 67 };
    const size_t n = (size_t)g.imax * g.jmax * g.kmax; /* 71891 > one 65536 chunk */
    double* f[4];
    for (int c = 0; c < 4; ++c) {
        f[c] = malloc(n * sizeof(double));
        for (size_t q = 0; q < n; ++q) f[c][q] = (double)(q % 1013) * 0.25 - c * 1e5;
    }
    char cwd[1024];
    CHECK(getcwd(cwd, sizeof cwd) != NULL);
    CHECK(chdir(dir) == 0);
    for (int fmt = 0; fmt < 2; ++fmt) {
        VtkOptions o = { .fmt = fmt ? BINARY : ASCII, .grid = g };
        vtkOpen(&o, fmt ? "sanitize_bin" : "sanitize_ascii");
        vtkScalar(&o, "pressure", f[0]);
        vtkVector(&o, "velocity", (VtkVector){ f[1], f[2], f[3] });
        vtkClose(&o);
        FILE* fh = fopen(fmt ? "sanitize_bin.vtk" : "sanitize_ascii.vtk", "rb");
        CHECK(fh != NULL);
        if (fh) {
            fseek(fh, 0, SEEK_END);
            const long sz = ftell(fh);
            /* binary: 4 values per point (1 scalar + 3 vector) of 8 bytes */
            CHECK(sz > (long)(fmt ? 32 * n : 8 * n));
            fclose(fh);
        }
    }
    CHECK(chdir(cwd) == 0);
    for (int c = 0; c < 4; ++c) free(f[c]);
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        printf("Usage: %s <output dir> <file.par>...\n", argv[0]);
        return 2;
    }
    for (int k = 2; k < argc; ++k) checkPar(argv[k]);
    checkCommFile(argv[1]);
    checkVtk(argv[1]);
    if (fails) fprintf(stderr, "%d checks failed\n", fails);
    else printf("host-check: all checks passed\n");
    return fails ? 1 : 0;
}
