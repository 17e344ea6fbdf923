/* util.h -- host utilities (assignment-4/src/{allocate,timing}.c, util.h) */
#ifndef MISOR_HOST_UTIL_H
#define MISOR_HOST_UTIL_H
#include <stddef.h>

#ifndef MIN
#define MIN(x, y) ((x) < (y) ? (x) : (y))
#endif
#ifndef MAX
#define MAX(x, y) ((x) > (y) ? (x) : (y))
#endif

/* posix_memalign wrapper; prints and exits on failure like allocate.c:11-37 */
void* allocate(int alignment, size_t bytesize);
/* CLOCK_MONOTONIC seconds, timing.c:10-15 */
double getTimeStamp(void);
/* print libmisor's last error and exit(EXIT_FAILURE) when rc != 0 */
void misorCheck(int rc, const char* what);
#endif
