#include <errno.h>
#include <stdio.h>
#include <stdlib.h>

#include "util.h"

void* allocate(int alignment, size_t bytesize)
{
    void* ptr = NULL;
    int rc = posix_memalign(&ptr, (size_t)alignment, bytesize);
    if (rc == EINVAL) {
        fprintf(stderr, "Error: Alignment parameter is not a power of two\n");
        exit(EXIT_FAILURE);
    }
    if (rc == ENOMEM || ptr == NULL) {
        fprintf(stderr, "Error: Insufficient memory to fulfill the request\n");
        exit(EXIT_FAILURE);
    }
    return ptr;
}
