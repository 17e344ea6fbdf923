/* comm-file -- the communicator-id handshake of ranks.c on its own, for the
 * CPU tests (tests/test_host_cpu.py): no RCCL, the id is given as text.
 *
 *   comm-file publish <world> <id-text> <readers>   rank 0: publish, wait for
 *        <readers> acknowledgements (<path>.ack<k>), then remove the files
 *   comm-file fetch <world> <k>                      rank k: print the id
 * The launch tag comes from the environment exactly as in ranks.c. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "comm_file.h"

#define ID_BYTES 128

int main(int argc, char** argv)
{
    if (argc < 4) return 2;
    char tag[COMM_TAG_BYTES], path[1024], ack[1100], id[ID_BYTES];
    if (commFileTag(tag, sizeof tag) != 0) snprintf(tag, sizeof tag, "file");
    commFilePath(atoi(argv[2]), tag, path, sizeof path);
    memset(id, 0, sizeof id);
    if (strcmp(argv[1], "publish") == 0 && argc >= 5) {
        unlink(path);
        snprintf(id, sizeof id, "%s", argv[3]);
        if (commFilePublish(path, tag, id, sizeof id) != 0) return 1;
        const int readers = atoi(argv[4]);
        for (int k = 1; k <= readers; ++k) {
            snprintf(ack, sizeof ack, "%s.ack%d", path, k);
            for (int t = 0; t < 3000 && access(ack, F_OK) != 0; ++t) {
                struct timespec ts = { 0, 10000000 };
                nanosleep(&ts, NULL);
            }
            unlink(ack);
        }
        unlink(path);
        return 0;
    }
    if (strcmp(argv[1], "fetch") == 0) {
        if (commFileFetch(path, tag, id, sizeof id, 20.0) != 0) return 1;
        printf("%s\n", id);
        fflush(stdout);
        snprintf(ack, sizeof ack, "%s.ack%d", path, atoi(argv[3]));
        FILE* fp = fopen(ack, "w");
        if (fp) fclose(fp);
        return 0;
    }
    return 2;
}
