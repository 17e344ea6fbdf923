/* ranks.c -- see ranks.h */
#include "ranks.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "util.h"

static __thread const RankCtx* tls_ctx;
static const RankCtx single = { 0, 1, -1, NULL };

const RankCtx* currentRank(void) { return tls_ctx ? tls_ctx : &single; }

typedef struct {
    RankCtx ctx;
    int (*fn)(const RankCtx*, void*);
    void* arg;
    int result;
} Job;

static void* thread_main(void* p)
{
    Job* j = (Job*)p;
    tls_ctx = &j->ctx;
    j->result = j->fn(&j->ctx, j->arg);
    return NULL;
}

static int env_int(const char* name, int dflt)
{
    const char* s = getenv(name);
    return (s && *s) ? atoi(s) : dflt;
}

/* rank 0 writes the id (tmp file + rename: readers never see a partial id) */
static void publish_or_fetch_id(int rank, int world, char* id)
{
    char path[512], tmp[600];
    const char* f = getenv("MISOR_COMM_FILE");
    if (f && *f)
        snprintf(path, sizeof path, "%s", f);
    else
        snprintf(path, sizeof path, "/tmp/misor_comm_%d.id", world);
    if (rank == 0) {
        misorCheck(misor_comm_unique_id(id), "misor_comm_unique_id");
        snprintf(tmp, sizeof tmp, "%s.%d.tmp", path, (int)getpid());
        FILE* fp = fopen(tmp, "wb");
        if (!fp || fwrite(id, 1, MISOR_COMM_ID_BYTES, fp) != MISOR_COMM_ID_BYTES) {
            printf("Error: cannot write %s\n", tmp);
            exit(EXIT_FAILURE);
        }
        fclose(fp);
        if (rename(tmp, path) != 0) {
            printf("Error: cannot publish %s\n", path);
            exit(EXIT_FAILURE);
        }
        return;
    }
    for (int tries = 0; tries < 1200; ++tries) { /* up to 60 s */
        FILE* fp = fopen(path, "rb");
        if (fp) {
            size_t n = fread(id, 1, MISOR_COMM_ID_BYTES, fp);
            fclose(fp);
            if (n == MISOR_COMM_ID_BYTES) return;
        }
        struct timespec ts = { 0, 50000000 };
        nanosleep(&ts, NULL);
    }
    printf("Error: no communicator id in %s\n", path);
    exit(EXIT_FAILURE);
}

int runRanks(int (*fn)(const RankCtx*, void*), void* arg)
{
    const int world = env_int("WORLD_SIZE", 1);
    const int threads = env_int("MISOR_RANKS", 1);
    if (world > 1) { /* one process per rank, RCCL */
        static char id[MISOR_COMM_ID_BYTES];
        RankCtx c;
        c.rank = env_int("RANK", 0);
        c.size = world;
        c.device = env_int("LOCAL_RANK", 0);
        publish_or_fetch_id(c.rank, world, id);
        c.comm_id = id;
        tls_ctx = &c;
        return fn(&c, arg);
    }
    if (threads <= 1) {
        tls_ctx = &single;
        return fn(&single, arg);
    }
    int ndev = 1;
    misorCheck(misor_device_count(&ndev), "misor_device_count");
    if (ndev < 1) ndev = 1;
    static char lid[MISOR_COMM_ID_BYTES];
    memset(lid, 0, sizeof lid);
    snprintf(lid, sizeof lid, "LOCAL:host-%d", (int)getpid());
    Job* jobs = (Job*)calloc((size_t)threads, sizeof(Job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) {
        printf("Error: out of memory\n");
        exit(EXIT_FAILURE);
    }
    for (int r = 0; r < threads; ++r) {
        jobs[r].ctx.rank = r;
        jobs[r].ctx.size = threads;
        jobs[r].ctx.device = r % ndev;
        jobs[r].ctx.comm_id = lid;
        jobs[r].fn = fn;
        jobs[r].arg = arg;
        if (pthread_create(&th[r], NULL, thread_main, &jobs[r]) != 0) {
            printf("Error: cannot start rank %d\n", r);
            exit(EXIT_FAILURE);
        }
    }
    int rc = 0;
    for (int r = 0; r < threads; ++r) {
        pthread_join(th[r], NULL);
        if (jobs[r].result && !rc) rc = jobs[r].result;
    }
    free(jobs);
    free(th);
    return rc;
}
