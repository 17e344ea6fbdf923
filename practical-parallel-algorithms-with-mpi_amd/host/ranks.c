/* ranks.c -- see ranks.h */
#include "ranks.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "comm_file.h"
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

/* the communicator id of this launch: rank 0 creates and publishes it, the
 * others read it (comm_file.h); rank 0 removes the file when the program ends */
static char comm_path[1024];

static void remove_comm_file(void) { unlink(comm_path); }

static void publish_or_fetch_id(int rank, int world, char* id)
{
    char tag[COMM_TAG_BYTES];
    if (commFileTag(tag, sizeof tag) != 0) {
        if (!getenv("MISOR_COMM_FILE")) {
            printf("Error: WORLD_SIZE > 1 needs MASTER_PORT, TORCHELASTIC_RUN_ID, MISOR_RUN_TAG "
                   "or MISOR_COMM_FILE to tell this launch apart\n");
            exit(EXIT_FAILURE);
        }
        snprintf(tag, sizeof tag, "file");
    }
    commFilePath(world, tag, comm_path, sizeof comm_path);
    if (rank == 0) {
        unlink(comm_path); /* a file left by a crashed launch with the same tag */
        misorCheck(misor_comm_unique_id(id), "misor_comm_unique_id");
        if (commFilePublish(comm_path, tag, id, MISOR_COMM_ID_BYTES) != 0) {
            printf("Error: cannot publish %s\n", comm_path);
            exit(EXIT_FAILURE);
        }
        atexit(remove_comm_file);
        return;
    }
    if (commFileFetch(comm_path, tag, id, MISOR_COMM_ID_BYTES, 60.0) != 0) {
        printf("Error: no communicator id for launch %s in %s\n", tag, comm_path);
        exit(EXIT_FAILURE);
    }
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
