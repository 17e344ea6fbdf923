/*
 * ranks.h -- how the host programs run as several ranks without MPI.
 *
 * The reference's MPI programs (assignment-5/skeleton/src/main.c:18-66) are
 * started as `mpirun -np N exe <par>`; every rank runs the same main loop on
 * its subdomain and rank 0 prints and writes the output.  Here a rank is one
 * libmisor grid of a decomposed domain, driven either by
 *   - a thread of this process: MISOR_RANKS=N (in-process transport; rank r
 *     on GPU r % device_count, so one process drives all GPUs of a node), or
 *   - a process per rank started by a launcher that sets WORLD_SIZE, RANK and
 *     LOCAL_RANK (torchrun style): RCCL between the processes, rank 0
 *     publishes the communicator id in a file tagged with the launch
 *     (comm_file.h: MISOR_COMM_FILE, default /tmp/misor_comm_<WORLD_SIZE>_<tag>.id).
 * With neither set the program is the single-GPU one.
 */
#ifndef MISOR_HOST_RANKS_H
#define MISOR_HOST_RANKS_H
#include "misor.h"

typedef struct {
    int rank, size, device;
    const void* comm_id; /* MISOR_COMM_ID_BYTES, NULL for a single rank */
} RankCtx;

/* run fn on every rank of this process (one or more threads); returns the
 * first non-zero result */
int runRanks(int (*fn)(const RankCtx*, void*), void* arg);
/* the calling thread's rank (valid inside fn; rank 0 of 1 otherwise) */
const RankCtx* currentRank(void);
#endif
