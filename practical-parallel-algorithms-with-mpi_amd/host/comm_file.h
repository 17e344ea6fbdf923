/*
 * comm_file.h -- hand the RCCL communicator id from rank 0 to the other
 * processes of one launch (WORLD_SIZE > 1, see ranks.h) through a file.
 *
 * The reference's MPI programs get their communicator from MPI_Init
 * (assignment-5/skeleton/src/main.c:25); here rank 0 creates the id and the
 * other ranks read it.  The file name and its content carry a tag of the
 * launch (MISOR_RUN_TAG, else torchrun's TORCHELASTIC_RUN_ID + MASTER_PORT,
 * else MASTER_ADDR:MASTER_PORT), so a file left by an earlier launch is
 * never taken for this one's; rank 0 writes it atomically (tmp + rename) and
 * removes it when the program ends.
 */
#ifndef MISOR_HOST_COMM_FILE_H
#define MISOR_HOST_COMM_FILE_H
#include <stddef.h>

#define COMM_TAG_BYTES 96

/* the launch tag (0) or -1 when the environment names no launch */
int commFileTag(char* tag, size_t n);
/* MISOR_COMM_FILE, else /tmp/misor_comm_<world>_<tag>.id (tag sanitised) */
void commFilePath(int world, const char* tag, char* path, size_t n);
/* rank 0: write tag + id (id_bytes) to path; 0 or -1 */
int commFilePublish(const char* path, const char* tag, const void* id, size_t id_bytes);
/* other ranks: wait up to timeout_s for a file at path whose tag is `tag`,
 * copy its id; 0 or -1 (timeout) */
int commFileFetch(const char* path, const char* tag, void* id, size_t id_bytes,
                  double timeout_s);
#endif
