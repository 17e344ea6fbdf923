/* comm_file.c -- see comm_file.h */
#include "comm_file.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static const char kMagic[8] = { 'M', 'I', 'S', 'O', 'R', 'I', 'D', '1' };

static const char* env(const char* name)
{
    const char* s = getenv(name);
    return (s && *s) ? s : NULL;
}

int commFileTag(char* tag, size_t n)
{
    const char* t = env("MISOR_RUN_TAG");
    const char* run = env("TORCHELASTIC_RUN_ID");
    const char* addr = env("MASTER_ADDR");
    const char* port = env("MASTER_PORT");
    if (t)
        snprintf(tag, n, "%s", t);
    else if (run && strcmp(run, "none") != 0)
        snprintf(tag, n, "%s-%s", run, port ? port : "");
    else if (port)
        snprintf(tag, n, "%s-%s", addr ? addr : "", port);
    else
        return -1;
    return 0;
}

void commFilePath(int world, const char* tag, char* path, size_t n)
{
    const char* f = env("MISOR_COMM_FILE");
    if (f) {
        snprintf(path, n, "%s", f);
        return;
    }
    char safe[COMM_TAG_BYTES];
    size_t k = 0;
    for (; tag[k] && k + 1 < sizeof safe; ++k) {
        const char c = tag[k];
        const int ok = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
                       c == '-' || c == '_' || c == '.';
        safe[k] = ok ? c : '_';
    }
    safe[k] = '\0';
    snprintf(path, n, "/tmp/misor_comm_%d_%s.id", world, safe);
}

int commFilePublish(const char* path, const char* tag, const void* id, size_t id_bytes)
{
    char tmp[1024], t[COMM_TAG_BYTES];
    memset(t, 0, sizeof t);
    snprintf(t, sizeof t, "%s", tag);
    snprintf(tmp, sizeof tmp, "%s.%d.tmp", path, (int)getpid());
    FILE* fp = fopen(tmp, "wb");
    if (!fp) return -1;
    const int ok = fwrite(kMagic, 1, sizeof kMagic, fp) == sizeof kMagic &&
                   fwrite(t, 1, sizeof t, fp) == sizeof t &&
                   fwrite(id, 1, id_bytes, fp) == id_bytes;
    if (fclose(fp) != 0 || !ok) {
        unlink(tmp);
        return -1;
    }
    if (rename(tmp, path) != 0) {
        unlink(tmp);
        return -1;
    }
    return 0;
}

int commFileFetch(const char* path, const char* tag, void* id, size_t id_bytes, double timeout_s)
{
    char want[COMM_TAG_BYTES];
    memset(want, 0, sizeof want);
    snprintf(want, sizeof want, "%s", tag);
    const long polls = (long)(timeout_s / 0.02) + 1;
    for (long k = 0; k < polls; ++k) {
        FILE* fp = fopen(path, "rb");
        if (fp) {
            char m[sizeof kMagic], t[COMM_TAG_BYTES];
            const int ok = fread(m, 1, sizeof m, fp) == sizeof m &&
                           fread(t, 1, sizeof t, fp) == sizeof t &&
                           memcmp(m, kMagic, sizeof m) == 0 && memcmp(t, want, sizeof t) == 0 &&
                           fread(id, 1, id_bytes, fp) == id_bytes;
            fclose(fp);
            if (ok) return 0;  /* a file of another launch: keep waiting for ours */
        }
        struct timespec ts = { 0, 20000000 };
        nanosleep(&ts, NULL);
    }
    return -1;
}
