/* progress.h -- the reference's progress bar (assignment-6/src/progress.c:17-51) */
#ifndef MISOR_HOST_PROGRESS_H
#define MISOR_HOST_PROGRESS_H
void initProgress(double end);
void printProgress(double current);
void stopProgress(void);
#endif
