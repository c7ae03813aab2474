/* ora_io.h -- TEST INFRASTRUCTURE ONLY (see ora.h): .pss and skeleton I/O. */
#ifndef ULG_ORA_IO_H
#define ULG_ORA_IO_H
#include "ora.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int n;
    char **names;
    int64_t *offsets;   /* n+1 */
    ora_varset *sets;   /* file order within each variable */
    float *costs;       /* -1 * atof(score token) */
} ora_pss;

int ora_pss_write(const char *path, int n, const char *names, int name_stride,
                  const int *arity, const int64_t *offsets, const ora_varset *sets,
                  const float *scores, const char *input_file, int64_t num_records,
                  int parent_limit, const char *score_type);
int ora_pss_read(const char *path, ora_pss *out);
void ora_pss_free(ora_pss *p);
/* returns number of vertices (first row token count / n_expected for .arc),
 * or -1 if the file cannot be opened. */
int ora_skeleton_read(const char *path, int n_expected, ora_varset *edges, int max_n);

#ifdef __cplusplus
}
#endif
#endif
