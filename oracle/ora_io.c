/* ora_io.c -- TEST INFRASTRUCTURE ONLY (see ora.h).
 *
 * Restates the reference's text formats on the hot path:
 *   .pss writer     score/score_main.cpp:173-203 (per variable), :383-400 (header)
 *   .pss reader     score_cache/score_cache.cpp:30-160 (two passes, case-
 *                   insensitive substring tests for "var " and "meta")
 *   skeleton        base/skeleton.cpp:19-105 (matrix: "TRUE" or |x| > 0.05;
 *                   arc list "Xn,Xm" with atoi(token+2))
 */
#define _GNU_SOURCE
#include "ora_io.h"
#include "ora_internal.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

/* ---- writer ---------------------------------------------------------- */
int ora_pss_write(const char *path, int n, const char *names, int name_stride,
                  const int *arity, const int64_t *offsets, const ora_varset *sets,
                  const float *scores, const char *input_file, int64_t num_records,
                  int parent_limit, const char *score_type) {
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    fprintf(f, "META pss_version = 0.1\nMETA input_file=%s\nMETA num_records=%lld\n",
            input_file, (long long)num_records);
    fprintf(f, "META parent_limit=%d\nMETA score_type=%s\nMETA ess=1\n\n", parent_limit, score_type);
    for (int v = 0; v < n; v++) {
        fprintf(f, "VAR %s\n", names + (size_t)v * name_stride);
        fprintf(f, "META arity=%d\n", arity[v]);
        for (int64_t i = offsets[v]; i < offsets[v + 1]; i++) {
            fprintf(f, "%f ", (double)scores[i]);
            for (int p = 0; p < n; p++)
                if ((sets[i] >> p) & 1ULL) fprintf(f, "%s ", names + (size_t)p * name_stride);
            fprintf(f, "\n");
        }
        fprintf(f, "\n");
    }
    fclose(f);
    return 0;
}

/* ---- reader ---------------------------------------------------------- */
static int icontains(const char *line, const char *needle) {
    size_t ln = strlen(line), nn = strlen(needle);
    if (nn > ln) return 0;
    for (size_t i = 0; i + nn <= ln; i++)
        if (strncasecmp(line + i, needle, nn) == 0) return 1;
    return 0;
}
/* boost::trim then boost::split(tokens, s, is_any_of(delims), token_compress_on) */
static int tokenize(const char *src, const char *delims, char ***out) {
    while (*src && isspace((unsigned char)*src)) src++;
    size_t l = strlen(src);
    while (l > 0 && isspace((unsigned char)src[l - 1])) l--;
    char *s = (char *)malloc(l + 1);
    memcpy(s, src, l); s[l] = 0;
    int cap = 16, nt = 0;
    char **tok = (char **)malloc(sizeof(char *) * (size_t)cap);
    char *p = s;
    tok[nt++] = p;
    for (; *p; p++) {
        if (strchr(delims, *p)) {
            *p = 0;
            while (p[1] && strchr(delims, p[1])) p++;
            if (nt == cap) { cap *= 2; tok = (char **)realloc(tok, sizeof(char *) * (size_t)cap); }
            tok[nt++] = p + 1;
        }
    }
    *out = tok;
    return nt; /* tok[0] owns the buffer */
}
static void free_tokens(char **tok) { free(tok[0]); free(tok); }

typedef struct { char **names; int n, cap; } namelist;
static int name_index(const namelist *nl, const char *name) {
    for (int i = 0; i < nl->n; i++) if (strcmp(nl->names[i], name) == 0) return i;
    return -1;
}

int ora_pss_read(const char *path, ora_pss *out) {
    memset(out, 0, sizeof(*out));
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char *line = NULL;
    size_t cap = 0;
    ssize_t len;
    namelist nl = {NULL, 0, 0};
    char **tok;
    int nt, started = 0;
    /* pass 1: META lines, then variable names */
    while ((len = getline(&line, &cap, f)) >= 0) {
        if (len > 0 && line[len - 1] == '\n') line[--len] = 0;
        if (len == 0 || line[0] == '#') continue;
        if (!started) {
            if (icontains(line, "var ")) started = 1;
            else {
                if (!icontains(line, "meta")) { free(line); fclose(f); return -2; }
                continue;
            }
        }
        if (icontains(line, "var ")) {
            nt = tokenize(line, " ", &tok);
            if (nt >= 2) {
                if (name_index(&nl, tok[1]) >= 0) { free_tokens(tok); free(line); fclose(f); return -3; }
                if (nl.n == nl.cap) { nl.cap = nl.cap ? nl.cap * 2 : 16; nl.names = (char **)realloc(nl.names, sizeof(char *) * (size_t)nl.cap); }
                nl.names[nl.n++] = strdup(tok[1]);
            }
            free_tokens(tok);
        }
    }
    const int n = nl.n;
    out->n = n;
    out->names = nl.names;
    /* pass 2: parent sets */
    rewind(f);
    int64_t *cnt = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t total = 0, tcap = 1024;
    int *var_of = (int *)malloc(sizeof(int) * (size_t)tcap);
    ora_varset *sets = (ora_varset *)malloc(sizeof(ora_varset) * (size_t)tcap);
    float *costs = (float *)malloc(sizeof(float) * (size_t)tcap);
    int cur = -1;
    while ((len = getline(&line, &cap, f)) >= 0) {
        if (len > 0 && line[len - 1] == '\n') line[--len] = 0;
        if (len == 0 || line[0] == '#' || icontains(line, "meta")) continue;
        nt = tokenize(line, " ", &tok);
        if (icontains(line, "var ")) {
            cur = nt >= 2 ? name_index(&nl, tok[1]) : -1;
            if (cur < 0) cur = 0; /* nameToIndex[] default-inserts 0 */
            free_tokens(tok);
            continue;
        }
        if (cur < 0) { free_tokens(tok); continue; }
        float c = -1 * atof(tok[0]); /* score_cache.cpp:151 */
        ora_varset ps = 0;
        for (int i = 1; i < nt; i++) {
            int idx = name_index(&nl, tok[i]);
            if (idx < 0) idx = 0; /* nameToIndex[] default-inserts 0 */
            ps |= 1ULL << idx;
        }
        free_tokens(tok);
        if (total == tcap) {
            tcap *= 2;
            var_of = (int *)realloc(var_of, sizeof(int) * (size_t)tcap);
            sets = (ora_varset *)realloc(sets, sizeof(ora_varset) * (size_t)tcap);
            costs = (float *)realloc(costs, sizeof(float) * (size_t)tcap);
        }
        var_of[total] = cur; sets[total] = ps; costs[total] = c; total++;
        cnt[cur]++;
    }
    free(line);
    fclose(f);
    /* putScore: (*cache[v])[parents] = score (score_cache.h:47-49) -- a repeated
     * set keeps one entry, its first position in file order and its last value */
    omap *seen = (omap *)malloc(sizeof(omap) * (size_t)(n > 0 ? n : 1));
    for (int v = 0; v < n; v++) { omap_init(&seen[v], 64); cnt[v] = 0; }
    int64_t *slot = (int64_t *)malloc(sizeof(int64_t) * (size_t)(total ? total : 1));
    for (int64_t i = 0; i < total; i++) {
        const int v = var_of[i];
        uint64_t first;
        if (omap_get(&seen[v], sets[i], &first)) { slot[i] = -1 - (int64_t)first; continue; }
        omap_put(&seen[v], sets[i], (uint64_t)cnt[v]);
        slot[i] = cnt[v]++;
    }
    /* group by variable, keeping file order within each variable */
    out->offsets = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    out->offsets[0] = 0;
    for (int v = 0; v < n; v++) out->offsets[v + 1] = out->offsets[v] + cnt[v];
    out->sets = (ora_varset *)malloc(sizeof(ora_varset) * (size_t)(total ? total : 1));
    out->costs = (float *)malloc(sizeof(float) * (size_t)(total ? total : 1));
    for (int64_t i = 0; i < total; i++) {
        const int v = var_of[i];
        const int64_t k = slot[i] >= 0 ? slot[i] : -1 - slot[i];
        out->sets[out->offsets[v] + k] = sets[i];
        out->costs[out->offsets[v] + k] = costs[i];
    }
    for (int v = 0; v < n; v++) omap_free(&seen[v]);
    free(seen); free(slot); free(cnt); free(var_of); free(sets); free(costs);
    return 0;
}

void ora_pss_free(ora_pss *p) {
    for (int i = 0; i < p->n; i++) free(p->names[i]);
    free(p->names); free(p->offsets); free(p->sets); free(p->costs);
    memset(p, 0, sizeof(*p));
}

/* ---- skeleton -------------------------------------------------------- */
int ora_skeleton_read(const char *path, int n_expected, ora_varset *edges, int max_n) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char *line = NULL;
    size_t cap = 0;
    ssize_t len;
    const size_t pl = strlen(path);
    int is_arc = pl >= 4 && strcmp(path + pl - 4, ".arc") == 0;
    for (int i = 0; i < max_n; i++) edges[i] = 0;
    int nv = 0;
    if (is_arc) {
        nv = n_expected;
        while ((len = getline(&line, &cap, f)) >= 0) {
            char **tok;
            int nt = tokenize(line, ",", &tok);
            if (nt >= 2 && strlen(tok[0]) >= 2 && strlen(tok[1]) >= 2) {
                int v1 = atoi(tok[0] + 2) - 1, v2 = atoi(tok[1] + 2) - 1;
                if (v1 >= 0 && v2 >= 0 && v1 < max_n && v2 < max_n) {
                    edges[v1] |= 1ULL << v2; edges[v2] |= 1ULL << v1;
                }
            }
            free_tokens(tok);
        }
    } else {
        int row = 0;
        while ((len = getline(&line, &cap, f)) >= 0) {
            /* boost::char_separator(", \n\r"): empty tokens dropped */
            int col = 0;
            char *save = NULL;
            for (char *t = strtok_r(line, ", \n\r", &save); t; t = strtok_r(NULL, ", \n\r", &save)) {
                if (strcmp(t, "TRUE") == 0 || fabs(atof(t)) > 0.05) {
                    if (row < max_n && col < 64) edges[row] |= 1ULL << col;
                    if (col < max_n && row < 64) edges[col] |= 1ULL << row;
                }
                col++;
            }
            if (row == 0) nv = col;
            row++;
        }
    }
    free(line);
    fclose(f);
    return nv;
}
