/* ora_cli.c -- TEST INFRASTRUCTURE ONLY (see ora.h).
 *
 * CPU-oracle command lines mirroring the reference CLIs for the hot path:
 *   ref_score  <in.csv> <out.pss> -f cBIC --lambda L [-k skel] [-p k] [-t T] [-s] [-d ,]
 *              (score/score_main.cpp:209-403)
 *   ref_astar  <in.pss> [-k skel] [-n netFile] [-a pdCount]
 *              (astar/astar_main.cpp:548-709; post-processing skipped, N8)
 *   ref_triplet <in.pss> [-k skel] [-n netFile] [-a pdCount]
 *              (astar/triplet_astar.cpp:991-1687)
 *   ref_calc_dag_score <in.pss> <dag.csv>...
 *              (astar/calc_dag_score.cpp:10-176)
 * Built once per command from this file (-DORA_SCORE / -DORA_ASTAR / ...).
 */
#define _GNU_SOURCE
#include "ora.h"
#include "ora_io.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static const char *opt_val(int argc, char **argv, int *i) {
    char *a = argv[*i];
    char *eq = strchr(a, '=');
    if (eq && a[0] == '-' && a[1] == '-') return eq + 1;
    if (*i + 1 < argc) { (*i)++; return argv[*i]; }
    return NULL;
}

static int64_t binom(int m, int k) {
    if (k < 0 || k > m) return 0;
    int64_t r = 1;
    for (int i = 1; i <= k; i++) r = r * (m - k + i) / i;
    return r;
}

#ifdef ORA_SCORE
int main(int argc, char **argv) {
    const char *pos[2] = {NULL, NULL};
    int npos = 0;
    const char *skel = NULL, *sf = "BIC";
    double lambda = 0.5;
    int maxp = 0, threads = 1, has_header = 0;
    char delim = ',';
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (!strcmp(a, "-l") || !strncmp(a, "--lambda", 8)) lambda = atof(opt_val(argc, argv, &i));
        else if (!strcmp(a, "-k") || !strncmp(a, "--skeleton", 10)) skel = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-f") || !strncmp(a, "--function", 10)) sf = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-p") || !strncmp(a, "--maxParents", 12)) maxp = atoi(opt_val(argc, argv, &i));
        else if (!strcmp(a, "-t") || !strncmp(a, "--threads", 9)) threads = atoi(opt_val(argc, argv, &i));
        else if (!strcmp(a, "-d") || !strncmp(a, "--delimiter", 11)) delim = opt_val(argc, argv, &i)[0];
        else if (!strcmp(a, "-s") || !strcmp(a, "--hasHeader")) has_header = 1;
        else if (!strcmp(a, "-r") || !strncmp(a, "--time", 6)) (void)opt_val(argc, argv, &i);
        else if (a[0] == '-' && a[1]) { fprintf(stderr, "ref_score: option %s ignored\n", a); }
        else if (npos < 2) pos[npos++] = a;
    }
    if (npos < 2) { fprintf(stderr, "usage: ref_score in.csv out.pss -f cBIC --lambda L [-k skel] [-p k] [-t T]\n"); return 2; }
    char sfl[64];
    snprintf(sfl, sizeof sfl, "%s", sf);
    for (char *c = sfl; *c; c++) *c = (char)tolower((unsigned char)*c);
    if (strcmp(sfl, "cbic") != 0) { fprintf(stderr, "ref_score: only -f cBIC is on the hot path\n"); return 2; }
    if (threads < 1) threads = 1;
    int64_t nrec = 0;
    int arity[64];
    char names[64 * 256];
    int n = ora_record_stats(pos[0], delim, has_header, &nrec, arity, 64, names, 256);
    if (n <= 0 || n > 63) { fprintf(stderr, "ref_score: cannot read %s (n=%d)\n", pos[0], n); return 1; }
    ora_dataset *ds = ora_dataset_from_csv(pos[0]);
    if (!ds) { fprintf(stderr, "ref_score: cannot load %s\n", pos[0]); return 1; }
    if (maxp > n || maxp < 1) maxp = n - 1; /* score_main.cpp:296-298 */
    ora_varset edges[64];
    ora_varset cands[64];
    int have_skel = 0;
    if (skel && *skel) {
        int nv = ora_skeleton_read(skel, n, edges, 64);
        if (nv >= 0) have_skel = 1;
        else for (int v = 0; v < 64; v++) edges[v] = 1; /* default Skeleton(1): all_bit_set = {0} */
        if (nv < 0) have_skel = 1;
    }
    for (int v = 0; v < n; v++) cands[v] = ora_candidates(have_skel ? edges : NULL, n, v);
    int64_t caps[64];
    int64_t total = 0;
    for (int v = 0; v < n; v++) {
        int m = __builtin_popcountll(cands[v] & ~(1ULL << v));
        int64_t c = 1;
        for (int L = 1; L <= maxp; L++) c += binom(m, L);
        caps[v] = c; total += c;
    }
    ora_varset *sets = (ora_varset *)malloc(sizeof(ora_varset) * (size_t)total);
    float *scores = (float *)malloc(sizeof(float) * (size_t)total);
    int64_t offsets[65];
    double t0 = now_s();
    if (ora_score_all(ds, lambda, cands, maxp, threads, caps, sets, scores, offsets) != 0) {
        fprintf(stderr, "ref_score: scoring failed\n"); return 1;
    }
    double t1 = now_s();
    int64_t scored = 0;
    for (int v = 0; v < n; v++) {
        int m = __builtin_popcountll(cands[v] & ~(1ULL << v));
        for (int L = 0; L <= maxp; L++) scored += binom(m, L);
    }
    printf("ref_score: n=%d N=%lld k=%d threads=%d sets_scored=%lld stored=%lld time=%.3fs rate=%.1f sets/s\n",
           n, (long long)ora_dataset_N(ds), maxp, threads, (long long)scored, (long long)offsets[n],
           t1 - t0, (double)scored / (t1 - t0));
    if (ora_pss_write(pos[1], n, names, 256, arity, offsets, sets, scores, pos[0], nrec, maxp, sfl) != 0) {
        fprintf(stderr, "ref_score: cannot write %s\n", pos[1]); return 1;
    }
    free(sets); free(scores);
    ora_dataset_free(ds);
    return 0;
}
#endif

#ifdef ORA_ASTAR
/* setFromCsv (typedefs.h:737-754): comma-separated variable indices */
static int set_from_csv(const char *csv, ora_varset *vs) {
    /* boost::split with token_compress_on: runs of ',' are one separator, a
       leading or trailing ',' leaves an empty token (which fails the check) */
    const char *p = csv;
    if (!*p) return 0;
    for (;;) {
        const char *q = strchr(p, ',');
        const size_t len = q ? (size_t)(q - p) : strlen(p);
        char tok[64];
        snprintf(tok, sizeof tok, "%.*s", (int)(len < 63 ? len : 63), p);
        const int var = atoi(tok);
        if ((var == 0 && tok[0] != '0') || var < 0 || var >= 64) return -1;
        *vs |= 1ULL << var;
        if (!q) break;
        while (*q == ',') q++;
        p = q;
    }
    return 0;
}

int main(int argc, char **argv) {
    const char *pss = NULL, *skel = "", *net = "", *anc_arg = "", *scc_arg = "";
    int pd = 2;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (!strcmp(a, "-k") || !strncmp(a, "--skeleton", 10)) skel = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-n") || !strncmp(a, "--netFile", 9)) net = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-a") || !strncmp(a, "--argument", 10)) pd = atoi(opt_val(argc, argv, &i));
        else if (!strcmp(a, "-p")) anc_arg = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-s")) scc_arg = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-i") || !strcmp(a, "-f") || !strcmp(a, "-l") || !strcmp(a, "-b") ||
                 !strcmp(a, "-e") || !strcmp(a, "-r") || !strcmp(a, "-w"))
            (void)opt_val(argc, argv, &i);
        else if (a[0] == '-' && a[1]) fprintf(stderr, "ref_astar: option %s ignored\n", a);
        else if (!pss) pss = a;
    }
    if (!pss) { fprintf(stderr, "usage: ref_astar in.pss [-k skel] [-n netFile] [-a 2] [-p anc] [-s scc]\n"); return 2; }
    ora_pss p;
    if (ora_pss_read(pss, &p) != 0) { fprintf(stderr, "ref_astar: cannot read %s\n", pss); return 1; }
    const int n = p.n;
    /* astar_main.cpp:590-598: no -s -> every variable, -p ignored */
    ora_varset ancestors = 0, scc = (n >= 64) ? ~0ULL : ((1ULL << n) - 1ULL);
    if (*scc_arg) {
        scc = 0;
        if (set_from_csv(scc_arg, &scc) || set_from_csv(anc_arg, &ancestors)) {
            fprintf(stderr, "ref_astar: Invalid csv string\n");
            return 1;
        }
    }
    ora_search *s = ora_search_create(n, p.offsets, p.sets, p.costs);
    ora_varset edges[64];
    int good = 0;
    if (skel && *skel) good = ora_skeleton_read(skel, n, edges, 64) >= 0;
    ora_varset vpar[64];
    int order[64];
    float cost = 0;
    int64_t expanded = 0;
    char *text = (char *)malloc(1 << 20);
    double t0 = now_s();
    int rc = ora_astar_scc(s, good ? edges : NULL, pd, ancestors, scc, vpar, order, &cost, &expanded, text, 1 << 20);
    double t1 = now_s();
    printf("Found solution: %f\nNodes expanded: %lld\nref_astar: time=%.6fs\n", (double)cost, (long long)expanded, t1 - t0);
    if (rc == 2) fprintf(stderr, "ref_astar: reference heap __down_heap would not terminate\n");
    if (net && *net) {
        FILE *f = fopen(net, "w");
        if (f) { fputs(text, f); fclose(f); }
        char csv[4096];
        snprintf(csv, sizeof csv, "%s.csv", net);
        f = fopen(csv, "w");
        if (f) {
            for (int v = 0; v < n; v++)
                for (int i = 0; i < n; i++) fprintf(f, "%d%c", ((vpar[v] >> i) & 1ULL) ? 1 : 0, i == n - 1 ? '\n' : ',');
            fclose(f);
        }
    }
    free(text);
    ora_search_free(s);
    ora_pss_free(&p);
    return rc == 0 ? 0 : 1;
}
#endif

#ifdef ORA_TRIPLET
/* ref_triplet <in.pss> [-k skeleton] [-n netFile] [-a pdCount]
 * (astar/triplet_astar.cpp:991-1687): netFile.csv = directed_graph. */
int main(int argc, char **argv) {
    const char *pss = NULL, *skel = "", *net = "";
    int pd = 2;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        if (!strcmp(a, "-k") || !strncmp(a, "--skeleton", 10)) skel = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-n") || !strncmp(a, "--netFile", 9)) net = opt_val(argc, argv, &i);
        else if (!strcmp(a, "-a") || !strncmp(a, "--argument", 10)) pd = atoi(opt_val(argc, argv, &i));
        else if (!strcmp(a, "-i") || !strcmp(a, "-f") || !strcmp(a, "-l") || !strcmp(a, "-b") ||
                 !strcmp(a, "-e") || !strcmp(a, "-r") || !strcmp(a, "-w") || !strcmp(a, "-p") || !strcmp(a, "-s"))
            (void)opt_val(argc, argv, &i);
        else if (a[0] == '-' && a[1]) fprintf(stderr, "ref_triplet: option %s ignored\n", a);
        else if (!pss) pss = a;
    }
    if (!pss) { fprintf(stderr, "usage: ref_triplet in.pss [-k skel] [-n netFile] [-a 2]\n"); return 2; }
    ora_pss p;
    if (ora_pss_read(pss, &p) != 0) { fprintf(stderr, "ref_triplet: cannot read %s\n", pss); return 1; }
    const int n = p.n;
    ora_search *s = ora_search_create(n, p.offsets, p.sets, p.costs);
    ora_varset edges[64];
    int good = 0;
    if (skel && *skel) good = ora_skeleton_read(skel, n, edges, 64) >= 0;
    int *dg = (int *)calloc((size_t)(n * n), sizeof(int));
    int64_t runs = 0, distinct = 0, expanded = 0;
    double t0 = now_s();
    int rc = ora_triplet_astar(s, good ? edges : NULL, pd, dg, &runs, &distinct, &expanded);
    double t1 = now_s();
    printf("ref_triplet: A* runs %lld (distinct clusters %lld), expanded %lld, time %.3fs\n", (long long)runs,
           (long long)distinct, (long long)expanded, t1 - t0);
    if (net && *net) {
        FILE *f = fopen(net, "w");
        if (f) fclose(f); /* the reference leaves netFile empty (post-processing commented out) */
        char csv[4096];
        snprintf(csv, sizeof csv, "%s.csv", net);
        f = fopen(csv, "w");
        if (f) {
            for (int i = 0; i < n; i++)
                for (int j = 0; j < n; j++) fprintf(f, "%d%c", dg[i * n + j], j == n - 1 ? '\n' : ',');
            fclose(f);
        }
    }
    free(dg);
    ora_search_free(s);
    ora_pss_free(&p);
    return rc == 0 ? 0 : 1;
}
#endif

#ifdef ORA_DAGSCORE
/* ref_calc_dag_score <in.pss> <dag.csv>... (astar/calc_dag_score.cpp:121-176):
 * one output line "NAME  score  edges E  [remove R ]..." for all DAGs. */
static int dag_tokens(const char *line, double *vals, int cap) {
    int n = 0;
    const char *p = line;
    while (*p) {
        while (*p && strchr(", \n\r", *p)) p++;
        if (!*p) break;
        const char *b = p;
        while (*p && !strchr(", \n\r", *p)) p++;
        char tok[256];
        size_t l = (size_t)(p - b) < sizeof tok - 1 ? (size_t)(p - b) : sizeof tok - 1;
        memcpy(tok, b, l);
        tok[l] = 0;
        if (n < cap) vals[n] = atof(tok);
        n++;
    }
    return n;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: ref_calc_dag_score in.pss dag.csv...\n"); return 2; }
    ora_pss p;
    ora_search *s = NULL;
    FILE *probe = fopen(argv[1], "r");
    if (probe) {
        fclose(probe);
        if (ora_pss_read(argv[1], &p) == 0) s = ora_search_create(p.n, p.offsets, p.sets, p.costs);
    }
    for (int m = 2; m < argc; m++) {
        /* model name: basename, cut at the first ".csv", upper case */
        const char *base = strrchr(argv[m], '/');
        base = base ? base + 1 : argv[m];
        char name[1024];
        snprintf(name, sizeof name, "%s", base);
        char *dot = strstr(name, ".csv");
        if (dot) *dot = 0;
        for (char *c = name; *c; c++) *c = (char)toupper((unsigned char)*c);
        float total = 0, alt = 0;
        int ne = 0, rm = 0, rma = 0;
        FILE *f = fopen(argv[m], "r");
        if (!f) {
            fprintf(stderr, "Invalid model file %s\n", argv[m]);
        } else {
            char *line = NULL;
            size_t cap = 0;
            ora_varset rows[64];
            double vals[64];
            int variableCount = 0, nrows = 0;
            if (getline(&line, &cap, f) >= 0) {
                variableCount = dag_tokens(line, vals, 64);
                do {
                    const int nt = dag_tokens(line, vals, 64);
                    ora_varset par = 0;
                    for (int i = 0; i < nt && i < 64; i++)
                        if (fabsf((float)vals[i]) > 1e-5f) par |= 1ULL << i;
                    rows[nrows++] = par;
                } while (getline(&line, &cap, f) >= 0 && nrows < variableCount && nrows < 64);
            }
            free(line);
            fclose(f);
            ora_dag_score(s, variableCount, nrows, rows, &total, &alt, &ne, &rm, &rma);
        }
        const float score = total > alt ? alt : total;
        const int to_remove = total > alt ? rm : rma;
        if (m == 2) printf("%s  %f  edges %d  ", name, (double)score, ne);
        else printf("%s  %f  edges %d remove %d ", name, (double)score, ne, to_remove);
    }
    printf("\n");
    if (s) { ora_search_free(s); ora_pss_free(&p); }
    return 0;
}
#endif
