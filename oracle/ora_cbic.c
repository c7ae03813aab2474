/* ora_cbic.c -- TEST INFRASTRUCTURE ONLY (see ora.h).
 *
 * Plain-C restatement of the reference's continuous-BIC scoring path:
 *   BIC_OLS_Function ctor         urlearning/scoring_function/BIC_OLS.cpp:30-123
 *   find_best_subset_score        BIC_OLS.cpp:125-172
 *   calculateScore                BIC_OLS.cpp:174-276
 *   calculateScoreAndBeta         BIC_OLS.cpp:277-389 (+ mlpack 3.x
 *                                 LinearRegression(X,Y,0,false): normal
 *                                 equations, ComputeError = |Y-b'X|^2/N)
 *   calculateScores_internal      score_calculator.cpp:54-135
 *   scoringThread striping        score/score_main.cpp:132-207
 *   RecordFile / Variable arity   base/record_file.h:39-54, variable.h:58-64
 * The per-set OLS deliberately works over all N rows like mlpack does, so
 * the timed CPU baseline keeps the reference's cost profile.
 */
#define _GNU_SOURCE
#include "ora.h"
#include "ora_internal.h"

#include <ctype.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct ora_dataset {
    int64_t N;
    int n;
    double *raw;  /* column-major N x n, as loaded */
    double *norm; /* column-major N x n, normalised */
};

/* ---- Armadillo-style mean / var (arma op_mean / op_var direct forms) ---- */
static double arma_mean(const double *x, int64_t N) {
    double a1 = 0.0, a2 = 0.0;
    int64_t i, j;
    for (i = 0, j = 1; j < N; i += 2, j += 2) { a1 += x[i]; a2 += x[j]; }
    if (i < N) a1 += x[i];
    return (a1 + a2) / (double)N;
}
static double arma_var(const double *x, int64_t N) {
    if (N < 2) return 0.0;
    double m = arma_mean(x, N);
    double acc2 = 0.0, acc3 = 0.0;
    for (int64_t i = 0; i < N; i++) { double t = m - x[i]; acc2 += t * t; acc3 += t; }
    return (acc2 - acc3 * acc3 / (double)N) / (double)(N - 1);
}

/* BIC_OLS.cpp:66-97: centre each column, divide by the sample std of the
 * centred column. */
static void normalise(ora_dataset *ds) {
    for (int c = 0; c < ds->n; c++) {
        const double *x = ds->raw + (int64_t)c * ds->N;
        double *z = ds->norm + (int64_t)c * ds->N;
        double mean = arma_mean(x, ds->N);
        double *tmp = (double *)malloc(sizeof(double) * (size_t)ds->N);
        for (int64_t j = 0; j < ds->N; j++) tmp[j] = x[j] - mean;
        double dev = sqrt(arma_var(tmp, ds->N));
        for (int64_t j = 0; j < ds->N; j++) z[j] = (x[j] - mean) / dev;
        free(tmp);
    }
}

ora_dataset *ora_dataset_from_colmajor(const double *x, int64_t N, int n) {
    ora_dataset *ds = (ora_dataset *)calloc(1, sizeof(*ds));
    ds->N = N; ds->n = n;
    ds->raw = (double *)malloc(sizeof(double) * (size_t)(N * n));
    ds->norm = (double *)malloc(sizeof(double) * (size_t)(N * n));
    memcpy(ds->raw, x, sizeof(double) * (size_t)(N * n));
    normalise(ds);
    return ds;
}

/* Armadillo csv_ascii semantics (via mlpack::data::Load(file, m, true,
 * false), BIC_OLS.cpp:48): n_rows = number of lines, n_cols = max tokens
 * per line, matrix zero-filled, tokens converted with strtod; a token that
 * does not convert stays 0. */
ora_dataset *ora_dataset_from_csv(const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) return NULL;
    char *line = NULL;
    size_t lcap = 0;
    ssize_t len;
    int64_t rows = 0;
    int cols = 0;
    while ((len = getline(&line, &lcap, f)) >= 0) {
        int t = 1;
        for (ssize_t i = 0; i < len; i++) if (line[i] == ',') t++;
        if (t > cols) cols = t;
        rows++;
    }
    if (rows == 0 || cols == 0) { free(line); fclose(f); return NULL; }
    double *x = (double *)calloc((size_t)(rows * cols), sizeof(double));
    rewind(f);
    int64_t r = 0;
    while ((len = getline(&line, &lcap, f)) >= 0 && r < rows) {
        if (len > 0 && line[len - 1] == '\n') line[--len] = 0;
        if (len > 0 && line[len - 1] == '\r') line[--len] = 0;
        char *p = line;
        int c = 0;
        for (;;) {
            char *comma = strchr(p, ',');
            if (comma) *comma = 0;
            char *end = NULL;
            double v = strtod(p, &end);
            if (end != p) x[(int64_t)c * rows + r] = v;
            c++;
            if (!comma) break;
            p = comma + 1;
        }
        r++;
    }
    free(line);
    fclose(f);
    ora_dataset *ds = ora_dataset_from_colmajor(x, rows, cols);
    free(x);
    return ds;
}

void ora_dataset_free(ora_dataset *ds) {
    if (!ds) return;
    free(ds->raw); free(ds->norm); free(ds);
}
int ora_dataset_n(const ora_dataset *ds) { return ds->n; }
int64_t ora_dataset_N(const ora_dataset *ds) { return ds->N; }
const double *ora_dataset_norm(const ora_dataset *ds) { return ds->norm; }

/* ---- RecordFile token statistics -------------------------------------- */
static char *trim(char *s) {
    while (*s && isspace((unsigned char)*s)) s++;
    size_t l = strlen(s);
    while (l > 0 && isspace((unsigned char)s[l - 1])) s[--l] = 0;
    return s;
}
/* boost::split(..., is_any_of(delim), token_compress_on) */
static int split_compress(char *s, char delim, char **tok, int max_tok) {
    int nt = 0;
    char *p = s;
    tok[nt++] = p;
    for (; *p; p++) {
        if (*p == delim) {
            *p = 0;
            while (p[1] == delim) p++;
            if (nt < max_tok) tok[nt++] = p + 1;
        }
    }
    return nt;
}
static uint64_t fnv1a(const char *s) {
    uint64_t h = 1469598103934665603ULL;
    for (; *s; s++) { h ^= (unsigned char)*s; h *= 1099511628211ULL; }
    return h;
}

int ora_record_stats(const char *path, char delim, int has_header,
                     int64_t *num_records, int *arity_out, int max_cols,
                     char *names_out, int name_stride) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char *line = NULL;
    size_t lcap = 0;
    char *tok[4096];
    int ncols = -1;
    int64_t nrec = 0;
    omap *seen = (omap *)calloc((size_t)max_cols, sizeof(omap));
    for (int c = 0; c < max_cols; c++) omap_init(&seen[c], 64);
    int first = 1;
    while (getline(&line, &lcap, f) >= 0) {
        char *s = trim(line);
        int nt = split_compress(s, delim, tok, 4096);
        if (first && has_header) {
            for (int c = 0; c < nt && c < max_cols; c++)
                snprintf(names_out + (size_t)c * name_stride, (size_t)name_stride, "%s", tok[c]);
            first = 0;
            continue;
        }
        if (ncols < 0) ncols = nt;
        first = 0;
        for (int c = 0; c < nt && c < max_cols; c++) omap_put(&seen[c], fnv1a(tok[c]), 1);
        nrec++;
    }
    free(line);
    fclose(f);
    if (ncols < 0) ncols = 0;
    for (int c = 0; c < ncols && c < max_cols; c++) {
        arity_out[c] = (int)seen[c].size;
        if (!has_header)
            snprintf(names_out + (size_t)c * name_stride, (size_t)name_stride, "Variable_%d", c);
    }
    for (int c = 0; c < max_cols; c++) omap_free(&seen[c]);
    free(seen);
    *num_records = nrec;
    return ncols;
}

/* ---- calculateScoreAndBeta (BIC_OLS.cpp:277-389) ----------------------- */

/* LU with partial pivoting (LAPACK gesv order), solves A x = b in place. */
static int lu_solve(double *A, double *b, int k) {
    for (int c = 0; c < k; c++) {
        int piv = c;
        double mx = fabs(A[c * k + c]);
        for (int r = c + 1; r < k; r++)
            if (fabs(A[r * k + c]) > mx) { mx = fabs(A[r * k + c]); piv = r; }
        if (mx == 0.0) return -1;
        if (piv != c) {
            for (int j = 0; j < k; j++) { double t = A[c * k + j]; A[c * k + j] = A[piv * k + j]; A[piv * k + j] = t; }
            double t = b[c]; b[c] = b[piv]; b[piv] = t;
        }
        for (int r = c + 1; r < k; r++) {
            double l = A[r * k + c] / A[c * k + c];
            A[r * k + c] = l;
            for (int j = c + 1; j < k; j++) A[r * k + j] -= l * A[c * k + j];
            b[r] -= l * b[c];
        }
    }
    for (int r = k - 1; r >= 0; r--) {
        double s = b[r];
        for (int j = r + 1; j < k; j++) s -= A[r * k + j] * b[j];
        b[r] = s / A[r * k + r];
    }
    return 0;
}

typedef struct {
    double *X;   /* k x N copy of parent columns (arma trans(norm.cols(pv))) */
    double *Y;   /* N copy of the child column */
    double *tmp; /* N */
    int64_t cap_rows;
    int cap_k;
} ols_ws;

static void ws_reserve(ols_ws *w, int64_t N, int k) {
    if (w->cap_rows < N || w->cap_k < k) {
        free(w->X); free(w->Y); free(w->tmp);
        w->cap_rows = N; w->cap_k = k > w->cap_k ? k : w->cap_k;
        if (w->cap_k < 8) w->cap_k = 8;
        w->X = (double *)malloc(sizeof(double) * (size_t)(N * w->cap_k));
        w->Y = (double *)malloc(sizeof(double) * (size_t)N);
        w->tmp = (double *)malloc(sizeof(double) * (size_t)N);
    }
}

static float cbic_raw_ws(const ora_dataset *ds, double lambda, int v,
                         const int *pv, int k, ols_ws *w) {
    const int64_t N = ds->N;
    if (k == 0) return 0.0f; /* BIC_OLS.cpp:302-305 */
    ws_reserve(w, N, k);
    /* arma::rowvec Y = trans(norm_data.col(variable)); X = trans(norm.cols) */
    memcpy(w->Y, ds->norm + (int64_t)v * N, sizeof(double) * (size_t)N);
    for (int a = 0; a < k; a++)
        memcpy(w->X + (int64_t)a * N, ds->norm + (int64_t)pv[a] * N, sizeof(double) * (size_t)N);
    /* double varY = sqrt(var(Y)) (BIC_OLS.cpp:309; value unused) */
    volatile double varY = sqrt(arma_var(w->Y, N));
    (void)varY;
    /* LinearRegression::Train: cov = X X^T (+0*I), rhs = X Y^T, solve */
    double cov[64 * 64], rhs[64];
    for (int a = 0; a < k; a++) {
        const double *xa = w->X + (int64_t)a * N;
        for (int b = 0; b < k; b++) {
            const double *xb = w->X + (int64_t)b * N;
            double s = 0.0;
            for (int64_t j = 0; j < N; j++) s += xa[j] * xb[j];
            cov[a * k + b] = s;
        }
        double s = 0.0;
        for (int64_t j = 0; j < N; j++) s += xa[j] * w->Y[j];
        rhs[a] = s;
    }
    if (lu_solve(cov, rhs, k) != 0) {
        /* singular normal equations: arma::solve would fail; report +inf */
        return INFINITY;
    }
    /* ComputeError: temp = Y - beta' X ; dot(temp,temp)/N */
    double err = 0.0;
    for (int64_t j = 0; j < N; j++) w->tmp[j] = 0.0;
    for (int a = 0; a < k; a++) {
        const double *xa = w->X + (int64_t)a * N;
        const double ba = rhs[a];
        for (int64_t j = 0; j < N; j++) w->tmp[j] += ba * xa[j];
    }
    for (int64_t j = 0; j < N; j++) { double t = w->Y[j] - w->tmp[j]; err += t * t; }
    double error_L2 = err / (double)N;
    /* Yhat = beta' X; error = Yhat - Y; sum_error_sq (BIC_OLS.cpp:345-350,
     * computed by the reference and unused) */
    volatile double sum_error_sq = 0.0;
    {
        double s = 0.0;
        for (int64_t j = 0; j < N; j++) {
            double yh = 0.0;
            for (int a = 0; a < k; a++) yh += rhs[a] * w->X[(int64_t)a * N + j];
            double e = yh - w->Y[j];
            s += e * e;
        }
        sum_error_sq = s;
    }
    (void)sum_error_sq;
    /* BIC_OLS.cpp:366: num_err*log(error_L2) + lambda*log(num_err)*num_parents - raw_data_bic(=0) */
    const int num_err = (int)N;
    double the_score = num_err * log(error_L2) + lambda * log((double)num_err) * k - 0.0;
    return (float)the_score;
}

static int parent_vec(int n, int v, vs_t P, int *pv) {
    int np = 0;
    for (int i = 0; i < n; i++)
        if (i != v && ((P >> i) & 1ULL)) pv[np++] = i;
    return np;
}

float ora_cbic_raw(const ora_dataset *ds, double lambda, int v, ora_varset parents) {
    int pv[64] = {0};
    int k = parent_vec(ds->n, v, parents, pv);
    ols_ws w = {0};
    float s = cbic_raw_ws(ds, lambda, v, pv, k, &w);
    free(w.X); free(w.Y); free(w.tmp);
    return s;
}

/* ---- find_best_subset_score (BIC_OLS.cpp:125-172) ---------------------- */
/* Exact restatement, including the partially filled new_parent_vec that is
 * passed down with num_parents-1 entries (entries past j are zero: pinned
 * Armadillo >= 10.5 zero-initialisation) and VARSET_CLEAR being
 * an XOR toggle (typedefs.h:657). */
static float fbss(vs_t parents, const omap *cache, const int *pv, int m, omap *checked) {
    float best = 0.0f;
    for (int idx = 0; idx < m; idx++) {
        const int u = pv[idx];
        const vs_t thin = parents ^ (1ULL << u);
        if (omap_get(checked, thin, NULL)) continue;
        uint64_t bits;
        if (omap_get(cache, thin, &bits)) {
            float val = u2f(bits);
            if (val > best) best = val;
        } else {
            int npv[64];
            memset(npv, 0, sizeof(int) * (size_t)(m > 1 ? m - 1 : 1));
            int j = 0;
            for (int i = 0; i < m; i++) {
                if (u == pv[i]) continue;
                npv[j++] = pv[i];
                float s = fbss(thin, cache, npv, m - 1, checked);
                omap_put(checked, thin, 1);
                if (s > best) best = s;
            }
        }
    }
    return best;
}

/* fbss over a cache of a finished run, seen as it stood when P (|P| = L) was
 * scored under the two-phase layer order: every stored set of a
 * smaller layer, plus -- when P lacks variable 0 -- the same layer's sets that
 * contain variable 0. */
static int cache_at(const omap *cache, vs_t K, int L, int p_has0, float *val) {
    uint64_t bits;
    if (!omap_get(cache, K, &bits)) return 0;
    const int pc = popc64(K);
    if (pc > L || (pc == L && (p_has0 || !(K & 1ULL)))) return 0;
    *val = u2f(bits);
    return 1;
}

static float fbss_at(vs_t parents, const omap *cache, int L, int p_has0, const int *pv, int m, omap *checked) {
    float best = 0.0f;
    for (int idx = 0; idx < m; idx++) {
        const int u = pv[idx];
        const vs_t thin = parents ^ (1ULL << u);
        if (omap_get(checked, thin, NULL)) continue;
        float val;
        if (cache_at(cache, thin, L, p_has0, &val)) {
            if (val > best) best = val;
        } else {
            int npv[64];
            memset(npv, 0, sizeof(int) * (size_t)(m > 1 ? m - 1 : 1));
            int j = 0;
            for (int i = 0; i < m; i++) {
                if (u == pv[i]) continue;
                npv[j++] = pv[i];
                float s = fbss_at(thin, cache, L, p_has0, npv, m - 1, checked);
                omap_put(checked, thin, 1);
                if (s > best) best = s;
            }
        }
    }
    return best;
}

ora_cache *ora_cache_create(const ora_varset *sets, const float *scores, int64_t count) {
    omap *m = (omap *)malloc(sizeof(omap));
    omap_init(m, (size_t)(count > 16 ? count : 16));
    for (int64_t i = 0; i < count; i++) omap_put(m, sets[i], f2u(scores[i]));
    return (ora_cache *)m;
}

void ora_cache_free(ora_cache *c) {
    omap_free((omap *)c);
    free(c);
}

int ora_decide(const ora_dataset *ds, double lambda, int v, ora_varset P, const ora_cache *cache, float *value) {
    int pv[64] = {0};
    const int np = parent_vec(ds->n, v, P, pv);
    ols_ws w = {0};
    const float the_score = cbic_raw_ws(ds, lambda, v, pv, np, &w);
    free(w.X); free(w.Y); free(w.tmp);
    *value = -the_score;
    if (np == 0) return 1;                       /* cache[empty] = -0.0f */
    if (the_score >= 0.0f) return -the_score < 0.0f;  /* stored by the caller iff < 0 */
    omap checked;
    omap_init(&checked, 64);
    omap_put(&checked, 0ULL, 1);
    const float best = fbss_at(P, (const omap *)cache, popc64(P), (int)(P & 1ULL), pv, np, &checked);
    omap_free(&checked);
    return !((double)best + 0.0 >= (double)(-the_score));
}

/* ---- calculateScore (BIC_OLS.cpp:174-276) ------------------------------ */
static float calculate_score(const ora_dataset *ds, double lambda, int v, vs_t P,
                             omap *cache, omap *checked, ols_ws *w) {
    int pv[64] = {0};
    const int np = parent_vec(ds->n, v, P, pv);
    const double bic_threshold = 0.0;
    float the_score = cbic_raw_ws(ds, lambda, v, pv, np, w);
    if (np > 0 && the_score >= bic_threshold) return -the_score;
    omap_clear(checked);
    omap_put(checked, 0ULL, 1); /* checked.insert(empty_set) */
    float best = fbss(P, cache, pv, np, checked);
    if (np > 0 && (double)best + bic_threshold >= (double)(-the_score)) return -the_score;
    omap_put(cache, P, f2u(-the_score));
    return -the_score;
}

/* typedefs.h:692-697 */
static inline vs_t next_permutation(vs_t vs) {
    vs_t temp = (vs | (vs - 1)) + 1;
    return temp | ((((temp & (0 - temp)) / (vs & (0 - vs))) >> 1) - 1);
}

typedef struct { vs_t set; float score; } entry_t;
static int cmp_entry(const void *a, const void *b) {
    const entry_t *x = (const entry_t *)a, *y = (const entry_t *)b;
    int px = popc64(x->set), py = popc64(y->set);
    if (px != py) return px < py ? -1 : 1;
    if (x->set != y->set) return x->set < y->set ? -1 : 1;
    return 0;
}

/* calculateScores_internal (score_calculator.cpp:54-135) */
static int64_t score_variable_ws(const ora_dataset *ds, double lambda, int v,
                                 vs_t candidates, int max_parents,
                                 ora_varset *sets, float *scores, int64_t cap,
                                 ols_ws *w, int sched, double frac, int64_t *nscored) {
    const int n = ds->n;
    omap cache, checked;
    omap_init(&cache, 1024);
    omap_init(&checked, 256);
    /* empty set first; stored because score (-0.0f) < 1 (:56-61) */
    float sc = calculate_score(ds, lambda, v, 0ULL, &cache, &checked, w);
    if (sc < 1) omap_put(&cache, 0ULL, f2u(sc));
    if (nscored) (*nscored)++;
    int nbr[64];
    int nn = 0;
    for (int i = 0; i < n; i++)
        if ((candidates >> i) & 1ULL) nbr[nn++] = i;
    for (int layer = 1; layer <= max_parents; layer++) {
        vs_t compact = 0;
        for (int i = 0; i < layer; i++) compact |= 1ULL << i;
        const vs_t max = (nn >= 64) ? ~0ULL : (1ULL << nn);
        /* bounded-sample timing mode (bench.py cpu_baseline): only the first
         * ceil(frac * |layer|) sets of each layer in Gosper order */
        int64_t budget = INT64_MAX;
        if (frac < 1.0) {
            double c = 1.0;
            const int m = nn - (int)((candidates >> v) & 1ULL);
            for (int i = 1; i <= layer; i++) c = c * (double)(m - layer + i) / (double)i;
            budget = (int64_t)ceil(frac * c);
        }
        if (sched == 0) {
            while (compact < max && budget > 0) {
                vs_t vars = 0;
                for (int i = 0; i < nn; i++)
                    if ((compact >> i) & 1ULL) vars |= 1ULL << nbr[i];
                if (!((vars >> v) & 1ULL)) {
                    float s = calculate_score(ds, lambda, v, vars, &cache, &checked, w);
                    if (s < 0) omap_put(&cache, vars, f2u(s));
                    if (nscored) (*nscored)++;
                    budget--;
                }
                compact = next_permutation(compact);
                if (compact == 0) break;
            }
        } else {
            /* Validation schedule for the GPU's two-launch layers:
             * sets containing variable 0 first, then the rest, each phase in
             * REVERSE Gosper order. */
            int64_t cnt = 0, capl = 1024;
            vs_t *lay = (vs_t *)malloc(sizeof(vs_t) * (size_t)capl);
            while (compact < max) {
                vs_t vars = 0;
                for (int i = 0; i < nn; i++)
                    if ((compact >> i) & 1ULL) vars |= 1ULL << nbr[i];
                if (!((vars >> v) & 1ULL)) {
                    if (cnt == capl) { capl *= 2; lay = (vs_t *)realloc(lay, sizeof(vs_t) * (size_t)capl); }
                    lay[cnt++] = vars;
                }
                compact = next_permutation(compact);
                if (compact == 0) break;
            }
            for (int phase = 0; phase < 2; phase++)
                for (int64_t i = cnt - 1; i >= 0; i--) {
                    const int has0 = (int)(lay[i] & 1ULL);
                    if ((phase == 0) != has0) continue;
                    float s = calculate_score(ds, lambda, v, lay[i], &cache, &checked, w);
                    if (s < 0) omap_put(&cache, lay[i], f2u(s));
                }
            free(lay);
        }
    }
    /* output sorted by (|set|, set) == the reference's insertion order */
    int64_t cnt = (int64_t)cache.size;
    int64_t ret = cnt;
    if (cnt > cap) ret = -1;
    else {
        entry_t *e = (entry_t *)malloc(sizeof(entry_t) * (size_t)(cnt ? cnt : 1));
        int64_t t = 0;
        for (size_t i = 0; i < cache.cap; i++)
            if (cache.used[i]) { e[t].set = cache.keys[i]; e[t].score = u2f(cache.vals[i]); t++; }
        qsort(e, (size_t)cnt, sizeof(entry_t), cmp_entry);
        for (int64_t i = 0; i < cnt; i++) { sets[i] = e[i].set; scores[i] = e[i].score; }
        free(e);
    }
    omap_free(&cache);
    omap_free(&checked);
    return ret;
}

int64_t ora_score_variable(const ora_dataset *ds, double lambda, int v,
                           ora_varset candidates, int max_parents,
                           ora_varset *sets, float *scores, int64_t cap) {
    ols_ws w = {0};
    int64_t r = score_variable_ws(ds, lambda, v, candidates, max_parents, sets, scores, cap, &w, 0, 1.0, NULL);
    free(w.X); free(w.Y); free(w.tmp);
    return r;
}

ora_varset ora_candidates(const ora_varset *edges, int n, int v) {
    const vs_t all = (n >= 64) ? ~0ULL : ((1ULL << n) - 1ULL);
    if (!edges) return all;
    vs_t orig = edges[v], nb = orig;
    for (int j = 0; j < n; j++)
        if (((orig >> j) & 1ULL) && j != v) nb |= edges[j];
    return nb;
}

typedef struct {
    const ora_dataset *ds;
    double lambda;
    const ora_varset *cands;
    int max_parents, threads, tid;
    const int64_t *cap;
    const int64_t *base;
    ora_varset *sets;
    float *scores;
    int64_t *counts;
    int err;
    double frac;
    int64_t nscored;
    const int *vlist;
    int nvl;
} thr_arg;

static void *score_thread(void *p) {
    thr_arg *a = (thr_arg *)p;
    ols_ws w = {0};
    const int nl = a->vlist ? a->nvl : a->ds->n;
    for (int vi = 0; vi < nl; vi++) {
        const int v = a->vlist ? a->vlist[vi] : vi;
        if (vi % a->threads != a->tid) continue; /* score_main.cpp:136-139 */
        int64_t c = score_variable_ws(a->ds, a->lambda, v, a->cands[v], a->max_parents,
                                      a->sets + a->base[v], a->scores + a->base[v], a->cap[v], &w, 0, a->frac, &a->nscored);
        if (c < 0) a->err = 1;
        a->counts[v] = c;
    }
    free(w.X); free(w.Y); free(w.tmp);
    return NULL;
}

int ora_score_all(const ora_dataset *ds, double lambda,
                  const ora_varset *candidates, int max_parents, int threads,
                  const int64_t *cap_per_var, ora_varset *sets, float *scores,
                  int64_t *offsets) {
    const int n = ds->n;
    if (threads < 1) threads = 1;
    int64_t *base = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *counts = (int64_t *)calloc((size_t)n, sizeof(int64_t));
    base[0] = 0;
    for (int v = 0; v < n; v++) base[v + 1] = base[v] + cap_per_var[v];
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    thr_arg *args = (thr_arg *)calloc((size_t)threads, sizeof(thr_arg));
    for (int t = 0; t < threads; t++) {
        thr_arg a = {ds, lambda, candidates, max_parents, threads, t, cap_per_var, base, sets, scores, counts, 0, 1.0, 0, NULL, 0};
        args[t] = a;
        pthread_create(&th[t], NULL, score_thread, &args[t]);
    }
    int err = 0;
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); err |= args[t].err; }
    /* compact to contiguous per-variable ranges */
    int64_t off = 0;
    for (int v = 0; v < n; v++) {
        offsets[v] = off;
        if (counts[v] > 0 && base[v] != off) {
            memmove(sets + off, sets + base[v], sizeof(ora_varset) * (size_t)counts[v]);
            memmove(scores + off, scores + base[v], sizeof(float) * (size_t)counts[v]);
        }
        off += counts[v] > 0 ? counts[v] : 0;
    }
    offsets[n] = off;
    free(base); free(counts); free(th); free(args);
    return err ? -1 : 0;
}

/* score_main.cpp:191 writes "%f"; score_cache.cpp:151 reads
 * float score = -1 * atof(token). */
float ora_quantize_cost(float score) {
    char buf[128];
    snprintf(buf, sizeof buf, "%f", (double)score);
    float cost = -1 * atof(buf);
    return cost;
}

int64_t ora_score_variable_sched(const ora_dataset *ds, double lambda, int v,
                                 ora_varset candidates, int max_parents, int sched,
                                 ora_varset *sets, float *scores, int64_t cap) {
    ols_ws w = {0};
    int64_t r = score_variable_ws(ds, lambda, v, candidates, max_parents, sets, scores, cap, &w, sched, 1.0, NULL);
    free(w.X); free(w.Y); free(w.tmp);
    return r;
}

/* Bounded CPU-baseline sample: variables vlist[0..nvl) striped over T
 * threads, each layer truncated to its first ceil(frac * |layer|) sets in
 * Gosper order.  Returns the number of parent sets scored. */
int64_t ora_score_sample(const ora_dataset *ds, double lambda, const int *vlist, int nvl,
                         const ora_varset *candidates, int max_parents, double frac, int threads) {
    const int n = ds->n;
    if (threads < 1) threads = 1;
    int64_t *cap = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    int64_t *base = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t *counts = (int64_t *)calloc((size_t)n, sizeof(int64_t));
    base[0] = 0;
    for (int v = 0; v < n; v++) {
        const int m = popc64(candidates[v] & ~(1ULL << v));
        double c = 1.0, tot = 1.0;
        for (int L = 1; L <= max_parents && L <= m; L++) { c = c * (double)(m - L + 1) / (double)L; tot += ceil(frac * c); }
        cap[v] = (int64_t)tot + 1;
        base[v + 1] = base[v] + cap[v];
    }
    ora_varset *sets = (ora_varset *)malloc(sizeof(ora_varset) * (size_t)base[n]);
    float *scores = (float *)malloc(sizeof(float) * (size_t)base[n]);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    thr_arg *args = (thr_arg *)calloc((size_t)threads, sizeof(thr_arg));
    for (int t = 0; t < threads; t++) {
        thr_arg a = {ds, lambda, candidates, max_parents, threads, t, cap, base, sets, scores, counts, 0, frac, 0, vlist, nvl};
        args[t] = a;
        pthread_create(&th[t], NULL, score_thread, &args[t]);
    }
    int64_t tot = 0;
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); tot += args[t].nscored; }
    free(cap); free(base); free(counts); free(sets); free(scores); free(th); free(args);
    return tot;
}
