/*
 * ora.h -- CPU ORACLE for the cBIC-score + A* hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * algorithm (ninalu/urlearning-cpp) used as the parity checker for the HIP
 * path and as the timed CPU baseline ("kind": "port") in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product library (urlearning-cpp_amd/libulg.so) never links,
 * loads or calls anything in this directory.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to the reference's urlearning/ directory).  Parity pinning:
 *   - A* DAG outputs: pinned by triplet_data/Figure_{1,2}/astar_dag_*.csv
 *     (tests/test_oracle_golden.py runs CSV -> .pss -> A* -> DAG).
 *   - cBIC score values: no reference fixture holds them ("parity unpinned"
 *     for the absolute score values; see DESIGN.md section Oracle).
 *   - Pinned undefined behaviour of the reference (SURVEY.md 8a notes):
 *       N3: the partially-filled arma::uvec in find_best_subset_score is
 *           zero-initialised (Armadillo >= 10.5 behaviour).
 *       N6: the uninitialised optimal_parents VLA in astar() reads as 0.
 *       N7: SparseParentList ties are broken by (cost, file line order).
 */
#ifndef ULG_ORACLE_H
#define ULG_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint64_t ora_varset;
typedef struct ora_dataset ora_dataset;

/* ---- data (BIC_OLS.cpp:30-123, record_file.h:39-54, variable.h:58-64) -- */

/* Armadillo csv_ascii-like numeric load: rows = lines, cols = max tokens;
 * a token strtod cannot convert reads as 0 (a header row becomes a row of
 * zeros).  Returns NULL on I/O failure. */
ora_dataset *ora_dataset_from_csv(const char *path);
/* Build from a column-major N x n matrix (copied). */
ora_dataset *ora_dataset_from_colmajor(const double *x, int64_t N, int n);
void ora_dataset_free(ora_dataset *ds);
int ora_dataset_n(const ora_dataset *ds);
int64_t ora_dataset_N(const ora_dataset *ds);
/* normalised data, column-major N x n: (x - mean) / sqrt(var_{N-1}) */
const double *ora_dataset_norm(const ora_dataset *ds);

/* RecordFile-style token statistics: number of records and per-column
 * distinct-token counts ("META arity", score_main.cpp:178).  names_out
 * receives "Variable_i" or header tokens (bayesian_network.cpp:25-42).
 * Returns number of columns (first record's token count) or -1. */
int ora_record_stats(const char *path, char delim, int has_header,
                     int64_t *num_records, int *arity_out, int max_cols,
                     char *names_out, int name_stride);

/* ---- cBIC (BIC_OLS.cpp:174-389, score_calculator.cpp:54-135) ---------- */

/* calculateScoreAndBeta: float(N*ln(RSS/N) + lambda*ln(N)*k) with the OLS
 * solved per set over all N rows (normal equations, LU with partial
 * pivoting, explicit residual), k = |parents \ {v}|; 0 for k = 0. */
float ora_cbic_raw(const ora_dataset *ds, double lambda, int v,
                   ora_varset parents);

/* calculateScores_internal for one variable, sequential Gosper order with
 * the live cache (the reference's exact evaluation order).  Writes the
 * stored (set, score) pairs sorted by (|set|, set value) into sets/scores
 * (capacity cap) and returns the count, or -1 if cap is too small. */
int64_t ora_score_variable(const ora_dataset *ds, double lambda, int v,
                           ora_varset candidates, int max_parents,
                           ora_varset *sets, float *scores, int64_t cap);

/* Same, with an alternative evaluation schedule (sched = 1: per layer, sets
 * containing variable 0 first, then the rest, each phase in reverse Gosper
 * order) -- used to validate the GPU's two-launch layer schedule. */
int64_t ora_score_variable_sched(const ora_dataset *ds, double lambda, int v,
                                 ora_varset candidates, int max_parents, int sched,
                                 ora_varset *sets, float *scores, int64_t cap);

/* All variables, T threads striped by v % T (score_main.cpp:132-207).
 * candidates[v] is the candidate set of v (2-hop skeleton neighbourhood).
 * Output per variable v occupies [offsets[v], offsets[v+1]) of sets/scores;
 * per-variable capacity is cap_per_var[v] (host computes the bound
 * sum_{L<=k} C(m_v, L) + 1).  Returns 0 or -1. */
int ora_score_all(const ora_dataset *ds, double lambda,
                  const ora_varset *candidates, int max_parents, int threads,
                  const int64_t *cap_per_var, ora_varset *sets, float *scores,
                  int64_t *offsets);

/* Bounded CPU-baseline sample (bench.py): variables vlist striped over T
 * threads, each layer cut to its first ceil(frac*|layer|) Gosper sets.
 * Returns the number of parent sets scored. */
int64_t ora_score_sample(const ora_dataset *ds, double lambda, const int *vlist, int nvl,
                         const ora_varset *candidates, int max_parents, double frac, int threads);

/* 2-hop candidate set N(v) U N(N(v)) from skeleton rows
 * (score_main.cpp:146-153); edges==NULL means no skeleton (all bits). */
ora_varset ora_candidates(const ora_varset *edges, int n, int v);

/* ---- .pss text (score_main.cpp:173-203,383-400; score_cache.cpp:55-160) */

/* The "%f" write + atof read + (-1 *) round trip the A* input goes through:
 * returns float(-1 * atof(sprintf("%f", score))) using the C library. */
float ora_quantize_cost(float score);

/* ---- search (sparse_parent_list.cpp, static_pattern_database.cpp,
 *      priority_queue-inl.h, astar_main.cpp) ----------------------------- */

typedef struct ora_search ora_search;

/* Build the BestScore lists (list calculator, stable sort by cost with
 * file-order tie-break, pinned N7) from per-variable (set, cost) lists in
 * file order.  costs are A* costs (= -score after quantisation). */
ora_search *ora_search_create(int n, const int64_t *offsets,
                              const ora_varset *sets, const float *costs);
void ora_search_free(ora_search *s);
/* wall-clock budget of ora_astar / ora_astar_scc (the reference's -r
 * watchdog); 0 = none.  ora_search_out_of_time: the last search stopped on it */
void ora_search_set_time_limit(ora_search *s, double seconds);
int ora_search_out_of_time(const ora_search *s);
int64_t ora_search_last_open(const ora_search *s);
/* SparseParentList::getScore (sparse_parent_list.cpp:44-55): first entry
 * whose set is a subset of S; FLT_MAX if none.  *parents gets that set. */
float ora_bestscore(ora_search *s, int v, ora_varset S, ora_varset *parents);
/* Static PDB (static_pattern_database.cpp:82-134) over scc with pd_count
 * groups, ancestors as given. */
int ora_pdb_build(ora_search *s, int pd_count, ora_varset ancestors,
                  ora_varset scc);
/* StaticPatternDatabase::h (static_pattern_database.cpp:145-174). */
float ora_pdb_h(ora_search *s, ora_varset S, int *complete);
/* number of groups and group masks */
int ora_pdb_groups(ora_search *s, ora_varset *groups, int max_groups);
/* pattern-database value for group g, pattern R (R subset of group). */
float ora_pdb_value(ora_search *s, int g, ora_varset R);

/* astar() + run_astar_on_one_scc (astar_main.cpp:216-644), static PDB(pd_count)
 * over all variables, one A* per connected component of the skeleton
 * (edges==NULL: no skeleton, one component).  Outputs the final netFile.csv
 * parent matrix as vpar[v] (bit i = i -> v), the last component's total
 * ordering and goal cost, and expansions summed over components.  The
 * netFile text (astar_main.cpp:192-212) is written to net_text if non-NULL
 * (capacity net_cap).  Returns 0, or 1 if some component found no goal. */
/* One set's store decision under calculateScore (BIC_OLS.cpp:174-276) and
 * score_calculator.cpp:111-115, against the cache of a finished run as it
 * stood when the set was scored (SURVEY N4 two-phase order).  Returns 1 if P
 * is stored; *value = -ts.  Used to check a full-size GPU run set by set. */
typedef struct ora_cache ora_cache;
ora_cache *ora_cache_create(const ora_varset *sets, const float *scores, int64_t count);
void ora_cache_free(ora_cache *c);
int ora_decide(const ora_dataset *ds, double lambda, int v, ora_varset P, const ora_cache *cache, float *value);

/* MMPC skeleton with Fisher-z tests (ora_mmpc.c; parity unpinned: the
 * reference takes the skeleton from outside, README.md:16).  rows[i] bit j =
 * edge i-j (no diagonal).  max_cond < 0: no cap (24). */
int ora_mmpc(const ora_dataset *ds, double alpha, int max_cond, ora_varset *rows);
double ora_partial_z(const double *G, int n, double N, int X, int T, const int *S, int ns);
double ora_norm_quantile(double p);

/* get_dag_score (astar/calc_dag_score.cpp:10-119) over a parsed DAG file:
 * rows[v] (v < nrows <= variableCount) has bit i set iff |atof(token i)| >
 * 1e-5.  s == NULL means no readable score file (spgs all NULL): scores stay
 * 0 and only the edge count is computed.  Outputs the row-wise total, the
 * transposed ("alt") total, the undirected edge count and the two
 * "edges to remove" counts (bits differing from getParents()). */
void ora_dag_score(ora_search *s, int variableCount, int nrows, const ora_varset *rows, float *total,
                   float *alt, int *num_edges, int *remove, int *remove_alt);

int ora_astar(ora_search *s, const ora_varset *edges, int pd_count,
              ora_varset *vpar, int *order, float *goal_cost,
              int64_t *expanded, char *net_text, int64_t net_cap);
int ora_astar_scc(ora_search *s, const ora_varset *edges, int pd_count, ora_varset ancestors, ora_varset scc,
                  ora_varset *vpar, int *order, float *goal_cost,
                  int64_t *expanded, char *net_text, int64_t net_cap);

/* triplet_astar's astar() (astar/triplet_astar.cpp:991-1622): A* (with
 * closed-node re-opening and a PDB per cluster) on every triple's cluster,
 * v-structure / unfaithful-edge bookkeeping, Meek rules 2-4.  directed_graph
 * (n*n, row-major) receives netFile.csv: (i,j)=1 means i -> j, both set =
 * undirected.  edges == NULL means no skeleton (every variable a neighbour
 * of every variable, itself included).  A* results are memoised per cluster
 * (deterministic); astar_runs counts the reference's calls. */
int ora_triplet_astar(ora_search *s, const ora_varset *edges, int pd_count, int *directed_graph,
                      int64_t *astar_runs, int64_t *distinct_runs, int64_t *expanded);

#ifdef __cplusplus
}
#endif
#endif
