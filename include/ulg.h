/*
 * ulg.h -- C ABI of the MI355X-native URLearning hot path (libulg.so).
 *
 * Drop-in boundary for the reference's plugin points on the
 * cBIC-score + order-graph-search path (ninalu/urlearning-cpp, paths
 * relative to urlearning/):
 *
 *   ulg_cbic_load        replaces BIC_OLS_Function::BIC_OLS_Function
 *                        (scoring_function/BIC_OLS.cpp:30-123): data load,
 *                        centring/scaling, Gram matrix (the reference's
 *                        printed corr_mat = Z'Z/N, :105).
 *   ulg_cbic_score       replaces ScoreCalculator::calculateScores
 *                        (scoring_function/score_calculator.h:35,
 *                        score_calculator.cpp:33-135) driving
 *                        ScoringFunction::calculateScore (scoring_function.h:16-23,
 *                        BIC_OLS.cpp:174-389) for a batch of variables; the
 *                        stored-set rule and the find_best_subset_score
 *                        dominance recursion are reproduced exactly.
 *   ulg_cbic_fetch       hands the stored FloatMap contents back (what
 *                        scoringThread prints, score/score_main.cpp:173-203).
 *   ulg_bestscore_*      replaces bestscorecalculators::BestScoreCalculator
 *                        (score_cache/best_score_calculator.h:16-26) with the
 *                        list calculator's semantics
 *                        (score_cache/sparse_parent_list.cpp:20-55).
 *   ulg_pdb_*            replaces heuristics::StaticPatternDatabase
 *                        (heuristic/static_pattern_database.cpp:82-247).
 *   ulg_astar            replaces run_astar_on_one_scc
 *                        (astar/astar_main.cpp:216-546).
 *   ulg_triplet_astar    replaces triplet_astar's astar() driver and its
 *                        re-opening run_astar_on_one_scc
 *                        (astar/triplet_astar.cpp:285-674,811-1622).
 *
 * Conventions (mirroring the reference's): the caller owns host buffers;
 * device memory is owned by the context; hot calls report errors by an int
 * status (0 = ok) and ulg_last_error(); one context per host thread and per
 * GPU (one process per GPU for multi-GPU runs).  varsets are uint64 bit
 * masks (bit i = variable i), as in typedefs.h:647-755.  Scores are the
 * .pss "score" (higher is better); costs are A* costs (= -score after the
 * .pss "%f" round trip, score_cache.cpp:151).
 */
#ifndef ULG_H
#define ULG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ulg_ctx ulg_ctx;

#define ULG_OK 0
#define ULG_ERR_ARG 1
#define ULG_ERR_HIP 2
#define ULG_ERR_STATE 3
#define ULG_ERR_UNSUPPORTED 4

/* Largest parent-set size the HIP scorer handles.  Layers up to
 * ULG_UNROLLED_PARENTS_GPU run fully unrolled kernels (register Cholesky,
 * bitset dominance walk); larger layers (the reference's default -p = n-1 on
 * small n, e.g. data/hepatitis.clean.csv) run the wide-layer kernels, whose
 * find_best_subset_score walk keeps a 2^(k+1)-bit checked set per set. */
#define ULG_MAX_PARENTS_GPU 31
#define ULG_UNROLLED_PARENTS_GPU 8

/* ---- context --------------------------------------------------------- */
/* One device per context: ndev must be 1 (multi-GPU = one process per GPU). */
int ulg_create(const int *device_ids, int ndev, ulg_ctx **out);
void ulg_destroy(ulg_ctx *ctx);
const char *ulg_last_error(const ulg_ctx *ctx);
/* Library build identifier ("gfx950 ..."). */
const char *ulg_version(void);

/* ---- cBIC scoring (BIC_OLS.cpp, score_calculator.cpp) ----------------- */
/* data_colmajor: N x n doubles, column-major (column j = variable j), as
 * Armadillo holds raw_data.  n <= 63.  Normalises each column to zero mean
 * and unit sample variance (N-1) and builds the FP64 Gram matrix Z'Z on the
 * device (MFMA f64). */
int ulg_cbic_load(ulg_ctx *ctx, const double *data_colmajor, int64_t N, int n,
                  double lambda);
/* Copy the device Gram matrix Z'Z (n x n, row-major) to host. */
int ulg_cbic_gram(ulg_ctx *ctx, double *gram_out);

/* The skeleton the reference expects from outside (README.md:16, read by
 * Skeleton::read_matrix_file, base/skeleton.cpp:19-105): MMPC with Fisher-z
 * partial-correlation tests on the loaded data's Gram matrix.  Independent
 * iff |atanh(r)| sqrt(N - |S| - 3) <= Phi^-1(1 - alpha/2); conditioning sets
 * of at most max_cond variables (< 0: 24); AND symmetry rule.  rows[i] bit j
 * = edge i-j (no diagonal).  Exact rules: oracle/ora_mmpc.c. */
int ulg_mmpc(ulg_ctx *ctx, double alpha, int max_cond, uint64_t *rows);

/* Score all parent sets of size <= max_parents within each variable's
 * candidate set (candidates[i] for variable vars[i]; the variable's own bit
 * is ignored).  max_parents < 1 or > n - 1 means n - 1, the reference's
 * "a value less than 1 means no limit" (score_main.cpp:228,296-298).  Runs the layer-synchronous HIP scorer; results stay on the
 * device until ulg_cbic_fetch.  *total_stored = number of stored sets,
 * *total_scored = number of parent sets evaluated (incl. empty sets). */
int ulg_cbic_score(ulg_ctx *ctx, const int *vars, int nv,
                   const uint64_t *candidates, int max_parents,
                   int64_t *total_stored, int64_t *total_scored);
/* The same call split in two, so one host thread can keep several contexts'
 * scoring in flight (e.g. two steps of a throughput loop on one GPU):
 * ulg_cbic_score_async queues the whole call and returns without waiting
 * (when every layer is unrolled and no time limit is set; otherwise it runs
 * synchronously), ulg_cbic_score_finish waits for it and returns the counts
 * ulg_cbic_score would have.  Any later scorer call on the context
 * (ulg_cbic_score*, ulg_cbic_fetch) finishes a pending one first. */
int ulg_cbic_score_async(ulg_ctx *ctx, const int *vars, int nv,
                         const uint64_t *candidates, int max_parents);
int ulg_cbic_score_finish(ulg_ctx *ctx, int64_t *total_stored, int64_t *total_scored);
/* Copy the stored sets out.  offsets[nv+1]; variable vars[i] owns
 * [offsets[i], offsets[i+1]); within a variable, sets are ordered by
 * (|set|, set value) -- the reference's Gosper insertion order.
 * device_ptrs = 1: sets/scores/offsets are device pointers (e.g. torch
 * tensors on this context's device); 0: host pointers.
 * Stream contract: the copies run on the context's own stream, and the call
 * is synchronous -- it returns after they are complete, with host or device
 * pointers alike, so the destination may be read on any stream afterwards.
 * The copies are NOT ordered after work another stream queued on the
 * destination (e.g. a torch zero fill on torch's current stream): the caller
 * must finish that work first, or record an event after it and pass it to
 * ulg_stream_wait_event before this call. */
int ulg_cbic_fetch(ulg_ctx *ctx, uint64_t *sets, float *scores,
                   int64_t *offsets, int device_ptrs);
/* The context's stream waits (on the device, no host sync) for a hipEvent_t
 * the caller recorded on another stream of the same device; every later
 * launch and copy of the context is ordered after it. */
int ulg_stream_wait_event(ulg_ctx *ctx, void *event);
/* Convenience: ulg_cbic_score + ulg_cbic_fetch to host buffers of
 * capacity cap entries; returns ULG_ERR_ARG if cap is too small. */
int ulg_cbic_score_vars(ulg_ctx *ctx, const int *vars, int nv,
                        const uint64_t *candidates, int max_parents,
                        uint64_t *sets, float *scores, int64_t *offsets,
                        int64_t cap);

/* Per-call counterpart of ScoringFunction::calculateScore(variable, parents,
 * cache) (scoring_function.h:16-23, BIC_OLS.cpp:174-276): for each pair
 * (vars[i], parents[i]) the value it returns, -float(the_score) with
 * the_score = N ln(RSS/N) + lambda ln(N) |P| (calculateScoreAndBeta,
 * BIC_OLS.cpp:277-388; no parents -> -0.0f), batched on the device from the
 * loaded Gram matrix with the layer scorer's Cholesky, so a stored set's value
 * equals what ulg_cbic_score stored for it.  The variable's own bit is
 * ignored (parent_vec skips it).  The cache insertion rule (store iff the
 * value is < 0 and no subset dominates) stays with ulg_cbic_score, which
 * applies it layer by layer.  At most 31 parents per set. */
int ulg_cbic_score_sets(ulg_ctx *ctx, int64_t count, const int *vars,
                        const uint64_t *parents, float *neg_scores);

/* The .pss "%f" + atof round trip the A* input goes through
 * (score_main.cpp:191, score_cache.cpp:151), computed exactly on the
 * device: cost = float(-1 * strtod(printf("%f", score))). */
int ulg_quantize_costs(ulg_ctx *ctx, const float *scores, float *costs,
                       int64_t count);

/* ---- the .pss score-cache text (score_main.cpp:173-203,383-400) -------- */
/* Formats the lists of the last ulg_cbic_score (every variable scored) as
 * the .pss file the reference's score command writes: `header` verbatim
 * (the META block and its blank line), then for each variable in index
 * order "VAR <name>", "META arity=<a>", one line per stored set -- the
 * score as glibc "%f" prints it, a space, each parent's name followed by a
 * space -- and a blank line.  The text is formatted on the GPU; *text points
 * to a context-owned host buffer of *len bytes (NUL-terminated), valid until
 * the next format call or ulg_destroy. */
int ulg_pss_format(ulg_ctx *ctx, const char *header, const char *const *names,
                   const int *arity, const char **text, int64_t *len);
/* Same for host lists (offsets[n+1], sets, scores; variable v owns
 * [offsets[v], offsets[v+1]) ), e.g. after the multi-GPU exchange. */
int ulg_pss_format_lists(ulg_ctx *ctx, int n, const int64_t *offsets,
                         const uint64_t *sets, const float *scores,
                         const char *header, const char *const *names,
                         const int *arity, const char **text, int64_t *len);

/* ---- search side (best-score tables, pattern database, A*) ------------ */
/* Load per-variable parent-set lists (file order within each variable;
 * costs = A* costs, i.e. -1 * atof(score), score_cache.cpp:151) and build
 * the best-score lattice tables on the device.  Duplicate sets within a
 * variable must already be merged (ScoreCache::putScore semantics). */
int ulg_search_load(ulg_ctx *ctx, int n, const int64_t *offsets,
                    const uint64_t *sets, const float *costs);
/* Same from the lists the last ulg_cbic_score produced in this context
 * (every variable must have been scored); costs go through the device
 * "%f" round trip (ulg_quantize_costs), lists stay on the device. */
int ulg_search_from_scores(ulg_ctx *ctx);
/* Same from per-variable lists of .pss scores (not yet costs) in variable
 * order -- what the multi-GPU exchange hands every rank (one
 * all-gather of the per-variable lists, then local tables).  offsets[n+1] is
 * a host array (variable v owns [offsets[v], offsets[v+1]) of sets/scores);
 * device_ptrs = 1: sets and scores are device pointers on this context's GPU
 * (e.g. the all-gather's output tensor), 0: host pointers.  Scores go
 * through the device "%f" round trip like ulg_search_from_scores. */
int ulg_search_load_scores(ulg_ctx *ctx, int n, const int64_t *offsets,
                           const uint64_t *sets, const float *scores,
                           int device_ptrs);
/* SparseParentList::getScore / getParents for count (variable, S) pairs:
 * the cost of the first (cost, file-order) stored set that is a subset of
 * S, or FLT_MAX if none; parents[i] gets that set (0 if none). */
int ulg_bestscore_query(ulg_ctx *ctx, int64_t count, const int *vars,
                        const uint64_t *S, float *costs, uint64_t *parents);
/* StaticPatternDatabase with pd_count groups over scc (and ancestors);
 * static_pattern_database.cpp:82-247.  astar() builds it over all
 * variables with no ancestors. */
int ulg_pdb_build(ulg_ctx *ctx, int pd_count, uint64_t ancestors,
                  uint64_t scc);
/* StaticPatternDatabase::h for count subnetworks S. */
int ulg_pdb_query(ulg_ctx *ctx, int64_t count, const uint64_t *S, float *h,
                  int *complete);

#define ULG_ASTAR_EXACT 0 /* the reference's pop order: bit-exact DAG */
#define ULG_ASTAR_GPU 1   /* layer-synchronous GPU order-graph search */
/* astar() (astar_main.cpp:548-644): static PDB(pd_count) over all
 * variables, one search per connected component of the skeleton
 * (edges = n skeleton rows, bit j of row i = edge i-j, or NULL for no
 * skeleton).  Outputs what netFile.csv holds -- vpar[v] = parent set of v
 * (bit i set iff i -> v) -- the total ordering, the goal cost (g of the
 * goal node) and the number of expanded nodes; net_text (if non-NULL)
 * receives the netFile text.  Components are processed in order and each
 * overwrites the outputs, as the reference does. */
int ulg_astar(ulg_ctx *ctx, const uint64_t *edges, int pd_count, int mode,
              uint64_t *vpar, int *order, float *goal_cost, int64_t *expanded,
              char *net_text, int64_t net_cap);
/* astar() with the -p / -s options (astar_main.cpp:590-644, UAI '14): the
 * heuristic is built over (ancestors, scc); each skeleton component (all
 * variables without a skeleton) is searched from the root `ancestors` to
 * ancestors | component.  ulg_astar = ancestors 0, scc all.  Ancestors must
 * not overlap scc; the GPU mode takes no ancestors. */
int ulg_astar_scc(ulg_ctx *ctx, const uint64_t *edges, int pd_count, int mode,
                  uint64_t ancestors, uint64_t scc, uint64_t *vpar, int *order,
                  float *goal_cost, int64_t *expanded, char *net_text,
                  int64_t net_cap);

/* triplet_astar's astar() (astar/triplet_astar.cpp:991-1622): for every
 * variable i and pair of its skeleton neighbours, an exact-order A* with
 * re-opening (run_astar_on_one_scc, :285-674) over the union of the three
 * clusters (skipped above 26 variables, :837-844; one search per distinct
 * cluster -- the result depends on the cluster only), v-structure and
 * undirected-edge bookkeeping (process_triple, :811-989), the
 * unfaithful-edge fixpoint (:1256-1290) and Meek rules 2-4 (:1297-1478).
 * directed_graph (n*n ints, row-major) receives what netFile.csv holds:
 * [i*n+j] = 1 iff the MEC has i -> j (both set = undirected).  edges as in
 * ulg_astar (NULL = no skeleton: every row is the full set, self included).
 * stats (optional, 3 entries): A* runs requested, distinct clusters
 * searched, nodes expanded. */
int ulg_triplet_astar(ulg_ctx *ctx, const uint64_t *edges, int pd_count,
                      int *directed_graph, int64_t *stats);

/* Multi-GPU triplet_astar (distinct clusters are independent A*
 * problems).  The per-cluster results live in a memo on the context, valid
 * for the loaded lists and one pd_count; ulg_triplet_astar reads and fills
 * it, so its stats count only the searches that call made.
 *   ulg_triplet_clusters: the distinct clusters (<= 26 variables) of the
 *     driver's first sweep on the initial skeleton (triplet_astar.cpp:
 *     1148-1204), in first-request order, no searching; *count = how many
 *     (fails with ULG_ERR_ARG if cap is too small and nonzero).
 *   ulg_triplet_solve: the re-opening exact-order A* (:285-674) of each
 *     cluster into the memo; parents (optional, nc*n) receives each cluster
 *     DAG's parent sets.  stats as ulg_triplet_astar.
 *   ulg_triplet_memo_put: seed the memo with other ranks' results.
 * Sharded over ranks, the clusters are solved once each and gathered; every
 * rank then runs ulg_triplet_astar with a full memo and gets the same MEC a
 * single GPU would (a result depends on its cluster only). */
int ulg_triplet_clusters(ulg_ctx *ctx, const uint64_t *edges, uint64_t *clusters,
                         int64_t cap, int64_t *count);
int ulg_triplet_solve(ulg_ctx *ctx, const uint64_t *clusters, int64_t nc,
                      int pd_count, uint64_t *parents, int64_t *stats);
int ulg_triplet_memo_put(ulg_ctx *ctx, const uint64_t *clusters, int64_t nc,
                         int pd_count, const uint64_t *parents);

/* ---- order-graph sweep with variable-sharded tables ----------
 * Replaces run_astar_on_one_scc (astar_main.cpp:216-546) for a full skeleton
 * when one GPU cannot hold every variable's best-score lattice (n >= 31: at
 * n = 32, 32 x 2^31 x 4 B = 275 GB).  Every rank holds every variable's
 * parent-set lists (after the list all-gather) but builds the tables and
 * sweep slices of its own variables only.  Layer by layer (1..n):
 *   ulg_sweep_shard_layer writes, for each of the layer's C(n, layer) nodes
 *     in colex order, this rank's best candidate over the leaves it owns as
 *     a key (ordered cost << 8 | leaf position; 0xFFFFFFFFFF = none) into
 *     keys_dev (device memory, int64-compatible: every key is < 2^40);
 *   the caller MIN-all-reduces keys_dev over the ranks (one RCCL all-reduce
 *     per layer: the smallest cost, then the smallest leaf position -- the
 *     single-GPU sweep's first-strict-minimum rule);
 *   ulg_sweep_shard_commit turns the reduced keys into the layer's g and
 *     leaf bytes (every rank holds all of them).
 * ulg_sweep_shard_end reconstructs the DAG as ULG_ASTAR_GPU does; the result
 * equals the single-GPU ulg_astar(..., ULG_ASTAR_GPU, ...) on a full skeleton
 * bit for bit.  *max_layer_nodes = the largest C(n, layer) (size keys_dev for
 * it).  NaN costs are not supported (their key order differs from the
 * single-GPU float compare). */
int ulg_sweep_shard_begin(ulg_ctx *ctx, uint64_t own, int64_t *max_layer_nodes);
int ulg_sweep_shard_layer(ulg_ctx *ctx, int layer, uint64_t *keys_dev);
int ulg_sweep_shard_commit(ulg_ctx *ctx, int layer, const uint64_t *keys_dev);
int ulg_sweep_shard_end(ulg_ctx *ctx, uint64_t *vpar, int *order, float *goal_cost,
                        int64_t *expanded);

/* ---- tuning knobs -------------------------------------------------------
 * "score_variant" (1, 49, 65, 113, 241; default 241): bit 0 = fully
 * unrolled presence gather (layers <= 6), bit 4 = two-pass layers (the
 * scoring kernel settles every set it can without a walk and queues the rest
 * for a dense walk kernel with the hi-cover prune), bit 5 = that walk
 * bit-sliced (64 x K sets per wave), bit 6 = subset maxima (a per-slot table
 * of the largest stored value below each set settles sets with 2L-3L reads
 * before the rest are compacted for the 2^(L+1) presence gathers), bit 7 =
 * the sets the two-level rules leave to the walk compacted once more before
 * the rest of their gathers (round 6).  1 and 65 are one-pass (every set
 * decided in its lane).  All variants store identical lists.
 * "walk_bucket" (0 or 1; default 1, round 6): the layer-5 and layer-6 walk
 * launches of the two-pass variants with subset maxima (113, 241) walk their
 * queue sorted by walk key (which of the walk's first-level nodes a set may
 * expand): sets with one key share more of their union walk (C3 layer 6
 * without variable 0: its longest wave 811 -> ~465 union points, the
 * launch's union points 3x fewer).  Identical lists either way.
 * "walk_small_sets" (>= 0, default 200000): a layer-6 launch of fewer sets
 * walks one set per lane instead of four (the small launches of 4- and
 * 8-rank shares end with their longest walk wave; walk_bucket 0 only).
 * "walk_k6" (1, 2, 4 or 8; default 4): sets per lane of the other layer-6
 * walk launches: more sets share one walk of their union tree (less work per
 * set, longer waves).  4 gives the shortest single call; with several calls
 * in flight on one GPU (bench.py's slots) 8 gives the most sets per second
 * (C3: 10.17e9 against 9.80e9, single call 0.91 against 0.89 ms).
 * "table_budget_kb" (KiB; default 0 = half the free HBM): memory for the dense
 * best-score tables (16 B per entry incl. the host cost copy).  Lists whose
 * tables over all variables exceed it (e.g. n = 32 with a full skeleton) are
 * searched with tables built per skeleton component / triplet cluster, and
 * lookups outside the current tables scan the lists on the device -- same
 * answers, less memory.
 * "score_streams" (1..4, default 3): variable groups scored on concurrent
 * streams; "score_small_layers" (0..8, default 4): layers up to this size run
 * one one-pass launch per phase over all variables on one stream (they are
 * latency-bound), larger ones the two-pass form per group; "score_fused"
 * (0..4, default 3): layers up to this size (and up to score_small_layers)
 * run in ONE launch, a workgroup of 1024 threads per variable taking its
 * layers and phases in order with a barrier between them (score_variant 113
 * and 241 only, and not under time_limit_ms, whose budget is checked after every
 * layer; lists identical either way; C3 layers 1-3: 40 us against 54 us
 * for six launches, layer 4 in it 340 us: too many sets for one workgroup).
 * "time_limit_ms" (default 0 = none): the reference's -r running-time budget
 * (score: per calculateScores call, score_calculator.cpp:33-52,78,91; astar:
 * a watchdog over the search, astar_main.cpp:135-138,266,696-706).  The GPU
 * scorer checks it after every complete layer (it synchronises the scoring
 * streams there, so only set it when a budget is wanted) and keeps the layers
 * finished so far -- the reference stops mid-layer, at a point that depends
 * on its clock; the exact-order A* checks it every 4096 pops and stops
 * without a goal for that component, as the reference's loop does.
 * "sweep_table" (0/1, default 1): the GPU search (ULG_ASTAR_GPU) on a
 * component without a skeleton filter first lays the component's successor
 * costs out in its own (variable, layer, colex) order (m 2^(m-1) floats,
 * cached until the tables change) when that fits the free HBM; 0 reads the
 * binary-indexed lattice per predecessor instead; 2 uses the slices with
 * 64-bit index arithmetic (1 = 32-bit).
 * "wide_prune" (0/1, default 1): the wide-layer walks skip absent nodes
 * below which no present key reaches -ts (hi-cover tables per variable);
 * "wide_reduced" (0/1, default 1): they skip the recursion's re-tests that
 * cannot change its state (each expanded node costs O(m) tests, not O(m^2));
 * "wide_lds" (0/1/2, default 1): walks longer than 2^6 steps are replayed by
 * one workgroup each with their skip / hi bitsets in LDS (2^q <= 2^20 local
 * subsets; the hi bitset in HBM above 2^19); 2 replays every walk that way.
 * "wide_pool" (0/1/2, default 2): with score_streams > 1 the wide layers run
 * variable by variable on score_streams host threads, largest candidate set
 * first (0: every group's part of a layer together, the slowest group
 * holding the next layer; 1: always by variable; 2: by variable when the
 * wide variables' candidate counts span at least 2).
 * "wide_host" (iterations, default 1024, 0 = never): an LDS replay still
 * walking after that many iterations stops and is replayed from the start on
 * a host thread over the same bitsets (one wave issues at most one
 * instruction every 4 cycles; a host core runs the same sequential walk tens
 * of times faster); "wide_host_max" (default 4096): only launches of at
 * most this many LDS replays hand over; "wide_host_first" (default 0): launches
 * of at most this many replays go to the host whole, without the LDS phase;
 * "wide_host_q" (0..32, default 0 = off): ... as do launches of at most 128
 * replays whose local bits q reach this; "wide_host_threads" (1..64,
 * default 16): host threads for those replays.
 * All variants compute identical results; the knob exists for A/B timing. */
int ulg_set_option(ulg_ctx *ctx, const char *name, int64_t value);
/* Read-back of per-call state: "out_of_time" (1 if the last ulg_cbic_score,
 * ulg_astar* or ulg_triplet_astar ran out of time_limit_ms), "highest_completed_layer" (the
 * reference's ScoreCalculator::highestCompletedLayer of the last scoring call,
 * score_calculator.h:45), "exact_cycles" / "exact_instructions" /
 * "exact_cache_misses" (the last exact-order A*'s user-space host counters on
 * the calling thread, perf_event_open; -1 where the host does not grant
 * them), "score_error_word" (the last scoring call's device error word: 0,
 * or bit 0 a wide walk over its cap, bit 1 a walk-queue segment overflow,
 * bit 2 a walk entry naming a slot past the call's table -- any nonzero
 * word also made that call return a nonzero status). */
int ulg_get_info(ulg_ctx *ctx, const char *name, int64_t *value);

/* ---- profiling (per-kernel HIP-event timing on the context stream) ---- */
int ulg_profile_enable(ulg_ctx *ctx, int on);
/* Average duration (ms) and launch count of kernels whose name matches
 * `name` exactly, since the last reset.  Returns ULG_ERR_ARG if none. */
int ulg_profile_get(ulg_ctx *ctx, const char *name, double *avg_ms,
                    int64_t *count, double *total_ms);
/* Writes a newline-separated "name count total_ms" listing into buf. */
int ulg_profile_dump(ulg_ctx *ctx, char *buf, int64_t cap);
int ulg_profile_reset(ulg_ctx *ctx);
/* Time only the kernels named in the comma-separated list (NULL or "" = all):
 * each timed kernel costs two event records on the host, which the small
 * launches of a scoring call notice. */
int ulg_profile_select(ulg_ctx *ctx, const char *names);

/* ---- diagnostics (tests only; no reference counterpart) ---- */
/* One host pattern-database build in the form the triplet look-ahead pool
 * uses (StaticPatternDatabase, static_pattern_database.cpp:82-247, over
 * `cluster`), with the pool's cancel flag preset when cancel_preset != 0.
 * out[4]: built, cancelled, entries built, entries equal to the device PDB's. */
int ulg_diag_pdb_host(ulg_ctx *ctx, uint64_t cluster, int pd_count, int cancel_preset, int64_t *out);

#ifdef __cplusplus
}
#endif
#endif
