/* ora_search.c -- TEST INFRASTRUCTURE ONLY (see ora.h).
 *
 * Plain-C restatement of the reference's order-graph search:
 *   SparseParentList             score_cache/sparse_parent_list.cpp:20-55
 *   StaticPatternDatabase        heuristic/static_pattern_database.cpp:82-247
 *   Node / CompareNodeStar       base/node.h:24-135
 *   PriorityQueue + heap         priority_queue/priority_queue.cpp:36-64,
 *                                priority_queue/priority_queue-inl.h:19-234
 *   run_astar_on_one_scc         astar/astar_main.cpp:216-546
 *   reconstructSolution/outputs  astar_main.cpp:140-212,505-533
 *   astar() driver               astar_main.cpp:548-644
 *   Skeleton components          base/skeleton.cpp:187-230
 */
#define _GNU_SOURCE
#include "ora.h"
#include "ora_internal.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { vs_t set; float cost; int64_t idx; } spl_entry;

typedef struct {
    int64_t count;
    vs_t *parents;
    float *scores;
} spl_t;

typedef struct {
    vs_t group;
    int size;
    int *bitpos;     /* group bit positions, ascending */
    float *pd;       /* 2^size, indexed by pext(R, group) */
    uint8_t *present;
} pdb_group;

struct ora_search {
    int n;
    spl_t *spl;
    int best_index; /* SparseParentList::bestIndex (stateful) */
    int pd_count;
    vs_t ancestors, scc;
    pdb_group *groups;
    double time_limit_s; /* -r (astar_main.cpp:135-138,696-706): 0 = none */
    int out_of_time;
    int64_t last_open; /* open-list size when the last search ended */
};

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* the -r watchdog: the search loop ends (outOfTime, astar_main.cpp:266)
 * once the budget is spent; the expansions so far are still reported */
void ora_search_set_time_limit(ora_search *s, double seconds) { s->time_limit_s = seconds; }
int ora_search_out_of_time(const ora_search *s) { return s->out_of_time; }
int64_t ora_search_last_open(const ora_search *s) { return s->last_open; }

static int cmp_spl(const void *a, const void *b) {
    const spl_entry *x = (const spl_entry *)a, *y = (const spl_entry *)b;
    if (x->cost < y->cost) return -1;
    if (x->cost > y->cost) return 1;
    /* pinned tie-break: file line order */
    return x->idx < y->idx ? -1 : (x->idx > y->idx ? 1 : 0);
}

ora_search *ora_search_create(int n, const int64_t *offsets,
                              const ora_varset *sets, const float *costs) {
    ora_search *s = (ora_search *)calloc(1, sizeof(*s));
    s->n = n;
    s->spl = (spl_t *)calloc((size_t)n, sizeof(spl_t));
    for (int v = 0; v < n; v++) {
        int64_t c = offsets[v + 1] - offsets[v];
        spl_entry *e = (spl_entry *)malloc(sizeof(spl_entry) * (size_t)(c ? c : 1));
        /* ScoreCache::putScore overwrites duplicate parent sets: keep the
         * last value at the first position (FloatMap semantics). */
        omap seen;
        omap_init(&seen, (size_t)c + 1);
        int64_t m = 0;
        for (int64_t i = 0; i < c; i++) {
            uint64_t pos;
            vs_t st = sets[offsets[v] + i];
            if (omap_get(&seen, st, &pos)) { e[pos].cost = costs[offsets[v] + i]; continue; }
            omap_put(&seen, st, (uint64_t)m);
            e[m].set = st; e[m].cost = costs[offsets[v] + i]; e[m].idx = i; m++;
        }
        omap_free(&seen);
        qsort(e, (size_t)m, sizeof(spl_entry), cmp_spl);
        s->spl[v].count = m;
        s->spl[v].parents = (vs_t *)malloc(sizeof(vs_t) * (size_t)(m ? m : 1));
        s->spl[v].scores = (float *)malloc(sizeof(float) * (size_t)(m ? m : 1));
        for (int64_t i = 0; i < m; i++) { s->spl[v].parents[i] = e[i].set; s->spl[v].scores[i] = e[i].cost; }
        free(e);
    }
    return s;
}

static void free_groups(ora_search *s) {
    if (!s->groups) return;
    for (int g = 0; g < s->pd_count; g++) {
        free(s->groups[g].bitpos); free(s->groups[g].pd); free(s->groups[g].present);
    }
    free(s->groups);
    s->groups = NULL;
}

void ora_search_free(ora_search *s) {
    if (!s) return;
    for (int v = 0; v < s->n; v++) { free(s->spl[v].parents); free(s->spl[v].scores); }
    free(s->spl);
    free_groups(s);
    free(s);
}

/* SparseParentList::getScore (sparse_parent_list.cpp:44-55) */
static float spl_get(ora_search *s, int v, vs_t pars, int64_t *best) {
    const spl_t *l = &s->spl[v];
    int64_t i;
    for (i = 0; i < l->count; i++)
        if ((pars & l->parents[i]) == l->parents[i]) break;
    *best = i;
    if (i == l->count) return FLT_MAX;
    return l->scores[i];
}

float ora_bestscore(ora_search *s, int v, ora_varset S, ora_varset *parents) {
    int64_t b;
    float c = spl_get(s, v, S, &b);
    if (parents) *parents = (b < s->spl[v].count) ? s->spl[v].parents[b] : 0;
    return c;
}

/* ---- static pattern database ------------------------------------------ */
static int64_t pext_group(const pdb_group *g, vs_t R) {
    int64_t r = 0;
    for (int i = 0; i < g->size; i++)
        if ((R >> g->bitpos[i]) & 1ULL) r |= 1LL << i;
    return r;
}
static vs_t pdep_group(const pdb_group *g, int64_t r) {
    vs_t R = 0;
    for (int i = 0; i < g->size; i++)
        if ((r >> i) & 1) R |= 1ULL << g->bitpos[i];
    return R;
}

/* createPatternDatabase + expand (static_pattern_database.cpp:176-247).
 * Layers are dense arrays over R = group \ key; keys are visited in
 * ascending R order (the reference iterates a boost::unordered_map; the
 * value is order-independent whenever all costs are <= 0). */
static void create_pdb(ora_search *s, vs_t allVariables, pdb_group *g) {
    const int64_t full = 1LL << g->size;
    float *prev = (float *)calloc((size_t)full, sizeof(float));
    uint8_t *prevp = (uint8_t *)calloc((size_t)full, 1);
    float *cur = (float *)calloc((size_t)full, sizeof(float));
    uint8_t *curp = (uint8_t *)calloc((size_t)full, 1);
    g->pd = (float *)calloc((size_t)full, sizeof(float));
    g->present = (uint8_t *)calloc((size_t)full, 1);
    /* previousLayer[allVariables] = 0; R = group \ allVariables (empty) */
    int64_t r0 = pext_group(g, g->group & ~allVariables);
    prev[r0] = 0.0f; prevp[r0] = 1;
    for (int layer = 0; layer <= g->size; layer++) {
        memset(cur, 0, sizeof(float) * (size_t)full);
        memset(curp, 0, (size_t)full);
        for (int64_t r = 0; r < full; r++) {
            if (!prevp[r]) continue;
            const vs_t key = allVariables & ~pdep_group(g, r);
            const float value = prev[r];
            /* expand(key, value, ...) */
            for (int leaf = 0; leaf < s->n; leaf++) {
                if (!((key >> leaf) & 1ULL) || !((g->group >> leaf) & 1ULL)) continue;
                const vs_t parentChoices = key | s->ancestors;
                int64_t b;
                const float the_score = spl_get(s, leaf, parentChoices, &b);
                const float newG = the_score + value;
                const vs_t nk = key ^ (1ULL << leaf);
                const int64_t nr = pext_group(g, g->group & ~nk);
                const float oldG = curp[nr] ? cur[nr] : 0.0f;
                curp[nr] = 1;
                if (oldG == 0 || newG < oldG) cur[nr] = newG;
                else cur[nr] = oldG;
            }
            /* pattern = variableSet & ~key & ~ancestors */
            const vs_t pattern = g->group & ~key & ~s->ancestors;
            const int64_t pr = pext_group(g, pattern);
            g->pd[pr] = value; g->present[pr] = 1;
        }
        float *t = prev; prev = cur; cur = t;
        uint8_t *tp = prevp; prevp = curp; curp = tp;
    }
    for (int64_t r = 0; r < full; r++) {
        if (!prevp[r]) continue;
        const vs_t key = allVariables & ~pdep_group(g, r);
        const int64_t pr = pext_group(g, g->group & ~key);
        g->pd[pr] = prev[r]; g->present[pr] = 1;
    }
    free(prev); free(prevp); free(cur); free(curp);
}

/* StaticPatternDatabase::initialize(spgs) (static_pattern_database.cpp:82-134) */
int ora_pdb_build(ora_search *s, int pd_count, ora_varset ancestors, ora_varset scc) {
    free_groups(s);
    if (pd_count < 1) return -1;
    s->pd_count = pd_count;
    s->ancestors = ancestors;
    s->scc = scc;
    s->groups = (pdb_group *)calloc((size_t)pd_count, sizeof(pdb_group));
    const vs_t allVariables = scc;
    int remainingCount = popc64(scc);
    int var = scc ? __builtin_ctzll(scc) : -1; /* VARSET_FIND_FIRST_SET */
    const int pds = (int)ceil((float)remainingCount / pd_count);
    int x = 0;
    for (int pd_i = 0; pd_i < pd_count; pd_i++) {
        vs_t group = 0;
        int sz;
        for (sz = 0; sz < pds && x < remainingCount; sz++) {
            group |= 1ULL << var;
            /* VARSET_FIND_NEXT_SET: index + ffsl(vs >> (index+1)) */
            vs_t rest = (var + 1 < 64) ? (scc >> (var + 1)) : 0;
            var = var + (rest ? (__builtin_ctzll(rest) + 1) : 0);
            ++x;
        }
        pdb_group *g = &s->groups[pd_i];
        g->group = group;
        g->size = sz;
        g->bitpos = (int *)malloc(sizeof(int) * (size_t)(sz ? sz : 1));
        int t = 0;
        for (int b = 0; b < 64 && t < sz; b++)
            if ((group >> b) & 1ULL) g->bitpos[t++] = b;
        create_pdb(s, allVariables, g);
    }
    return 0;
}

/* StaticPatternDatabase::h (static_pattern_database.cpp:145-174) */
float ora_pdb_h(ora_search *s, ora_varset S, int *complete) {
    float h = 0;
    const vs_t mask = (s->n >= 64) ? ~0ULL : ((1ULL << s->n) - 1ULL);
    const vs_t remaining = (~S) & mask;
    for (int pd_i = 0; pd_i < s->pd_count; pd_i++) {
        const pdb_group *g = &s->groups[pd_i];
        const vs_t vs = g->group & remaining;
        const int64_t r = pext_group(g, vs);
        if (!g->present[r]) return FLT_MAX / 64.0f;
        if (vs == remaining) {
            if (complete) *complete = 1;
            return g->pd[r];
        }
        h += g->pd[r];
    }
    return h;
}

int ora_pdb_groups(ora_search *s, ora_varset *groups, int max_groups) {
    for (int g = 0; g < s->pd_count && g < max_groups; g++) groups[g] = s->groups[g].group;
    return s->pd_count;
}

float ora_pdb_value(ora_search *s, int g, ora_varset R) {
    const pdb_group *gr = &s->groups[g];
    return gr->pd[pext_group(gr, R & gr->group)];
}

/* ---- Node / heap -------------------------------------------------------- */
typedef struct {
    float g, h;
    vs_t sub;
    uint8_t leaf;
    int pqPos;
} node_t;

typedef struct {
    node_t **a;
    int64_t size, cap;
    int hang;
} heap_t;

/* CompareNodeStar (node.h:124-135): true if a has LOWER priority than b */
static inline int cns(const node_t *a, const node_t *b) {
    volatile float fa = a->g + a->h;
    volatile float fb = b->g + b->h;
    volatile float diff = fa - fb;
    if (fabsf(diff) < FLT_EPSILON) {
        int la = popc64(a->sub) & 0xff, lb = popc64(b->sub) & 0xff;
        return (lb - la) > 0;
    }
    return diff > 0;
}

static void hp_push_hole(heap_t *H, int64_t hole, int64_t top, node_t *value) {
    int64_t parent = (hole - 1) / 2;
    while (hole > top && cns(H->a[parent], value)) {
        H->a[hole] = H->a[parent];
        H->a[hole]->pqPos = (int)hole;
        hole = parent;
        parent = (hole - 1) / 2;
    }
    H->a[hole] = value;
    value->pqPos = (int)hole;
}

static void hp_push(heap_t *H, node_t *n) {
    if (H->size == H->cap) {
        H->cap = H->cap ? H->cap * 2 : 1024;
        H->a = (node_t **)realloc(H->a, sizeof(node_t *) * (size_t)H->cap);
    }
    H->a[H->size++] = n;
    hp_push_hole(H, H->size - 1, 0, n);
}

static void hp_adjust(heap_t *H, int64_t hole, int64_t len, node_t *value) {
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (cns(H->a[second], H->a[second - 1])) second--;
        H->a[hole] = H->a[second];
        H->a[hole]->pqPos = (int)hole;
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        H->a[hole] = H->a[second - 1];
        H->a[hole]->pqPos = (int)hole;
        hole = second - 1;
    }
    hp_push_hole(H, hole, top, value);
}

static node_t *hp_pop(heap_t *H) {
    node_t *ret = H->a[0];
    const int64_t last = H->size - 1;
    node_t *value = H->a[last];
    H->a[last] = H->a[0];
    hp_adjust(H, 0, last, value);
    H->size--;
    return ret;
}

static void hp_update(heap_t *H, node_t *n) {
    const int64_t pos = n->pqPos;
    const int64_t parent = (pos - 1) / 2;
    node_t *value = H->a[pos];
    if (pos > 0 && cns(H->a[parent], value)) {
        /* __up_heap */
        int64_t par = (pos - 1) / 2, index = pos;
        while (index > 0 && cns(H->a[par], value)) {
            H->a[index] = H->a[par];
            H->a[index]->pqPos = (int)index;
            index = par;
            par = (par - 1) / 2;
        }
        if (pos != index) { H->a[index] = value; value->pqPos = (int)index; }
    } else {
        /* __down_heap, including its left-only descent and missing pqPos
         * update of the moved value (priority_queue-inl.h:176-208). */
        const int64_t len = H->size;
        int64_t index = pos, left = 2 * index + 1, right = 2 * index + 2, largest = len;
        int64_t guard = 0;
        while (index < len) {
            if ((right >= len) || ((left < len) && cns(H->a[right], H->a[left]))) largest = left;
            if (largest < len && cns(value, H->a[largest])) {
                if (largest == index) { H->hang = 1; break; } /* reference loops forever here */
                H->a[index] = H->a[largest];
                H->a[largest]->pqPos = (int)index;
                index = largest;
                left = index * 2 + 1;
                right = index * 2 + 2;
            } else break;
            if (++guard > 128) { H->hang = 1; break; }
        }
        if (pos != index) H->a[index] = value;
    }
}

/* ---- A* ------------------------------------------------------------------ */
typedef struct {
    node_t *blocks[4096];
    int nblocks;
    int64_t used;
} pool_t;
#define POOL_BLOCK (1 << 16)
static node_t *pool_new(pool_t *p) {
    int64_t b = p->used / POOL_BLOCK, o = p->used % POOL_BLOCK;
    if (b >= p->nblocks) {
        if (p->nblocks >= 4096) { fprintf(stderr, "oracle A*: node pool exhausted\n"); abort(); }
        p->blocks[p->nblocks++] = (node_t *)malloc(sizeof(node_t) * POOL_BLOCK);
    }
    p->used++;
    return &p->blocks[b][o];
}
static void pool_free(pool_t *p) {
    for (int i = 0; i < p->nblocks; i++) free(p->blocks[i]);
    p->nblocks = 0; p->used = 0;
}

/* connected components (skeleton.cpp:187-230) in discovery order */
static int components(const vs_t *edges, int n, vs_t *out) {
    int nc = 0;
    vs_t visited = 0;
    for (int v = 0; v < n; v++) {
        if ((visited >> v) & 1ULL) continue;
        vs_t comp = 0;
        /* explore_one_scc: DFS over ascending neighbour index */
        int stack[64], it[64], sp = 0;
        stack[sp] = v; it[sp] = 0; sp++;
        visited |= 1ULL << v; comp |= 1ULL << v;
        while (sp > 0) {
            int cur = stack[sp - 1];
            int i = it[sp - 1];
            for (; i < n; i++) {
                if ((visited >> i) & 1ULL) continue;
                if ((edges[cur] >> i) & 1ULL) break;
            }
            if (i < n) {
                it[sp - 1] = i + 1;
                visited |= 1ULL << i; comp |= 1ULL << i;
                stack[sp] = i; it[sp] = 0; sp++;
            } else sp--;
        }
        out[nc++] = comp;
    }
    return nc;
}

static int run_astar_one(ora_search *s, const vs_t *edges, int skeleton_good,
                         vs_t ancestors, vs_t the_scc, vs_t *vpar, int *order,
                         float *goal_cost, int64_t *expanded, char *net_text,
                         int64_t net_cap, int *hang) {
    const int n = s->n;
    omap generated;
    omap_init(&generated, 1 << 12);
    pool_t pool;
    memset(&pool, 0, sizeof pool);
    heap_t open;
    memset(&open, 0, sizeof open);

    /* VARSET_FIND_NEXT_SET(the_scc, 0) = 0 + ffsl(the_scc >> 1) */
    const vs_t r1 = the_scc >> 1;
    node_t *root = pool_new(&pool);
    root->g = 0.0f; root->h = 0.0f; root->sub = ancestors;
    root->leaf = (uint8_t)(r1 ? __builtin_ctzll(r1) + 1 : 0);
    root->pqPos = 0;
    hp_push(&open, root);

    node_t *goal = NULL;
    const vs_t allVariables = ancestors | the_scc;
    const float upperBound = FLT_MAX;
    int64_t nodesExpanded = 0;
    const double t_end = s->time_limit_s > 0 ? now_s() + s->time_limit_s : 0.0;
    s->out_of_time = 0;
    while (open.size > 0) {
        if (t_end > 0 && (nodesExpanded & 1023) == 0 && now_s() > t_end) {
            s->out_of_time = 1;
            break;
        }
        node_t *u = hp_pop(&open);
        nodesExpanded++;
        const vs_t variables = u->sub;
        if (variables == allVariables) { goal = u; break; }
        if (u->g + u->h > upperBound) break;
        u->pqPos = -2;
        for (int leaf = 0; leaf < n; leaf++) {
            if ((variables >> leaf) & 1ULL) continue;
            if (!((the_scc >> leaf) & 1ULL)) continue;
            if (skeleton_good && variables != 0) {
                if ((variables & edges[leaf]) == 0) continue;
            }
            const vs_t nv = variables | (1ULL << leaf);
            uint64_t idx;
            node_t *succ = NULL;
            if (omap_get(&generated, nv, &idx)) succ = (node_t *)(uintptr_t)idx;
            if (succ == NULL) {
                int64_t b;
                const float leaf_score = spl_get(s, leaf, nv, &b);
                const float g = u->g + leaf_score;
                int complete = 0;
                const float h = ora_pdb_h(s, nv, &complete);
                succ = pool_new(&pool);
                succ->g = g; succ->h = h; succ->sub = nv; succ->leaf = (uint8_t)leaf; succ->pqPos = 0;
                hp_push(&open, succ);
                omap_put(&generated, nv, (uint64_t)(uintptr_t)succ);
                continue;
            }
            if (succ->pqPos == -2) continue;
            int64_t b;
            const float g = u->g + spl_get(s, leaf, variables, &b);
            if (g < succ->g) {
                succ->leaf = (uint8_t)leaf;
                succ->g = g;
                hp_update(&open, succ);
            }
        }
    }
    *expanded += nodesExpanded;
    s->last_open = open.size;
    if (open.hang) *hang = 1;
    int ok = 0;
    if (goal) {
        ok = 1;
        /* reconstructSolution (astar_main.cpp:140-166) */
        int *total = (int *)calloc((size_t)n, sizeof(int));
        vs_t *opt = (vs_t *)calloc((size_t)n, sizeof(vs_t));
        vs_t remaining = goal->sub;
        node_t *current = goal;
        const int count = popc64(the_scc);
        for (int i = 0; i < count && current; i++) {
            const int leaf = current->leaf;
            total[count - 1 - i] = leaf;
            int64_t b;
            (void)spl_get(s, leaf, remaining, &b);
            opt[count - 1 - i] = (b < s->spl[leaf].count) ? s->spl[leaf].parents[b] : 0;
            remaining ^= 1ULL << leaf;
            uint64_t idx;
            current = omap_get(&generated, remaining, &idx) ? (node_t *)(uintptr_t)idx : NULL;
        }
        /* netFile (astar_main.cpp:192-212) */
        if (net_text && net_cap > 0) {
            int64_t len = 0;
            len += snprintf(net_text + len, (size_t)(net_cap - len), "NumVars %d\n", n);
            for (int v = 0; v < n && len < net_cap; v++) {
                len += snprintf(net_text + len, (size_t)(net_cap - len), "Var %d, parents", total[v] + 1);
                for (int i = 0; i < n && len < net_cap; i++)
                    if ((opt[v] >> i) & 1ULL) len += snprintf(net_text + len, (size_t)(net_cap - len), ", %d", i + 1);
                if (len < net_cap) len += snprintf(net_text + len, (size_t)(net_cap - len), "\n");
            }
        }
        /* netFile.csv parent matrix (astar_main.cpp:505-533) */
        for (int v = 0; v < n; v++) vpar[v] = 0;
        for (int v = 0; v < n; v++) vpar[total[v]] = opt[v];
        for (int v = 0; v < n; v++) order[v] = total[v];
        *goal_cost = goal->g;
        free(total);
        free(opt);
    }
    omap_free(&generated);
    pool_free(&pool);
    free(open.a);
    return ok;
}

int ora_astar(ora_search *s, const ora_varset *edges, int pd_count,
              ora_varset *vpar, int *order, float *goal_cost,
              int64_t *expanded, char *net_text, int64_t net_cap) {
    const int n = s->n;
    const vs_t all = (n >= 64) ? ~0ULL : ((1ULL << n) - 1ULL);
    return ora_astar_scc(s, edges, pd_count, 0ULL, all, vpar, order, goal_cost, expanded, net_text, net_cap);
}

/* astar() with -p / -s (astar_main.cpp:590-644): the heuristic is built over
 * (ancestors, scc); every skeleton component (all variables without a
 * skeleton) is searched from the root `ancestors` to ancestors | component. */
int ora_astar_scc(ora_search *s, const ora_varset *edges, int pd_count, ora_varset ancestors, ora_varset scc,
                  ora_varset *vpar, int *order, float *goal_cost,
                  int64_t *expanded, char *net_text, int64_t net_cap) {
    const int n = s->n;
    const vs_t all = (n >= 64) ? ~0ULL : ((1ULL << n) - 1ULL);
    if (ora_pdb_build(s, pd_count, ancestors, scc) != 0) return -1;
    vs_t comps[64];
    int nc;
    int skeleton_good = edges != NULL;
    if (edges) nc = components(edges, n, comps);
    else { comps[0] = all; nc = 1; }
    *expanded = 0;
    int fail = 0, hang = 0;
    for (int i = 0; i < n; i++) { vpar[i] = 0; order[i] = 0; }
    *goal_cost = 0.0f;
    if (net_text && net_cap > 0) net_text[0] = 0;
    for (int c = 0; c < nc; c++) {
        if (!run_astar_one(s, edges, skeleton_good, ancestors, comps[c], vpar, order,
                           goal_cost, expanded, net_text, net_cap, &hang))
            fail = 1;
    }
    if (hang) return 2;
    return fail;
}

/* ---- triplet_astar (astar/triplet_astar.cpp) ------------------------------ */

/* run_astar_on_one_scc of triplet_astar.cpp:285-674: a static PDB built on
 * (ancestors, the_scc) for every call, no skeleton filter (:411-424 is
 * commented out), EdgeConstraints with no ancestors (always satisfied), and
 * closed nodes RE-OPENED when a strictly better g arrives (:556-576).
 * Writes op[v] / oc[v] (optimal parents / children) for the cluster. */
static int triplet_astar_one(ora_search *s, int pd_count, vs_t ancestors, vs_t the_scc,
                             vs_t *op, vs_t *oc, int64_t *expanded, int *hang) {
    const int n = s->n;
    if (ora_pdb_build(s, pd_count, ancestors, the_scc) != 0) return -1;
    for (int v = 0; v < n; v++) { op[v] = 0; oc[v] = 0; }
    omap generated;
    omap_init(&generated, 1 << 12);
    pool_t pool;
    memset(&pool, 0, sizeof pool);
    heap_t open;
    memset(&open, 0, sizeof open);
    const vs_t r1 = the_scc >> 1;
    node_t *root = pool_new(&pool);
    root->g = 0.0f; root->h = 0.0f; root->sub = ancestors;
    root->leaf = (uint8_t)(r1 ? __builtin_ctzll(r1) + 1 : 0);
    root->pqPos = 0;
    hp_push(&open, root);
    node_t *goal = NULL;
    const vs_t allVariables = ancestors | the_scc;
    const float upperBound = FLT_MAX;
    int64_t nexp = 0;
    while (open.size > 0) {
        node_t *u = hp_pop(&open);
        nexp++;
        const vs_t variables = u->sub;
        if (variables == allVariables) { goal = u; break; }
        if (u->g + u->h > upperBound) break;
        u->pqPos = -2;
        for (int leaf = 0; leaf < n; leaf++) {
            if ((variables >> leaf) & 1ULL) continue;
            if (!((the_scc >> leaf) & 1ULL)) continue;
            const vs_t nv = variables | (1ULL << leaf);
            uint64_t idx;
            node_t *succ = NULL;
            if (omap_get(&generated, nv, &idx)) succ = (node_t *)(uintptr_t)idx;
            int64_t b;
            if (succ == NULL) {
                const float g = u->g + spl_get(s, leaf, nv, &b);
                int complete = 0;
                const float h = ora_pdb_h(s, nv, &complete);
                succ = pool_new(&pool);
                succ->g = g; succ->h = h; succ->sub = nv; succ->leaf = (uint8_t)leaf; succ->pqPos = 0;
                hp_push(&open, succ);
                omap_put(&generated, nv, (uint64_t)(uintptr_t)succ);
                continue;
            }
            const float g = u->g + spl_get(s, leaf, variables, &b);
            if (g < succ->g) {
                succ->leaf = (uint8_t)leaf;
                succ->g = g;
                if (succ->pqPos == -2) { succ->pqPos = 0; hp_push(&open, succ); }
                else hp_update(&open, succ);
            }
        }
    }
    *expanded += nexp;
    if (open.hang) *hang = 1;
    int ok = 0;
    if (goal) {
        ok = 1;
        /* reconstructSolution with children (triplet_astar.cpp:172-224) */
        const int count = popc64(the_scc);
        int total[64];
        vs_t opt[64], ch[64];
        int var2ord[64];
        for (int i = 0; i < 64; i++) { total[i] = 0; opt[i] = 0; ch[i] = 0; var2ord[i] = -1; }
        vs_t remaining = goal->sub;
        node_t *current = goal;
        for (int i = 0; i < count && current; i++) {
            const int leaf = current->leaf;
            total[count - 1 - i] = leaf;
            var2ord[leaf] = count - 1 - i;
            int64_t b;
            (void)spl_get(s, leaf, remaining, &b);
            opt[count - 1 - i] = (b < s->spl[leaf].count) ? s->spl[leaf].parents[b] : 0;
            remaining ^= 1ULL << leaf;
            uint64_t idx;
            current = omap_get(&generated, remaining, &idx) ? (node_t *)(uintptr_t)idx : NULL;
        }
        for (int i = 0; i < count; i++)
            for (int j = 0; j < n; j++)
                if (((opt[i] >> j) & 1ULL) && var2ord[j] >= 0) ch[var2ord[j]] |= 1ULL << total[i];
        const int num_vars = popc64(allVariables);
        for (int v = 0; v < num_vars; v++) { op[total[v]] = opt[v]; oc[total[v]] = ch[v]; }
    }
    omap_free(&generated);
    pool_free(&pool);
    free(open.a);
    return ok;
}

typedef struct {
    ora_search *s;
    int n, pd_count;
    vs_t *nb;             /* skeleton neighbours (mutable) */
    vs_t *clusters;
    int *dg;              /* directed_graph, n x n */
    vs_t *vstr_parents;
    int num_v_structures;
    omap triplets_checked;
    /* memo: the A* result depends only on the cluster */
    omap memo;
    vs_t *memo_op, *memo_oc;
    int memo_count, memo_cap;
    int64_t runs, distinct_runs, expanded;
    int hang;
} trip_t;

#define DG(t, a, b) ((t)->dg[(a) * (t)->n + (b)])

static int trip_astar_cached(trip_t *t, vs_t cluster, vs_t **op, vs_t **oc) {
    uint64_t slot;
    t->runs++;
    if (!omap_get(&t->memo, cluster, &slot)) {
        if (t->memo_count == t->memo_cap) {
            t->memo_cap = t->memo_cap ? 2 * t->memo_cap : 64;
            t->memo_op = (vs_t *)realloc(t->memo_op, sizeof(vs_t) * 64 * (size_t)t->memo_cap);
            t->memo_oc = (vs_t *)realloc(t->memo_oc, sizeof(vs_t) * 64 * (size_t)t->memo_cap);
        }
        slot = (uint64_t)t->memo_count++;
        triplet_astar_one(t->s, t->pd_count, 0ULL, cluster, t->memo_op + 64 * slot, t->memo_oc + 64 * slot,
                          &t->expanded, &t->hang);
        t->distinct_runs++;
        omap_put(&t->memo, cluster, slot);
    }
    *op = t->memo_op + 64 * slot;
    *oc = t->memo_oc + 64 * slot;
    return 0;
}

/* process_triple (triplet_astar.cpp:811-989) */
static void process_triple(trip_t *t, int i, int vj, int vk) {
    uint64_t arr[3] = {(uint64_t)i, (uint64_t)vj, (uint64_t)vk};
    for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++)
            if ((int)arr[b] < (int)arr[a]) { uint64_t x = arr[a]; arr[a] = arr[b]; arr[b] = x; }
    const vs_t big = t->clusters[i] | t->clusters[vj] | t->clusters[vk];
    if (popc64(big) > 26) return;
    const uint64_t key = (arr[0] << 40) + (arr[1] << 20) + arr[2];
    if (omap_get(&t->triplets_checked, key, NULL)) return;
    omap_put(&t->triplets_checked, key, 1);
    vs_t *op, *oc;
    trip_astar_cached(t, big, &op, &oc);
    const int parents_vj_vk = ((op[i] >> vj) & 1ULL) && ((op[i] >> vk) & 1ULL);
    const int parents_i_vj = ((op[vk] >> i) & 1ULL) && ((op[vk] >> vj) & 1ULL);
    const int parents_i_vk = ((op[vj] >> i) & 1ULL) && ((op[vj] >> vk) & 1ULL);
    if (parents_vj_vk) {
        t->num_v_structures++;
        DG(t, vj, i) = 1; DG(t, vk, i) = 1; DG(t, i, vj) = 0; DG(t, i, vk) = 0;
        if ((((op[vj] >> vk) & 1ULL) || ((op[vk] >> vj) & 1ULL)) && 0 == DG(t, vk, vj) && 0 == DG(t, vj, vk)) {
            DG(t, vk, vj) = 1; DG(t, vj, vk) = 1;
        }
        t->vstr_parents[i] |= 1ULL << vk;
        t->vstr_parents[i] |= 1ULL << vj;
    } else if (parents_i_vj) {
        t->num_v_structures++;
        DG(t, vj, vk) = 1; DG(t, i, vk) = 1; DG(t, vk, i) = 0; DG(t, vk, vj) = 0;
        if ((((op[vj] >> i) & 1ULL) || ((op[i] >> vj) & 1ULL)) && 0 == DG(t, i, vj) && 0 == DG(t, vj, i)) {
            DG(t, i, vj) = 1; DG(t, vj, i) = 1;
        }
        t->vstr_parents[vk] |= 1ULL << i;
        t->vstr_parents[vk] |= 1ULL << vj;
    } else if (parents_i_vk) {
        t->num_v_structures++;
        DG(t, vk, vj) = 1; DG(t, i, vj) = 1; DG(t, vj, i) = 0; DG(t, vj, vk) = 0;
        if ((((op[vk] >> i) & 1ULL) || ((op[i] >> vk) & 1ULL)) && 0 == DG(t, i, vk) && 0 == DG(t, vk, i)) {
            DG(t, i, vk) = 1; DG(t, vk, i) = 1;
        }
        t->vstr_parents[vj] |= 1ULL << i;
        t->vstr_parents[vj] |= 1ULL << vk;
    } else {
        if ((((op[vj] >> vk) & 1ULL) || ((op[vk] >> vj) & 1ULL)) && 0 == DG(t, vk, vj) && 0 == DG(t, vj, vk)) {
            DG(t, vk, vj) = 1; DG(t, vj, vk) = 1;
        }
        if ((((op[vj] >> i) & 1ULL) || ((op[i] >> vj) & 1ULL)) && 0 == DG(t, i, vj) && 0 == DG(t, vj, i)) {
            DG(t, i, vj) = 1; DG(t, vj, i) = 1;
        }
        if ((((op[vk] >> i) & 1ULL) || ((op[i] >> vk) & 1ULL)) && 0 == DG(t, i, vk) && 0 == DG(t, vk, i)) {
            DG(t, i, vk) = 1; DG(t, vk, i) = 1;
        }
    }
}

static void trip_add_edge(trip_t *t, int a, int b) {
    t->nb[a] |= 1ULL << b;
    t->nb[b] |= 1ULL << a;
    t->clusters[a] = t->nb[a];
    t->clusters[b] = t->nb[b];
}

/* astar() of triplet_astar.cpp:991-1622 */
int ora_triplet_astar(ora_search *s, const ora_varset *edges, int pd_count, int *directed_graph,
                      int64_t *astar_runs, int64_t *distinct_runs, int64_t *expanded) {
    const int n = s->n;
    trip_t T;
    memset(&T, 0, sizeof T);
    T.s = s; T.n = n; T.pd_count = pd_count;
    T.nb = (vs_t *)calloc(64, sizeof(vs_t));
    T.clusters = (vs_t *)calloc(64, sizeof(vs_t));
    T.vstr_parents = (vs_t *)calloc(64, sizeof(vs_t));
    T.dg = directed_graph;
    for (int a = 0; a < n * n; a++) T.dg[a] = 0;
    omap_init(&T.triplets_checked, 1024);
    omap_init(&T.memo, 64);
    const vs_t all = (n >= 64) ? ~0ULL : ((1ULL << n) - 1ULL);
    /* no skeleton: Skeleton::get_neighbors returns all_bit_set (self included) */
    for (int v = 0; v < n; v++) T.nb[v] = edges ? edges[v] : all;
    for (int v = 0; v < n; v++) T.clusters[v] = T.nb[v] | (1ULL << v);
    for (int i = 0; i < n; i++) {
        const vs_t pin = T.nb[i];
        int parents[64], np = 0;
        for (int j = 0; j < n; j++)
            if ((pin >> j) & 1ULL) parents[np++] = j;
        int unc[65], nu = 0;
        for (int j = 0; j < np; j++) unc[nu++] = parents[j];
        if (nu == 1 && np > 1) {
            for (int m = 0; m < np; m++)
                if (parents[m] != unc[0]) { unc[nu++] = parents[m]; break; }
        } else if (nu == 1 && np == 1 && i < parents[0] && popc64(T.nb[parents[0]]) == 1) {
            const int vj = unc[0];
            int64_t b;
            (void)spl_get(s, i, 1ULL << vj, &b);
            const vs_t thep = (b < s->spl[i].count) ? s->spl[i].parents[b] : 0;
            if (thep == (1ULL << vj)) { DG(&T, i, vj) = 1; DG(&T, vj, i) = 1; }
        }
        for (int j = 0; j < nu; j++) {
            const int vj = unc[j];
            for (int k = 0; k < j; k++) {
                const int vk = unc[k];
                process_triple(&T, i, vj, vk);
                if (!((T.nb[vj] >> vk) & 1ULL) && (DG(&T, vj, vk) || DG(&T, vk, vj))) trip_add_edge(&T, vj, vk);
            }
        }
    }
    /* unfaithful-edge fixpoint (triplet_astar.cpp:1256-1290) */
    int delta;
    do {
        delta = 0;
        for (int i = 0; i < n; i++) {
            for (int j = 0; j < i; j++) {
                const int unfaithful = (DG(&T, i, j) || DG(&T, j, i)) && 0 == ((T.nb[i] >> j) & 1ULL);
                delta += unfaithful;
                if (!unfaithful) continue;
                trip_add_edge(&T, i, j);
                for (int k = 0; k < n; k++)
                    if (k != i && k != j && (((T.clusters[i] >> k) & 1ULL) || ((T.clusters[j] >> k) & 1ULL)))
                        process_triple(&T, i, j, k);
            }
        }
    } while (delta > 0);
    /* Meek rules 2, 3, 4 until nothing changes (triplet_astar.cpp:1297-1478) */
    for (int iter = 0; iter < n; iter++) {
        int num_oriented = 0;
        for (int v = 0; v < n; v++) { /* rule 2 */
            int ins[64], outs[64], ni = 0, no = 0;
            for (int j = 0; j < n; j++) {
                if (1 == DG(&T, v, j) && 0 == DG(&T, j, v)) outs[no++] = j;
                else if (1 == DG(&T, j, v) && 0 == DG(&T, v, j)) ins[ni++] = j;
            }
            if (ni == 0 || no == 0) continue;
            for (int a = 0; a < ni; a++)
                for (int b = 0; b < no; b++) {
                    const int parent = ins[a], child = outs[b];
                    if (DG(&T, parent, child) && DG(&T, child, parent)) {
                        DG(&T, parent, child) = 1; DG(&T, child, parent) = 0; num_oriented++;
                    }
                }
        }
        for (int v = 0; v < n; v++) { /* rule 3 */
            const int num_vps = popc64(T.vstr_parents[v]);
            int vp[64], und[64], nvp = 0, nun = 0;
            for (int j = 0; j < n; j++) {
                if ((T.vstr_parents[v] >> j) & 1ULL) vp[nvp++] = j;
                if (1 == DG(&T, v, j) && 1 == DG(&T, j, v)) und[nun++] = j;
            }
            if (num_vps < 2 || nun == 0) continue;
            for (int a = 0; a < nun; a++) {
                const int neighbor = und[a];
                int cnt = 0;
                for (int b = 0; b < nvp; b++)
                    if (1 == DG(&T, vp[b], neighbor) && 1 == DG(&T, neighbor, vp[b])) cnt++;
                if (cnt >= 2) { DG(&T, v, neighbor) = 0; num_oriented++; }
            }
        }
        for (int v = 0; v < n; v++) { /* rule 4 */
            int ins[64], outs[64], und[64], ni = 0, no = 0, nun = 0;
            for (int j = 0; j < n; j++) {
                if (1 == DG(&T, v, j) && 0 == DG(&T, j, v)) outs[no++] = j;
                else if (1 == DG(&T, j, v) && 0 == DG(&T, v, j)) ins[ni++] = j;
                else if (1 == DG(&T, v, j) && 1 == DG(&T, j, v)) und[nun++] = j;
            }
            if (no == 0 || ni == 0 || nun == 0) continue;
            for (int a = 0; a < nun; a++) {
                const int neighbor = und[a];
                int nd = 0;
                for (int b = 0; b < ni; b++)
                    if (1 == DG(&T, neighbor, ins[b]) && 1 == DG(&T, ins[b], neighbor)) nd++;
                if (nd == 0) continue;
                for (int b = 0; b < no; b++) {
                    const int child = outs[b];
                    if (0 == DG(&T, neighbor, child) || 0 == DG(&T, child, neighbor)) continue;
                    num_oriented++;
                    DG(&T, child, neighbor) = 0;
                }
            }
        }
        if (num_oriented == 0) break;
    }
    if (astar_runs) *astar_runs = T.runs;
    if (distinct_runs) *distinct_runs = T.distinct_runs;
    if (expanded) *expanded = T.expanded;
    omap_free(&T.triplets_checked);
    omap_free(&T.memo);
    free(T.memo_op); free(T.memo_oc);
    free(T.nb); free(T.clusters); free(T.vstr_parents);
    return T.hang ? 2 : 0;
}

/* ---- calc_dag_score (astar/calc_dag_score.cpp) ------------------------------ */
void ora_dag_score(ora_search *s, int variableCount, int nrows, const ora_varset *rows, float *total,
                   float *alt, int *num_edges, int *remove, int *remove_alt) {
    vs_t alt_parents[64];
    int edges[64][64];
    for (int i = 0; i < 64; i++) {
        alt_parents[i] = 0;
        for (int j = 0; j < 64; j++) edges[i][j] = 0;
    }
    float t = 0.0f, a = 0.0f;
    int rm = 0, rma = 0;
    for (int v = 0; v < nrows; v++) {
        const vs_t parents = rows[v];
        for (int j = 0; j < 64; j++)
            if ((parents >> j) & 1ULL) {
                alt_parents[j] |= 1ULL << v;
                edges[v][j] = 1;
                edges[j][v] = 1;
            }
        if (s) {
            int64_t b;
            t += spl_get(s, v, parents, &b);
            const vs_t opt = (b < s->spl[v].count) ? s->spl[v].parents[b] : 0;
            rm += popc64(parents ^ opt);
        }
    }
    if (s)
        for (int i = 0; i < variableCount; i++) {
            int64_t b;
            a += spl_get(s, i, alt_parents[i], &b);
            const vs_t opt = (b < s->spl[i].count) ? s->spl[i].parents[b] : 0;
            rma += popc64(alt_parents[i] ^ opt);
        }
    int ne = 0;
    for (int i = 0; i < variableCount; i++)
        for (int j = i + 1; j < variableCount; j++) ne += edges[i][j];
    *total = t;
    *alt = a;
    *num_edges = ne;
    *remove = rm;
    *remove_alt = rma;
}
