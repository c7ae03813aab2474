// search_internal.h -- state and device helpers of the search side
// (best-score tables, pattern database, A*).
#pragma once

#include <cfloat>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "ulg_internal.h"

namespace ulg {

constexpr int kMaxGroups = 8;

// ---- device helpers ----------------------------------------------------------
__host__ __device__ inline uint64_t pext64(uint64_t x, uint64_t m) {
    uint64_t r = 0;
    int k = 0;
    while (m) {
        const uint64_t b = m & (0 - m);
        if (x & b) r |= 1ull << k;
        ++k;
        m ^= b;
    }
    return r;
}

// float -> uint32 whose unsigned order is the float order; -0 folds onto +0 so
// that ties between signed zeros fall to the file index, as in the reference's
// float compare (sparse_parent_list.cpp:7-9).
__host__ __device__ inline uint32_t ordkey(float f) {
    if (f == 0.0f) f = 0.0f;
    uint32_t u;
#ifdef __HIP_DEVICE_COMPILE__
    u = __float_as_uint(f);
#else
    __builtin_memcpy(&u, &f, 4);
#endif
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// inverse of ordkey; 0xFFFFFFFF (no stored subset) reads as FLT_MAX.  (Only
// the NaN 0x7FFFFFFF maps there too.)
__host__ __device__ inline float ord_cost(uint32_t k) {
    if (k == 0xFFFFFFFFu) return FLT_MAX;
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    float f;
#ifdef __HIP_DEVICE_COMPILE__
    f = __uint_as_float(u);
#else
    __builtin_memcpy(&f, &u, 4);
#endif
    return f;
}

__host__ __device__ inline float key_cost(uint64_t key) {
    if (key == ~0ull) return FLT_MAX;  // no stored subset: getScore returns FLT_MAX
    const uint32_t k = (uint32_t)(key >> 32);
    const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    float f;
#ifdef __HIP_DEVICE_COMPILE__
    f = __uint_as_float(u);
#else
    __builtin_memcpy(&f, &u, 4);
#endif
    return f;
}

// The .pss "%f" + atof round trip (score_main.cpp:191, score_cache.cpp:151):
// D = round-half-even(|x| * 10^6) in exact integers (glibc printf is exact,
// ties to even); strtod(D / 10^6) is the correctly rounded double quotient;
// cost = float(-1 * value).
__host__ __device__ inline float quantize_score(float x) {
    uint32_t u;
#ifdef __HIP_DEVICE_COMPILE__
    u = __float_as_uint(x);
#else
    __builtin_memcpy(&u, &x, 4);
#endif
    const uint32_t ex = (u >> 23) & 0xffu;
    const bool neg = (u >> 31) != 0;
    if (ex == 0xffu) return -x;  // inf -> -inf; nan stays nan
    uint64_t M;
    int E;
    if (ex == 0) { M = u & 0x7fffffu; E = -149; }
    else { M = (u & 0x7fffffu) | 0x800000u; E = (int)ex - 150; }
    double mag;
    if (E >= 0) {
        mag = neg ? -(double)x : (double)x;  // x * 10^6 is an integer: printed exactly
    } else {
        const int sh = -E;
        const uint64_t num = M * 1000000ull;  // < 2^44
        uint64_t D;
        if (sh >= 64) D = 0;
        else {
            D = num >> sh;
            const uint64_t rem = num & ((1ull << sh) - 1ull);
            const uint64_t half = 1ull << (sh - 1);
            if (rem > half || (rem == half && (D & 1ull))) ++D;
        }
        mag = (double)D / 1000000.0;
    }
    const double val = neg ? -mag : mag;
    return (float)(-1.0 * val);
}

// device view of the search tables (passed by value to kernels)
struct SearchDev {
    const uint32_t *table;   // ordered cost (ordkey) of the best stored subset, per subset of D_v
    const uint64_t *tb_off;  // [n+1]
    const uint64_t *support; // D_v
    const uint64_t *sets;    // per-variable lists, file order
    const int64_t *offsets;  // [n+1]
    const float *costs;      // per-variable costs, file order
    const float *pd;         // pattern databases
    const uint64_t *gmeta;   // groups[kMaxGroups], pd_off[kMaxGroups]
    uint64_t scope;          // the tables hold every stored set inside scope
    uint64_t table_vars;     // variables that have a table (all but in the sharded sweep)
    int tables;              // 1 if the tables are built (for scope)
    int pd_count;
    int n;
};

// The list calculator's answer by a scan of v's list (sparse_parent_list.cpp:
// 44-55 with the (cost, file order) tie rule): min over stored P subset of S.
__device__ inline uint64_t bs_key_scan(const SearchDev &d, int v, uint64_t S) {
    const int64_t b = d.offsets[v], e = d.offsets[v + 1];
    uint64_t best = ~0ull;
    for (int64_t i = b; i < e; ++i)
        if ((d.sets[i] & ~S) == 0) {
            const uint64_t k = ((uint64_t)ordkey(d.costs[i]) << 32) | (uint64_t)(i - b);
            best = k < best ? k : best;
        }
    return best;
}

// pext over the set bits of x (x a subset of m): |x| steps instead of |m|
__device__ inline uint64_t pext_sparse(uint64_t x, uint64_t m) {
    uint64_t r = 0;
    for (uint64_t y = x; y; y &= y - 1) r |= 1ull << __popcll(m & ((y & (0 - y)) - 1));
    return r;
}

// index of S in v's table: pext(S & D_v, D_v); a full skeleton's
// D_v = every variable but v closes the hole at v with two shifts
__device__ inline uint64_t bs_index(const SearchDev &d, int v, uint64_t S) {
    const uint64_t D = d.support[v];
    const uint64_t x = S & D;
    const uint64_t all = (d.n >= 64) ? ~0ull : ((1ull << d.n) - 1ull);
    const uint64_t lo = (1ull << v) - 1ull;
    return D == (all & ~(1ull << v)) ? (((v < 63 ? (x >> (v + 1)) : 0ull) << v) | (x & lo)) : pext_sparse(x, D);
}

// getScore(v, S): one 4-B read of the lattice when v has a table and S lies
// inside the tables' scope (every stored set that can be a subset of S is in
// the table), else the list scan.
__device__ inline float bs_cost(const SearchDev &d, int v, uint64_t S) {
    if (d.tables && (S & ~d.scope) == 0 && ((d.table_vars >> v) & 1ull))
        return ord_cost(d.table[d.tb_off[v] + bs_index(d, v, S)]);
    return key_cost(bs_key_scan(d, v, S));
}

// StaticPatternDatabase::h (static_pattern_database.cpp:145-174)
__device__ inline float pdb_h(const SearchDev &d, uint64_t S, int *complete) {
    const uint64_t mask = (d.n >= 64) ? ~0ull : ((1ull << d.n) - 1ull);
    const uint64_t remaining = ~S & mask;
    float h = 0.0f;
    for (int g = 0; g < d.pd_count; ++g) {
        const uint64_t grp = d.gmeta[g];
        const uint64_t vs = grp & remaining;
        const float val = d.pd[d.gmeta[kMaxGroups + g] + pext64(vs, grp)];
        if (vs == remaining) {
            *complete = 1;
            return val;
        }
        h += val;
    }
    return h;
}

// ---- host memory for the exact-order search -------------------------------------
// Anonymous mapping with transparent huge pages requested (the replay's
// random reads into GB-sized arrays would otherwise miss the TLB on almost
// every access); optionally page-locked for the device copies.  Pages are
// zero until touched.
struct HostHuge {
    void *p = nullptr;
    size_t bytes = 0;
    bool pinned = false;
    // (re)maps at least `want` bytes; returns false if the mapping fails
    bool reserve(size_t want, bool pin);
    void zero_prefix(size_t n);  // memset the first n bytes
    void release();
    ~HostHuge() { release(); }
};

// ---- host state -----------------------------------------------------------------
struct SearchState {
    int n = 0;
    std::vector<int64_t> offsets;  // [n+1] host copy
    DevBuf<uint64_t> d_sets;
    DevBuf<float> d_costs, d_scores_tmp;
    DevBuf<int64_t> d_offsets;
    // best-score tables
    std::vector<uint64_t> support, tb_off;
    std::vector<int> mbits;
    uint64_t table_entries = 0;
    DevBuf<uint32_t> d_table;      // ordkey(best cost) per subset of D_v
    DevBuf<uint64_t> d_tb_off, d_support;
    DevBuf<uint64_t> e_idx, e_idx2;  // sorted (table index, key) of the stored sets
    DevBuf<uint32_t> e_key, e_key2;
    DevBuf<unsigned char> sort_tmp;
    DevBuf<int> d_mbits, d_prefix;
    bool lists_ready = false;   // the per-variable lists are on the device
    bool tables_ready = false;  // the lattice tables are built for `scope`
    uint64_t scope = 0;         // tables cover every stored set inside scope
    uint64_t table_vars = 0;    // variables with a table (every variable, except for ulg_sweep_shard_*)
    // host copy of the per-subset best costs (exact-order search)
    DevBuf<float> d_cost_table;
    float *host_costs = nullptr;
    uint64_t host_cost_cap = 0;
    bool host_costs_ready = false;
    // exact-order search: one row of successor costs per subset of the scope,
    // row[pext(S, scope)][i] = getScore(scc_i, S) (FLT_MAX for scc_i in S)
    HostHuge host_rows;        // nl words per row: the successor costs (search.hip cost_rows_kernel)
    DevBuf<float> d_rows;      // device staging for the row chunks
    DevBuf<int> d_rowmeta;     // scope bit positions, scc variables
    uint64_t rows_scope = 0, rows_scc = 0;
    bool rows_ready = false;
    // GPU sweep: the component's successor costs in the sweep's own order,
    // sweep_w[j][p][colex rank of P among the (m-1)-subsets of comp \ {v_j}]
    // = getScore(v_j, P), |P| = p (one contiguous slice per variable and layer)
    DevBuf<float> d_sweep_w;
    // GPU sweep scratch, kept across calls
    DevBuf<uint64_t> gs_bn, gs_edges, gs_layer_off;
    DevBuf<int> gs_cv, gs_chain;
    DevBuf<float> gs_g0, gs_g1;
    DevBuf<uint8_t> gs_leaf;
    DevBuf<unsigned long long> gs_acc;
    uint64_t sweep_comp = 0;
    bool sweep_ready = false;
    // variable-sharded sweep (ulg_sweep_shard_*): this rank's tables and
    // sweep slices cover `shard_own`; the layers' g and leaf bytes are the
    // all-reduced ones
    bool shard_active = false;
    uint64_t shard_own = 0;
    int shard_layer = 0;
    DevBuf<float> shard_g0, shard_g1;
    DevBuf<uint8_t> shard_leaf;
    DevBuf<uint64_t> shard_bn, shard_loff;
    DevBuf<int> shard_wslot, shard_cv, shard_chain;
    DevBuf<unsigned long long> shard_acc;
    // pattern database
    int pd_count = 0;
    uint64_t ancestors = 0, scc = 0;
    std::vector<uint64_t> groups, pd_off;
    std::vector<float> pd_host;
    DevBuf<float> d_pd, d_bsv;
    DevBuf<int> d_bitpos;
    DevBuf<uint64_t> d_groups;
    bool pdb_ready = false;
    // triplet_astar's per-cluster A* results (cluster -> optimal parent set
    // per variable), valid for these lists and triplet_pd; filled by the
    // driver, by ulg_triplet_solve and by ulg_triplet_memo_put (other ranks)
    std::unordered_map<uint64_t, std::vector<uint64_t>> triplet_memo;
    int triplet_pd = 0;
    // query scratch
    DevBuf<int> q_vars;
    DevBuf<uint64_t> q_sets, q_par;
    DevBuf<float> q_costs;

    SearchDev dev() const {
        SearchDev d;
        d.table = d_table.p;
        d.tb_off = d_tb_off.p;
        d.support = d_support.p;
        d.sets = d_sets.p;
        d.offsets = d_offsets.p;
        d.costs = d_costs.p;
        d.scope = scope;
        d.table_vars = table_vars;
        d.tables = tables_ready ? 1 : 0;
        d.pd = d_pd.p;
        d.gmeta = d_groups.p;
        d.pd_count = pd_count;
        d.n = n;
        return d;
    }
    void release_all() {
        release(d_sets); release(d_costs); release(d_scores_tmp); release(d_offsets);
        release(d_table); release(d_tb_off); release(d_support); release(d_mbits); release(d_prefix);
        release(e_idx); release(e_key); release(e_idx2); release(e_key2); release(sort_tmp);
        release(d_cost_table); release(d_pd); release(d_bsv); release(d_bitpos); release(d_groups);
        release(q_vars); release(q_sets); release(q_par); release(q_costs);
        if (host_costs) (void)hipHostFree(host_costs);
        host_costs = nullptr;
        release(d_rows); release(d_rowmeta);
        release(d_sweep_w);
        sweep_ready = false;
        release(gs_bn); release(gs_edges); release(gs_layer_off); release(gs_cv); release(gs_chain);
        release(gs_g0); release(gs_g1); release(gs_leaf); release(gs_acc);
        release(shard_g0); release(shard_g1); release(shard_leaf); release(shard_bn); release(shard_loff);
        release(shard_wslot); release(shard_cv); release(shard_chain); release(shard_acc);
        shard_active = false;
        host_rows.release();
        rows_ready = false;
        host_cost_cap = 0;
    }
};

// Builds the lattice tables over the stored sets inside `scope`; returns
// ULG_ERR_UNSUPPORTED (tables untouched) if they would exceed the budget.
int search_build_tables(ulg_ctx *c, uint64_t scope, uint64_t tvars = ~0ull);
// Tables covering `need` (rebuilt for exactly `need` if the current ones do not).
int search_ensure_scope(ulg_ctx *c, uint64_t need);
int search_build_pdb(ulg_ctx *c, int pd_count, uint64_t ancestors, uint64_t scc);
int search_quantize_device(ulg_ctx *c, const float *d_scores, float *d_costs, int64_t count);
int search_cost_table_host(ulg_ctx *c);
// row table (SearchState::host_rows) for the dense exact-order search over
// scope = ancestors | scc; the tables must cover scope
// deadline_ns (steady_clock nanoseconds since its epoch, 0 = none): checked
// before every chunk of rows; past it the build stops, the rows stay
// unbuilt and *timed_out is set (the -r budget covers this preprocessing)
int search_cost_rows_host(ulg_ctx *c, uint64_t scope, uint64_t scc, int64_t deadline_ns = 0,
                          bool *timed_out = nullptr);
int search_query(ulg_ctx *c, int64_t count, const int *vars, const uint64_t *S, float *costs, uint64_t *parents);
int search_pdb_query(ulg_ctx *c, int64_t count, const uint64_t *S, float *h, int *complete);

}  // namespace ulg
