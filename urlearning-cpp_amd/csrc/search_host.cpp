// search_host.cpp -- C ABI of the search side and the exact-order A*.
//
// Exact-order mode (ULG_ASTAR_EXACT) replays the reference's sequential
// search -- run_astar_on_one_scc (astar/astar_main.cpp:216-546) with its
// libstdc++-derived heap (priority_queue/priority_queue-inl.h:19-234) and the
// epsilon/depth comparator (base/node.h:124-135) -- on the host, because the
// DAG the reference returns is decided by that heap's pop order among
// float-tied Markov-equivalent orders.  Every per-successor
// lookup it needs is O(1) on tables the GPU built: getScore() is one read of
// the best-score lattice (instead of the reference's linear scan of the
// sorted list, sparse_parent_list.cpp:44-55) and h() two reads of the
// pattern databases.  Parent sets for the reconstruction come from the device
// query kernel.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <x86intrin.h>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "search_exact.h"

using namespace ulg;
using namespace ulg::exact;

namespace {


// connected components of the skeleton (skeleton.cpp:187-230), discovery order
int components(const uint64_t *edges, int n, std::vector<uint64_t> &out) {
    out.clear();
    uint64_t visited = 0;
    for (int v = 0; v < n; ++v) {
        if ((visited >> v) & 1ull) continue;
        uint64_t comp = 0;
        std::vector<int> stack{v};
        visited |= 1ull << v;
        comp |= 1ull << v;
        while (!stack.empty()) {
            const int cur = stack.back();
            stack.pop_back();
            for (int i = 0; i < n; ++i)
                if (!((visited >> i) & 1ull) && ((edges[cur] >> i) & 1ull)) {
                    visited |= 1ull << i;
                    comp |= 1ull << i;
                    stack.push_back(i);
                }
        }
        out.push_back(comp);
    }
    return (int)out.size();
}

struct ExactResult {
    bool found = false;
    float goal_g = 0.0f;
    std::vector<int> total;
    std::vector<uint64_t> opt;
};

// run_astar_on_one_scc (astar_main.cpp:216-546)
using Clock = std::chrono::steady_clock;

int astar_one(ulg_ctx *c, const HostTables &T, const uint64_t *edges, bool skeleton_good, uint64_t ancestors,
              uint64_t the_scc, int64_t *expanded, bool *hang, ExactResult &res, const Clock::time_point *deadline) {
    const int n = T.n;
    std::vector<Node> nodes;
    nodes.reserve(1 << 16);
    SubsetIndex generated;
    generated.init(ancestors | the_scc);
    Heap open;
    open.nodes = &nodes;
    const uint64_t r1 = the_scc >> 1;
    nodes.push_back(Node{0.0f, 0.0f, ancestors, (uint8_t)(r1 ? __builtin_ctzll(r1) + 1 : 0), 0});
    open.push(0);
    int64_t goal = -1;
    const uint64_t allVariables = ancestors | the_scc;
    const float upperBound = FLT_MAX;
    int64_t nexp = 0;
    // ULG_EXACT_PROF=1: cycle split of the replay (pop / successor loop /
    // pushes / updates) on stderr -- diagnostics only
    static const bool prof = std::getenv("ULG_EXACT_PROF") != nullptr;
    uint64_t c_pop = 0, c_succ = 0, c_push = 0, c_upd = 0, t0 = 0, t1 = 0;
    int64_t n_push = 0, n_upd = 0, n_succ = 0, n_closed = 0;
    while (!open.empty()) {
        // the -r watchdog (astar_main.cpp:135-138,266): the loop ends without a goal
        if (deadline && (nexp & 4095) == 0 && Clock::now() > *deadline) {
            c->out_of_time = 1;
            break;
        }
        if (prof) t0 = __rdtsc();
        const uint32_t ui = open.pop();
        if (prof) { t1 = __rdtsc(); c_pop += t1 - t0; }
        ++nexp;
        const uint64_t variables = nodes[ui].sub;
        if (variables == allVariables) { goal = ui; break; }
        if (nodes[ui].g + nodes[ui].h > upperBound) break;
        nodes[ui].pq = -2;
        const float ug = nodes[ui].g;
        // the successors' index slots and lattice entries are independent
        // cache misses: issue them all before the first use
        // (bs(leaf, S u {leaf}) and bs(leaf, S) share one entry: leaf is
        // never in its own support)
        uint64_t leaves = the_scc & ~variables;
        if (skeleton_good && variables != 0)
            for (uint64_t x = leaves; x; x &= x - 1) {
                const int leaf = __builtin_ctzll(x);
                if ((variables & edges[leaf]) == 0) leaves &= ~(1ull << leaf);
            }
        for (uint64_t x = leaves; x; x &= x - 1) {
            const int leaf = __builtin_ctzll(x);
            generated.prefetch(variables | (1ull << leaf));
            T.prefetch_bs(leaf, variables);
        }
        for (uint64_t x = leaves; x; x &= x - 1) {
            const int leaf = __builtin_ctzll(x);
            const uint64_t nv = variables | (1ull << leaf);
            const int64_t si = generated.find(nv);
            if (si < 0) {
                const float leaf_score = T.bs(leaf, nv);
                const float g = ug + leaf_score;
                bool complete = false;
                const float h = T.h(nv, &complete);
                const uint32_t idx = (uint32_t)nodes.size();
                nodes.push_back(Node{g, h, nv, (uint8_t)leaf, 0});
                uint64_t tp = 0;
                if (prof) tp = __rdtsc();
                open.push(idx);
                if (prof) { c_push += __rdtsc() - tp; ++n_push; }
                generated.insert(nv, idx);
                continue;
            }
            if (nodes[si].pq == -2) { if (prof) ++n_closed; continue; }
            const float g = ug + T.bs(leaf, variables);
            if (g < nodes[si].g) {
                nodes[si].leaf = (uint8_t)leaf;
                nodes[si].g = g;
                uint64_t tu = 0;
                if (prof) tu = __rdtsc();
                open.update((uint32_t)si);
                if (prof) { c_upd += __rdtsc() - tu; ++n_upd; }
            }
        }
        if (prof) { c_succ += __rdtsc() - t1; n_succ += __builtin_popcountll(leaves); }
    }
    if (prof)
        std::fprintf(stderr,
                     "exact_prof expanded=%lld successors=%lld pushes=%lld updates=%lld closed_hits=%lld "
                     "heap_peak=%zu | Gcycles pop=%.3f succ_loop=%.3f (push %.3f, update %.3f) stale_scans=%lld\n",
                     (long long)nexp, (long long)n_succ, (long long)n_push, (long long)n_upd, (long long)n_closed,
                     open.a.size(), c_pop * 1e-9, c_succ * 1e-9, c_push * 1e-9, c_upd * 1e-9,
                     (long long)open.scans);
    *expanded += nexp;
    if (open.hang) *hang = true;
    if (goal < 0) return ULG_OK;
    // reconstructSolution (astar_main.cpp:140-166)
    const int count = __builtin_popcountll(the_scc);
    res.total.assign(n, 0);
    res.opt.assign(n, 0);
    std::vector<int> qv;
    std::vector<uint64_t> qs;
    std::vector<int> pos;
    uint64_t remaining = nodes[goal].sub;
    int64_t cur = goal;
    for (int i = 0; i < count && cur >= 0; ++i) {
        const int leaf = nodes[cur].leaf;
        res.total[count - 1 - i] = leaf;
        qv.push_back(leaf);
        qs.push_back(remaining);
        pos.push_back(count - 1 - i);
        remaining ^= 1ull << leaf;
        cur = generated.find(remaining);
    }
    if (!qv.empty()) {
        std::vector<float> qc(qv.size());
        std::vector<uint64_t> qp(qv.size());
        int rc = search_query(c, (int64_t)qv.size(), qv.data(), qs.data(), qc.data(), qp.data());
        if (rc) return rc;
        for (size_t i = 0; i < qv.size(); ++i) res.opt[pos[i]] = qp[i];
    }
    res.found = true;
    res.goal_g = nodes[goal].g;
    return ULG_OK;
}

// ---- the dense form of the same replay ---------------------------------------
// Scopes of at most kDenseScopeBits variables: every node of the order lattice
// has a fixed home, recs[pext(S, scope)] (16 B: g, h, the reference's pqPos,
// leaf), so a successor is one random access that can be prefetched together
// with its siblings', and the popped node's successor costs are one
// contiguous row (search_cost_rows_host) instead of one lattice read per
// successor.  Heap entries are (f, slot), 8 B; a node's layer is
// popcount(slot), as pext keeps the bit count.  The heap algorithms,
// comparator, first-generator-wins and no-reopen rule are exactly Heap's
// (search_exact.h) and the reference's.
constexpr int kDenseScopeBits = 26;
constexpr uint64_t kDenseRowsMaxBytes = 8ull << 30;

inline bool dense_eligible(uint64_t scope, uint64_t scc) {
    const int m = __builtin_popcountll(scope);
    return m <= kDenseScopeBits && ((1ull << m) * (uint64_t)__builtin_popcountll(scc) * 4) <= kDenseRowsMaxBytes;
}

// run_astar_on_one_scc (astar_main.cpp:216-546) over dense node homes; HeapT:
// the reference's heap in the flat (DenseHeap) or pair-block (BlockedHeap,
// ULG_EXACT_PF bit 8) physical layout -- same pops, same pqPos
template <class HeapT>
int astar_dense_t(ulg_ctx *c, const HostTables &T, const uint64_t *edges, bool skeleton_good, uint64_t ancestors,
                  uint64_t the_scc, int64_t *expanded, bool *hang, ExactResult &res, const Clock::time_point *deadline) {
    SearchState &s = *c->search;
    const int n = T.n;
    const uint64_t scope = ancestors | the_scc;
    const int m = __builtin_popcountll(scope);
    const uint64_t nslots = 1ull << m;
    const int nl = __builtin_popcountll(the_scc);
    const uint64_t W = (uint64_t)nl;  // row: the nl successor costs (search_cost_rows_host)
    const float *rows = static_cast<const float *>(s.host_rows.p);
    HostHuge recmem, heapmem;
    // the heap's buffer starts 8 B into a line, so a node's two children
    // (2i+1, 2i+2) share 16 aligned bytes and its 16 great-great-grandchildren
    // two lines
    constexpr bool kBlocked = HeapT::Layout::kBlocked;
    const uint64_t heap_entries =
        kBlocked ? (uint64_t)PairBlockLayout::capacity((int64_t)nslots + 16) : nslots + 16;
    if (!recmem.reserve(nslots * sizeof(DenseRec), false) || !heapmem.reserve(heap_entries * sizeof(DEnt), false))
        return set_err(c, ULG_ERR_HIP, "cannot map the dense search arrays");
    DenseRec *recs = static_cast<DenseRec *>(recmem.p);
    HeapT open;
    open.recs = recs;
    // flat: 8 B into a line (siblings share 16 aligned bytes); blocked: line-aligned blocks
    open.a = static_cast<DEnt *>(heapmem.p) + (kBlocked ? 0 : 1);
    // Prefetch modes (ULG_EXACT_PF, default 6, A/B only): bit 1, the pop also
    // prefetches 5 heap levels ahead (C3 17.6 -> 16.8 s on the box's EPYC
    // 9575F); bit 2, the heap top's successor records and cost row are
    // prefetched before its pop, so they arrive while the pop descends the
    // heap (C3 16.9 -> 14.0 s, 2 alternating A/B runs).  Every other layout
    // or prefetch tried was no faster and is gone.
    const int pfmode = std::getenv("ULG_EXACT_PF") ? std::atoi(std::getenv("ULG_EXACT_PF")) : 6;
    open.pf5 = (pfmode & 2) != 0;
    open.pfdeep = (pfmode & 512) != 0;  // blocked layout: the grandchildren's blocks too

    // slot bit of each variable, and its column in the row table
    uint32_t sbit[64] = {0};
    int col[64];
    for (int v = 0; v < 64; ++v) col[v] = -1;
    {
        int i = 0;
        for (uint64_t x = scope; x; x &= x - 1) sbit[__builtin_ctzll(x)] = 1u << i++;
        i = 0;
        for (uint64_t x = the_scc; x; x &= x - 1) col[__builtin_ctzll(x)] = i++;
    }
    auto slot_of = [&](uint64_t S) { return (uint32_t)(g_have_bmi2 ? pext_bmi2(S, scope) : pext64(S, scope)); };
    const uint32_t root = slot_of(ancestors), goal_slot = (uint32_t)(nslots - 1);
    const uint64_t r1 = the_scc >> 1;
    recs[root] = DenseRec{0.0f, 0.0f, 0, (uint8_t)(r1 ? __builtin_ctzll(r1) + 1 : 0), {0, 0, 0}};
    open.push(root);
    int64_t goal = -1;
    const float upperBound = FLT_MAX;
    int64_t nexp = 0;
    static const bool prof = std::getenv("ULG_EXACT_PROF") != nullptr;
    uint64_t c_pop = 0, c_succ = 0, t0 = 0, t1 = 0;
    uint64_t pop_hist[64][2] = {};  // pop cycles by log2(heap length)
    int64_t n_push = 0, n_upd = 0, n_succ = 0;
    while (open.len > 0) {
        if (deadline && (nexp & 4095) == 0 && Clock::now() > *deadline) {
            c->out_of_time = 1;
            break;
        }
        if (prof) t0 = __rdtsc();
        const int64_t hl = open.len;
        if (pfmode & 4) {
            // the node about to be popped is already known (the heap top):
            // its successor records and cost row are fetched while the pop
            // descends the heap, instead of after it
            const uint32_t top = open.A(0).slot();
            const uint64_t tv = g_have_bmi2 ? pdep_bmi2(top, scope) : pdep64(top, scope);
            const float *trow = rows + (uint64_t)top * W;
            __builtin_prefetch(trow);
            __builtin_prefetch(trow + W - 1);
            for (uint64_t x = the_scc & ~tv; x; x &= x - 1) __builtin_prefetch(&recs[top | sbit[__builtin_ctzll(x)]], 1);
        }
        const uint32_t ui = open.pop();
        if (prof) {
            t1 = __rdtsc();
            c_pop += t1 - t0;
            const int b = 63 - __builtin_clzll((uint64_t)hl | 1ull);
            pop_hist[b][0] += t1 - t0;
            pop_hist[b][1] += 1;
        }
        ++nexp;
        if (ui == goal_slot) { goal = ui; break; }
        DenseRec &U = recs[ui];
        if (U.g + U.h > upperBound) break;
        U.pq = -1;
        const float ug = U.g;
        const uint64_t variables = g_have_bmi2 ? pdep_bmi2(ui, scope) : pdep64(ui, scope);
        uint64_t leaves = the_scc & ~variables;
        if (skeleton_good && variables != 0)
            for (uint64_t x = leaves; x; x &= x - 1) {
                const int leaf = __builtin_ctzll(x);
                if ((variables & edges[leaf]) == 0) leaves &= ~(1ull << leaf);
            }
        const float *row = rows + (uint64_t)ui * W;
        if (!(pfmode & 4)) {
            __builtin_prefetch(row);
            __builtin_prefetch(row + W - 1);
            for (uint64_t x = leaves; x; x &= x - 1) __builtin_prefetch(&recs[ui | sbit[__builtin_ctzll(x)]], 1);
        }
        for (uint64_t x = leaves; x; x &= x - 1) {
            const int leaf = __builtin_ctzll(x);
            const uint32_t si = ui | sbit[leaf];
            DenseRec &R = recs[si];
            // getScore(leaf, S u {leaf}) == getScore(leaf, S): leaf is never in its own sets
            const float g = ug + row[col[leaf]];
            if (R.pq == 0) {
                bool complete = false;
                R.g = g;
                R.h = T.h(variables | (1ull << leaf), &complete);
                R.leaf = (uint8_t)leaf;
                open.push(si);
                if (prof) ++n_push;
                continue;
            }
            if (R.pq == -1) continue;
            if (g < R.g) {
                R.leaf = (uint8_t)leaf;
                R.g = g;
                open.update(si);
                if (prof) ++n_upd;
            }
        }
        if (prof) { c_succ += __rdtsc() - t1; n_succ += __builtin_popcountll(leaves); }
    }
    if (prof)
        std::fprintf(stderr,
                     "exact_prof(dense) expanded=%lld successors=%lld pushes=%lld updates=%lld heap_peak=%lld | "
                     "Gcycles pop=%.3f succ_loop=%.3f stale_scans=%lld\n",
                     (long long)nexp, (long long)n_succ, (long long)n_push, (long long)n_upd, (long long)open.hwm,
                     c_pop * 1e-9, c_succ * 1e-9, (long long)open.scans);
    if (prof) {  // are the records and heap on huge pages?  (THP can be off on a box)
        if (FILE *f = std::fopen("/proc/self/smaps_rollup", "r")) {
            char line[256];
            while (std::fgets(line, sizeof line, f))
                if (std::strncmp(line, "AnonHugePages", 13) == 0 || std::strncmp(line, "Rss:", 4) == 0)
                    std::fprintf(stderr, "exact_prof(dense) %s", line);
            std::fclose(f);
        }
    }
    if (prof)
        for (int b = 0; b < 64; ++b)
            if (pop_hist[b][1])
                std::fprintf(stderr, "exact_prof(dense) pops with heap 2^%d: %llu, %.0f cycles each\n", b,
                             (unsigned long long)pop_hist[b][1], (double)pop_hist[b][0] / (double)pop_hist[b][1]);
    *expanded += nexp;
    if (open.hang) *hang = true;
    if (goal < 0) return ULG_OK;
    // reconstructSolution (astar_main.cpp:140-166)
    const int count = nl;
    res.total.assign(n, 0);
    res.opt.assign(n, 0);
    std::vector<int> qv;
    std::vector<uint64_t> qs;
    std::vector<int> pos;
    // count = |the_scc|: when the skeleton component overlaps the ancestors
    // (-p/-s, astar_main.cpp:629-635) the walk reaches the root before count
    // steps; like the indexed form it stops at the first subnetwork that is
    // not in generatedNodes (the root never is, :236-237)
    uint32_t cur = (uint32_t)goal;
    for (int i = 0; i < count; ++i) {
        const int leaf = recs[cur].leaf;
        res.total[count - 1 - i] = leaf;
        qv.push_back(leaf);
        qs.push_back(g_have_bmi2 ? pdep_bmi2(cur, scope) : pdep64(cur, scope));
        pos.push_back(count - 1 - i);
        cur ^= sbit[leaf];
        if (cur == root || recs[cur].pq == 0) break;  // the root is never in generatedNodes
    }
    if (!qv.empty()) {
        std::vector<float> qc(qv.size());
        std::vector<uint64_t> qp(qv.size());
        int rc = search_query(c, (int64_t)qv.size(), qv.data(), qs.data(), qc.data(), qp.data());
        if (rc) return rc;
        for (size_t i = 0; i < qv.size(); ++i) res.opt[pos[i]] = qp[i];
    }
    res.found = true;
    res.goal_g = recs[goal].g;
    return ULG_OK;
}

int astar_dense(ulg_ctx *c, const HostTables &T, const uint64_t *edges, bool skeleton_good, uint64_t ancestors,
                uint64_t the_scc, int64_t *expanded, bool *hang, ExactResult &res, const Clock::time_point *deadline) {
    const int pfmode = std::getenv("ULG_EXACT_PF") ? std::atoi(std::getenv("ULG_EXACT_PF")) : 6;
    if (pfmode & 256)
        return astar_dense_t<BlockedHeap>(c, T, edges, skeleton_good, ancestors, the_scc, expanded, hang, res,
                                          deadline);
    return astar_dense_t<DenseHeap>(c, T, edges, skeleton_good, ancestors, the_scc, expanded, hang, res, deadline);
}

uint64_t all_vars(int n) { return (n >= 64) ? ~0ull : ((1ull << n) - 1ull); }

// New lists: tables over every variable when they fit the budget; otherwise
// none yet -- searches build tables per component / cluster, and lookups
// outside the tables' scope scan the lists on the device.
int lists_loaded(ulg_ctx *c) {
    SearchState &s = *c->search;
    s.lists_ready = true;
    s.tables_ready = false;
    s.pdb_ready = false;
    s.host_costs_ready = false;
    s.rows_ready = false;
    s.sweep_ready = false;
    s.triplet_memo.clear();
    const int rc = search_build_tables(c, all_vars(s.n));
    if (rc == ULG_ERR_UNSUPPORTED) {
        c->err.clear();
        return ULG_OK;
    }
    return rc;
}

SearchState &state(ulg_ctx *c) {
    if (!c->search) c->search = new SearchState();
    return *c->search;
}

}  // namespace

namespace ulg {
namespace exact {

void host_tables(const SearchState &s, HostTables &T) {
    const int n = s.n;
    const uint64_t all = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    T.cost = s.host_costs;
    T.tb_off = s.tb_off.data();
    T.support = s.support.data();
    T.all = all;
    T.n = n;
    T.hole.assign(n, -1);
    for (int v = 0; v < n; ++v) {
        const uint64_t D = s.support[v];
        const uint64_t miss = ~D & all;
        if (__builtin_popcountll(miss) == 1 && ((D & ~all) == 0)) T.hole[v] = __builtin_ctzll(miss);
    }
    T.pd = s.pd_host.data();
    T.groups = s.groups;
    T.pd_off = s.pd_off;
}

}  // namespace exact

int astar_gpu(ulg_ctx *c, const uint64_t *edges, uint64_t *vpar, int *order, float *goal_cost, int64_t *expanded);

}  // namespace ulg

extern "C" {

int ulg_search_load(ulg_ctx *c, int n, const int64_t *offsets, const uint64_t *sets, const float *costs) {
    if (!c || n < 1 || n > kMaxVars || !offsets || !sets || !costs) return set_err(c, ULG_ERR_ARG, "ulg_search_load: bad arguments");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = state(c);
    s.n = n;
    s.offsets.assign(offsets, offsets + n + 1);
    const int64_t total = offsets[n];
    for (int v = 0; v < n; ++v)
        if (offsets[v + 1] < offsets[v] || offsets[v + 1] - offsets[v] > 0xffffffffll)
            return set_err(c, ULG_ERR_ARG, "ulg_search_load: bad offsets");
    int rc;
    if ((rc = ensure(c, s.d_sets, (size_t)std::max<int64_t>(total, 1))) || (rc = ensure(c, s.d_costs, (size_t)std::max<int64_t>(total, 1))) ||
        (rc = ensure(c, s.d_offsets, (size_t)n + 1)))
        return rc;
    if (total) {
        ULG_HIP(c, hipMemcpyAsync(s.d_sets.p, sets, (size_t)total * 8, hipMemcpyHostToDevice, c->stream));
        ULG_HIP(c, hipMemcpyAsync(s.d_costs.p, costs, (size_t)total * 4, hipMemcpyHostToDevice, c->stream));
    }
    ULG_HIP(c, hipMemcpyAsync(s.d_offsets.p, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return lists_loaded(c);
}

int ulg_search_from_scores(ulg_ctx *c) {
    if (!c) return ULG_ERR_ARG;
    if (c->async_pending) {  // an async scoring call still owns the lists
        const int rc0 = ulg_cbic_score_finish(c, nullptr, nullptr);
        if (rc0) return rc0;
    }
    if (!c->scored) return set_err(c, ULG_ERR_STATE, "ulg_search_from_scores: call ulg_cbic_score first");
    if (c->nv != c->n) return set_err(c, ULG_ERR_STATE, "ulg_search_from_scores: every variable must be scored in this context");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = state(c);
    const int n = c->n;
    std::vector<int64_t> src(n + 1);
    ULG_HIP(c, hipMemcpyAsync(src.data(), c->out_offsets.p, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    const int64_t total = src[n];
    int rc;
    if ((rc = ensure(c, s.d_sets, (size_t)std::max<int64_t>(total, 1))) || (rc = ensure(c, s.d_costs, (size_t)std::max<int64_t>(total, 1))) ||
        (rc = ensure(c, s.d_offsets, (size_t)n + 1)) || (rc = ensure(c, s.d_scores_tmp, (size_t)std::max<int64_t>(total, 1))))
        return rc;
    // order the lists by variable index (the .pss variable order)
    std::vector<int> where(n, -1);
    for (int i = 0; i < n; ++i) where[c->vars[i]] = i;
    s.n = n;
    s.offsets.assign(n + 1, 0);
    for (int v = 0; v < n; ++v) {
        const int i = where[v];
        const int64_t cnt = src[i + 1] - src[i];
        s.offsets[v + 1] = s.offsets[v] + cnt;
        if (cnt) {
            ULG_HIP(c, hipMemcpyAsync(s.d_sets.p + s.offsets[v], c->out_sets.p + src[i], (size_t)cnt * 8, hipMemcpyDeviceToDevice, c->stream));
            ULG_HIP(c, hipMemcpyAsync(s.d_scores_tmp.p + s.offsets[v], c->out_scores.p + src[i], (size_t)cnt * 4, hipMemcpyDeviceToDevice, c->stream));
        }
    }
    ULG_HIP(c, hipMemcpyAsync(s.d_offsets.p, s.offsets.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if ((rc = search_quantize_device(c, s.d_scores_tmp.p, s.d_costs.p, total))) return rc;
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return lists_loaded(c);
}

int ulg_search_load_scores(ulg_ctx *c, int n, const int64_t *offsets, const uint64_t *sets, const float *scores,
                           int device_ptrs) {
    if (!c || n < 1 || n > kMaxVars || !offsets || !sets || !scores)
        return set_err(c, ULG_ERR_ARG, "ulg_search_load_scores: bad arguments");
    for (int v = 0; v < n; ++v)
        if (offsets[v + 1] < offsets[v] || offsets[v + 1] - offsets[v] > 0xffffffffll)
            return set_err(c, ULG_ERR_ARG, "ulg_search_load_scores: bad offsets");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = state(c);
    const int64_t total = offsets[n] - offsets[0];
    int rc;
    if ((rc = ensure(c, s.d_sets, (size_t)std::max<int64_t>(total, 1))) || (rc = ensure(c, s.d_costs, (size_t)std::max<int64_t>(total, 1))) ||
        (rc = ensure(c, s.d_offsets, (size_t)n + 1)) || (rc = ensure(c, s.d_scores_tmp, (size_t)std::max<int64_t>(total, 1))))
        return rc;
    s.n = n;
    s.offsets.assign(n + 1, 0);
    for (int v = 0; v <= n; ++v) s.offsets[v] = offsets[v] - offsets[0];
    const hipMemcpyKind kind = device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (total) {
        ULG_HIP(c, hipMemcpyAsync(s.d_sets.p, sets + offsets[0], (size_t)total * 8, kind, c->stream));
        ULG_HIP(c, hipMemcpyAsync(s.d_scores_tmp.p, scores + offsets[0], (size_t)total * 4, kind, c->stream));
    }
    ULG_HIP(c, hipMemcpyAsync(s.d_offsets.p, s.offsets.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if ((rc = search_quantize_device(c, s.d_scores_tmp.p, s.d_costs.p, total))) return rc;
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return lists_loaded(c);
}

int ulg_bestscore_query(ulg_ctx *c, int64_t count, const int *vars, const uint64_t *S, float *costs, uint64_t *parents) {
    if (!c || count < 0 || (count && (!vars || !S))) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready) return set_err(c, ULG_ERR_STATE, "ulg_bestscore_query: no parent-set lists");
    for (int64_t i = 0; i < count; ++i)
        if (vars[i] < 0 || vars[i] >= c->search->n) return set_err(c, ULG_ERR_ARG, "ulg_bestscore_query: bad variable");
    if (count == 0) return ULG_OK;
    ULG_HIP(c, hipSetDevice(c->device));
    return search_query(c, count, vars, S, costs, parents);
}

int ulg_pdb_build(ulg_ctx *c, int pd_count, uint64_t ancestors, uint64_t scc) {
    if (!c) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready) return set_err(c, ULG_ERR_STATE, "ulg_pdb_build: no parent-set lists");
    ULG_HIP(c, hipSetDevice(c->device));
    int rc = search_ensure_scope(c, ancestors | scc);  // lookups outside the tables scan the lists
    if (rc == ULG_ERR_UNSUPPORTED) c->err.clear();
    else if (rc) return rc;
    return search_build_pdb(c, pd_count, ancestors, scc);
}

int ulg_pdb_query(ulg_ctx *c, int64_t count, const uint64_t *S, float *h, int *complete) {
    if (!c || count < 0 || (count && (!S || !h))) return ULG_ERR_ARG;
    if (!c->search || !c->search->pdb_ready) return set_err(c, ULG_ERR_STATE, "ulg_pdb_query: no pattern database");
    if (count == 0) return ULG_OK;
    ULG_HIP(c, hipSetDevice(c->device));
    return search_pdb_query(c, count, S, h, complete);
}

namespace {
// The replay's host counters (perf_event_open on the calling thread, user
// space only): cycles, instructions and the kernel's generic cache-miss event
// (the last-level misses a pop or successor visit waits on).  A counter the
// host does not grant (containers, perf_event_paranoid) reads as -1.
struct HostPmu {
    int fd[3] = {-1, -1, -1};
    HostPmu() {
        const uint64_t cfg[3] = {PERF_COUNT_HW_CPU_CYCLES, PERF_COUNT_HW_INSTRUCTIONS, PERF_COUNT_HW_CACHE_MISSES};
        for (int i = 0; i < 3; ++i) {
            perf_event_attr pe;
            std::memset(&pe, 0, sizeof pe);
            pe.type = PERF_TYPE_HARDWARE;
            pe.size = sizeof pe;
            pe.config = cfg[i];
            pe.disabled = 1;
            pe.exclude_kernel = 1;
            pe.exclude_hv = 1;
            fd[i] = (int)syscall(SYS_perf_event_open, &pe, 0, -1, -1, 0);
            if (fd[i] >= 0) {
                ioctl(fd[i], PERF_EVENT_IOC_RESET, 0);
                ioctl(fd[i], PERF_EVENT_IOC_ENABLE, 0);
            }
        }
    }
    // first: acc holds nothing yet (it reads -1 until a counter is read)
    void stop(int64_t (&acc)[3], bool first) {
        for (int i = 0; i < 3; ++i) {
            if (fd[i] < 0) {
                acc[i] = -1;
                continue;
            }
            ioctl(fd[i], PERF_EVENT_IOC_DISABLE, 0);
            uint64_t v = 0;
            if (read(fd[i], &v, sizeof v) == (ssize_t)sizeof v && (first || acc[i] >= 0))
                acc[i] = (first ? 0 : acc[i]) + (int64_t)v;
            else acc[i] = -1;
            close(fd[i]);
            fd[i] = -1;
        }
    }
};
}  // namespace

int ulg_astar(ulg_ctx *c, const uint64_t *edges, int pd_count, int mode, uint64_t *vpar, int *order,
              float *goal_cost, int64_t *expanded, char *net_text, int64_t net_cap) {
    if (!c) return ULG_ERR_ARG;
    const int n = c->search ? c->search->n : 0;
    return ulg_astar_scc(c, edges, pd_count, mode, 0, all_vars(n), vpar, order, goal_cost, expanded, net_text,
                         net_cap);
}

int ulg_astar_scc(ulg_ctx *c, const uint64_t *edges, int pd_count, int mode, uint64_t ancestors, uint64_t scc,
                  uint64_t *vpar, int *order, float *goal_cost, int64_t *expanded, char *net_text,
                  int64_t net_cap) {
    if (!c || !vpar || !order || !goal_cost || !expanded) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready) return set_err(c, ULG_ERR_STATE, "ulg_astar: no parent-set lists");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = *c->search;
    const int n = s.n;
    const uint64_t all = all_vars(n);
    if ((ancestors | scc) & ~all) return set_err(c, ULG_ERR_ARG, "ulg_astar: ancestors / scc outside the variables");
    int rc;
    if (mode == ULG_ASTAR_GPU) {
        if (ancestors) return set_err(c, ULG_ERR_UNSUPPORTED, "ulg_astar(GPU): ancestors need the exact-order search");
        if ((rc = search_ensure_scope(c, all))) return rc;  // the whole lattice
    }
    // astar(): the heuristic is built over (ancestors, scc) (astar_main.cpp:590-611)
    if (!s.pdb_ready || s.pd_count != pd_count || s.scc != scc || s.ancestors != ancestors) {
        rc = search_ensure_scope(c, ancestors | scc);
        if (rc == ULG_ERR_UNSUPPORTED) c->err.clear();  // the PDB build scans the lists
        else if (rc) return rc;
        if ((rc = search_build_pdb(c, pd_count, ancestors, scc))) return rc;
    }
    *expanded = 0;
    *goal_cost = 0.0f;
    c->out_of_time = 0;
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(c->time_limit_ms);
    for (int i = 0; i < n; ++i) { vpar[i] = 0; order[i] = 0; }
    if (net_text && net_cap > 0) net_text[0] = 0;
    if (mode == ULG_ASTAR_GPU) return astar_gpu(c, edges, vpar, order, goal_cost, expanded);
    if (mode != ULG_ASTAR_EXACT) return set_err(c, ULG_ERR_ARG, "ulg_astar: unknown mode");
    // -1 (not measured) unless a component's search opens the counters
    c->exact_pmu[0] = c->exact_pmu[1] = c->exact_pmu[2] = -1;
    bool pmu_first = true;
    std::vector<uint64_t> comps;
    const bool good = edges != nullptr;
    if (good) components(edges, n, comps);
    else comps.push_back(all);
    bool hang = false;
    bool fail = false;
    for (uint64_t comp : comps) {
        // every lookup of this component's search lies inside ancestors | component
        ExactResult r;
        const bool dense = dense_eligible(ancestors | comp, comp) && !std::getenv("ULG_EXACT_SPARSE");
        if ((rc = search_ensure_scope(c, ancestors | comp))) return rc;
        // the -r budget also covers the successor-cost rows (up to 8 GiB)
        bool rows_late = false;
        const int64_t dl_ns =
            c->time_limit_ms > 0 ? std::chrono::duration_cast<std::chrono::nanoseconds>(deadline.time_since_epoch()).count()
                                 : 0;
        if ((rc = dense ? search_cost_rows_host(c, ancestors | comp, comp, dl_ns, &rows_late) : search_cost_table_host(c)))
            return rc;
        if (rows_late) {  // out of time before the search started: no goal (astar_main.cpp:266)
            c->out_of_time = 1;
            fail = true;
            continue;
        }
        HostTables T;
        host_tables(s, T);
        const Clock::time_point *dl = c->time_limit_ms > 0 ? &deadline : nullptr;
        HostPmu pmu;
        rc = dense ? astar_dense(c, T, edges, good, ancestors, comp, expanded, &hang, r, dl)
                   : astar_one(c, T, edges, good, ancestors, comp, expanded, &hang, r, dl);
        pmu.stop(c->exact_pmu, pmu_first);
        pmu_first = false;
        if (rc) return rc;
        if (!r.found) { fail = true; continue; }
        // each component rewrites netFile and netFile.csv (astar_main.cpp:470,519)
        for (int v = 0; v < n; ++v) vpar[v] = 0;
        for (int v = 0; v < n; ++v) vpar[r.total[v]] = r.opt[v];
        for (int v = 0; v < n; ++v) order[v] = r.total[v];
        *goal_cost = r.goal_g;
        if (net_text && net_cap > 0) {
            int64_t len = 0;
            len += snprintf(net_text + len, (size_t)(net_cap - len), "NumVars %d\n", n);
            for (int v = 0; v < n && len < net_cap; ++v) {
                len += snprintf(net_text + len, (size_t)(net_cap - len), "Var %d, parents", r.total[v] + 1);
                for (int i = 0; i < n && len < net_cap; ++i)
                    if ((r.opt[v] >> i) & 1ull) len += snprintf(net_text + len, (size_t)(net_cap - len), ", %d", i + 1);
                if (len < net_cap) len += snprintf(net_text + len, (size_t)(net_cap - len), "\n");
            }
        }
    }
    if (hang) return set_err(c, ULG_ERR_STATE, "ulg_astar: the reference heap's __down_heap would not terminate here");
    if (fail && !c->out_of_time) return set_err(c, ULG_ERR_STATE, "ulg_astar: a component has no goal");
    return ULG_OK;
}

}  // extern "C"
