// triplet_host.cpp -- ulg_triplet_astar: the reference's triplet_astar driver
// (astar/triplet_astar.cpp:991-1622) over the GPU-built best-score lattice.
//
// Every A* the driver asks for is over one "big cluster" (the union of the
// clusters of a triple) and its answer depends on that cluster alone, so the
// searches are memoised per cluster: on a full skeleton every triple maps to
// the same cluster and the reference's thousands of identical searches become
// one.  Each distinct cluster gets its own static pattern database built on
// the GPU (ulg_pdb_build(pd_count, 0, cluster), triplet_astar.cpp:303) and an
// exact-order search on the host over O(1) table reads -- the re-opening
// variant of run_astar_on_one_scc (:285-674), whose pop order decides which
// of several tied optimal DAGs the orientation rules see.
//
// The orientation state is held as bit rows: out[i] bit j == directed_graph
// [i][j].  Both directions set = undirected edge.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <unordered_set>

#include "search_exact.h"

using namespace ulg;
using namespace ulg::exact;

namespace {

constexpr int kMaxCluster = 26;  // triplet_astar.cpp:840

inline bool bit(uint64_t s, int i) { return (s >> i) & 1ull; }

struct SearchPool;

struct Triplet {
    ulg_ctx *c = nullptr;
    SearchState *s = nullptr;
    int n = 0, pd_count = 2;
    uint64_t nb[64] = {}, clusters[64] = {}, vstr[64] = {}, out[64] = {};
    std::unordered_set<uint64_t> checked;
    std::unordered_map<uint64_t, std::vector<uint64_t>> *memo = nullptr;  // SearchState::triplet_memo
    struct SpecResult {
        std::vector<uint64_t> op;
        int64_t nexp = 0;
        bool hang = false;
    };
    std::unordered_map<uint64_t, SpecResult> spec;  // searched ahead, not yet asked for
    SearchPool *pool = nullptr;  // look-ahead searches on host threads (ulg_triplet_astar)
    int threads = 1;           // host threads for searches ahead (ULG_TRIPLET_THREADS)
    bool parallel_ok = false;  // device tables cover every variable; host costs ready
    int ci = -1, cj = 0, ck = 0;  // the first sweep's current triple (speculate); -1: off
    int64_t runs = 0, distinct = 0, expanded = 0;
    int num_v_structures = 0;
    bool hang = false;
    int rc = ULG_OK;
    // the -r watchdog (triplet_astar.cpp:139-142,355,1674-1681): once the
    // budget is spent every A* ends without a goal ("No solution found",
    // :657-662), so process_triple sees the empty op of :855 -- also for
    // clusters solved before, which the reference would search again
    bool timed = false;
    std::chrono::steady_clock::time_point deadline;
    // set by the watchdog thread once the budget is spent: a search already
    // running stops at its next poll, as the reference's loop stops inside
    // run_astar_on_one_scc (`!outOfTime`, triplet_astar.cpp:355)
    std::atomic<bool> expired{false};
    const std::vector<uint64_t> *no_solution() {
        static const std::vector<uint64_t> none(64, 0);
        c->out_of_time = 1;
        return &none;
    }
    bool past_deadline() const { return timed && std::chrono::steady_clock::now() > deadline; }

    bool dg(int a, int b) const { return bit(out[a], b); }
    void set(int a, int b, bool v) {
        if (v) out[a] |= 1ull << b;
        else out[a] &= ~(1ull << b);
    }
    // an undirected a-b unless either direction is already decided
    void undirected_if_free(int a, int b, bool adjacent) {
        if (adjacent && !dg(a, b) && !dg(b, a)) {
            set(a, b, true);
            set(b, a, true);
        }
    }
    void add_edge(int a, int b) {  // Skeleton::add_edge + cluster refresh (:1186-1191)
        nb[a] |= 1ull << b;
        nb[b] |= 1ull << a;
        clusters[a] = nb[a];
        clusters[b] = nb[b];
    }
};

// One cluster's search, host side only: the goal's leaf chain (for the
// parent queries), expansions, and whether the reference heap would spin.
struct ClusterRun {
    int64_t nexp = 0;
    bool hang = false;
    bool cancelled = false;  // stopped by SearchPool::shutdown (never consumed)
    std::vector<int> qv;        // leaves from the goal back to the root
    std::vector<uint64_t> qs;   // the set each leaf was added to (incl. itself)
};

// run_astar_on_one_scc of triplet_astar.cpp:285-674 with ancestors = {} and
// the_scc = cluster: no skeleton filter, and a closed node whose g strictly
// improves is pushed back onto the open list (:556-576).  Reads only T.
void astar_cluster(const HostTables &T, uint64_t cluster, ClusterRun &R, const std::atomic<bool> *cancel) {
    std::vector<Node> nodes;
    nodes.reserve(1024);
    SubsetIndex generated;
    generated.init(cluster);
    Heap open;
    open.nodes = &nodes;
    const uint64_t r1 = cluster >> 1;
    nodes.push_back(Node{0.0f, 0.0f, 0, (uint8_t)(r1 ? __builtin_ctzll(r1) + 1 : 0), 0});
    open.push(0);
    int64_t goal = -1, nexp = 0;
    const float upperBound = FLT_MAX;
    while (!open.empty()) {
        if (cancel && (nexp & 4095) == 0 && cancel->load(std::memory_order_relaxed)) {
            R.cancelled = true;
            return;
        }
        const uint32_t ui = open.pop();
        ++nexp;
        const uint64_t variables = nodes[ui].sub;
        if (variables == cluster) { goal = ui; break; }
        if (nodes[ui].g + nodes[ui].h > upperBound) break;
        nodes[ui].pq = -2;
        const float ug = nodes[ui].g;
        uint64_t cand = cluster & ~variables;
        for (uint64_t x = cand; x; x &= x - 1) {
            const int leaf = __builtin_ctzll(x);
            generated.prefetch(variables | (1ull << leaf));
            T.prefetch_bs(leaf, variables);
        }
        while (cand) {
            const int leaf = __builtin_ctzll(cand);
            cand &= cand - 1;
            const uint64_t nv = variables | (1ull << leaf);
            const int64_t si = generated.find(nv);
            if (si < 0) {
                bool complete = false;
                const float g = ug + T.bs(leaf, nv);
                const float h = T.h(nv, &complete);
                const uint32_t idx = (uint32_t)nodes.size();
                nodes.push_back(Node{g, h, nv, (uint8_t)leaf, 0});
                open.push(idx);
                generated.insert(nv, idx);
                continue;
            }
            const float g = ug + T.bs(leaf, variables);
            if (g < nodes[si].g) {
                nodes[si].leaf = (uint8_t)leaf;
                nodes[si].g = g;
                if (nodes[si].pq == -2) open.push((uint32_t)si);  // re-open
                else open.update((uint32_t)si);
            }
        }
    }
    R.nexp = nexp;
    R.hang = open.hang;
    if (goal < 0) return;  // no goal: every parent set stays empty
    // reconstructSolution (:172-224): walk the leaves back from the goal
    const int count = __builtin_popcountll(cluster);
    uint64_t remaining = nodes[goal].sub;
    int64_t cur = goal;
    for (int i = 0; i < count && cur >= 0; ++i) {
        const int leaf = nodes[cur].leaf;
        R.qv.push_back(leaf);
        R.qs.push_back(remaining);
        remaining ^= 1ull << leaf;
        cur = generated.find(remaining);
    }
}

// astar_cluster over dense node homes: recs[pext(S, cluster)] (16 B) and
// 8-byte heap entries (DenseHeap, the same heap algorithms and comparator as
// Heap), so a successor is one read of a small array instead of an index
// probe plus a node-vector read.  Re-opening (:556-576) pushes a closed
// record back; a record's pq is 0 until its node is generated (the root is
// never a successor, so generatedNodes' missing root changes nothing).  The
// expansion count and the goal's leaf chain equal astar_cluster's (A/B:
// ULG_TRIPLET_DENSE=0, tests/test_gpu_triplet.py).
// Every cluster the driver searches qualifies (kMaxCluster): at 26 variables
// 1 GiB of records and 0.5 GiB of heap per search thread, kept per thread.
constexpr int kDenseClusterBits = kMaxCluster;

bool astar_cluster_dense(const HostTables &T, uint64_t cluster, ClusterRun &R, const std::atomic<bool> *cancel) {
    const int m = __builtin_popcountll(cluster);
    const uint64_t nslots = 1ull << m;
    thread_local HostHuge recmem, heapmem;
    if (!recmem.reserve(nslots * sizeof(DenseRec), false) || !heapmem.reserve((nslots + 16) * sizeof(DEnt), false))
        return false;
    DenseRec *recs = static_cast<DenseRec *>(recmem.p);
    recmem.zero_prefix(nslots * sizeof(DenseRec));
    DenseHeap open;
    open.recs = recs;
    open.a = static_cast<DEnt *>(heapmem.p) + 1;
    uint32_t sbit[64] = {0};
    {
        int i = 0;
        for (uint64_t x = cluster; x; x &= x - 1) sbit[__builtin_ctzll(x)] = 1u << i++;
    }
    const uint32_t goal_slot = (uint32_t)(nslots - 1);
    const uint64_t r1 = cluster >> 1;
    recs[0] = DenseRec{0.0f, 0.0f, 0, (uint8_t)(r1 ? __builtin_ctzll(r1) + 1 : 0), {0, 0, 0}};
    open.push(0);
    int64_t goal = -1, nexp = 0;
    const float upperBound = FLT_MAX;
    while (open.len > 0) {
        if (cancel && (nexp & 4095) == 0 && cancel->load(std::memory_order_relaxed)) {
            R.cancelled = true;
            return true;
        }
        {
            // the top's successor records are fetched while the pop descends
            // the heap (search_host.cpp's dense replay does the same)
            const uint32_t top = open.a[0].slot();
            const uint64_t tv = g_have_bmi2 ? pdep_bmi2(top, cluster) : pdep64(top, cluster);
            for (uint64_t x = cluster & ~tv; x; x &= x - 1) __builtin_prefetch(&recs[top | sbit[__builtin_ctzll(x)]], 1);
        }
        const uint32_t ui = open.pop();
        ++nexp;
        if (ui == goal_slot) { goal = ui; break; }
        DenseRec &U = recs[ui];
        if (U.g + U.h > upperBound) break;
        U.pq = -1;
        const float ug = U.g;
        const uint64_t variables = g_have_bmi2 ? pdep_bmi2(ui, cluster) : pdep64(ui, cluster);
        const uint64_t cand = cluster & ~variables;
        for (uint64_t x = cand; x; x &= x - 1) T.prefetch_bs(__builtin_ctzll(x), variables);
        for (uint64_t x = cand; x; x &= x - 1) {
            const int leaf = __builtin_ctzll(x);
            const uint32_t si = ui | sbit[leaf];
            DenseRec &S = recs[si];
            // getScore(leaf, S u {leaf}) == getScore(leaf, S): leaf is never in its own sets
            const float g = ug + T.bs(leaf, variables);
            if (S.pq == 0) {
                bool complete = false;
                S.g = g;
                S.h = T.h(variables | (1ull << leaf), &complete);
                S.leaf = (uint8_t)leaf;
                open.push(si);
                continue;
            }
            if (g < S.g) {
                S.leaf = (uint8_t)leaf;
                S.g = g;
                if (S.pq == -1) open.push(si);  // re-open
                else open.update(si);
            }
        }
    }
    R.nexp = nexp;
    R.hang = open.hang;
    if (goal < 0) return true;
    // reconstructSolution (:172-224)
    uint64_t remaining = cluster;
    uint32_t cur = (uint32_t)goal;
    for (int i = 0; i < m; ++i) {
        const int leaf = recs[cur].leaf;
        R.qv.push_back(leaf);
        R.qs.push_back(remaining);
        remaining ^= 1ull << leaf;
        cur ^= sbit[leaf];
        if (remaining == 0 || recs[cur].pq == 0) break;  // the root is not in generatedNodes
    }
    return true;
}

void search_cluster(const HostTables &T, uint64_t cluster, ClusterRun &R, const std::atomic<bool> *cancel = nullptr) {
    static const bool dense = !std::getenv("ULG_TRIPLET_DENSE") || std::atoi(std::getenv("ULG_TRIPLET_DENSE")) != 0;
    if (dense && __builtin_popcountll(cluster) <= kDenseClusterBits && astar_cluster_dense(T, cluster, R, cancel)) return;
    astar_cluster(T, cluster, R, cancel);  // the indexed form (or the mapping failed)
}

// each leaf's best parent set among its predecessors, from the device tables
int cluster_parents_of(Triplet &t, const ClusterRun &R, std::vector<uint64_t> &op) {
    op.assign(t.n, 0);
    if (R.qv.empty()) return ULG_OK;
    std::vector<float> qc(R.qv.size());
    std::vector<uint64_t> qp(R.qv.size());
    if (int rc = search_query(t.c, (int64_t)R.qv.size(), R.qv.data(), R.qs.data(), qc.data(), qp.data())) return rc;
    for (size_t i = 0; i < R.qv.size(); ++i) op[R.qv[i]] = qp[i];
    return ULG_OK;
}

int cluster_astar(Triplet &t, uint64_t cluster, std::vector<uint64_t> &op) {
    ulg_ctx *c = t.c;
    int rc;
    // every lookup of this search and of its PDB lies inside the cluster
    if ((rc = search_ensure_scope(c, cluster)) || (rc = search_cost_table_host(c))) return rc;
    if ((rc = search_build_pdb(c, t.pd_count, 0, cluster))) return rc;
    HostTables T;
    host_tables(*t.s, T);
    ClusterRun R;
    search_cluster(T, cluster, R, t.timed ? &t.expired : nullptr);
    t.expanded += R.nexp;
    if (R.hang) t.hang = true;
    return cluster_parents_of(t, R, op);
}

// StaticPatternDatabase over `scc` (static_pattern_database.cpp:95-120 groups,
// :176-219 reverse DP) on the host, with search_build_pdb's exact float
// operations and order (pdb_bs_kernel + pdb_layer_kernel), for the parallel
// cluster searches: each needs its own database while the device holds one.
// cancel (the -r watchdog of a look-ahead pool): checked per DP layer, so a
// 24-variable group stops within one layer's work; P.cancelled tells.
struct HostPdb {
    std::vector<uint64_t> groups, pd_off;
    std::vector<float> pd;
    bool cancelled = false;
};
bool pdb_host(const HostTables &T, uint64_t scc, int pd_count, HostPdb &P,
              const std::atomic<bool> *cancel = nullptr) {
    P.cancelled = false;
    auto stopped = [&]() {
        if (cancel && cancel->load(std::memory_order_relaxed)) P.cancelled = true;
        return P.cancelled;
    };
    const int remaining = __builtin_popcountll(scc);
    const int pds = (int)std::ceil((float)remaining / pd_count);
    int var = scc ? __builtin_ctzll(scc) : -1;
    int x = 0;
    P.groups.clear();
    for (int g = 0; g < pd_count; ++g) {
        uint64_t grp = 0;
        for (int sz = 0; sz < pds && x < remaining; ++sz) {
            grp |= 1ull << var;
            const uint64_t rest = (var + 1 < 64) ? (scc >> (var + 1)) : 0;
            var = var + (rest ? (__builtin_ctzll(rest) + 1) : 0);
            ++x;
        }
        P.groups.push_back(grp);
    }
    P.pd_off.assign(pd_count + 1, 0);
    for (int g = 0; g < pd_count; ++g) {
        const int sz = __builtin_popcountll(P.groups[g]);
        if (sz > 24) return false;
        P.pd_off[g + 1] = P.pd_off[g] + (1ull << sz);
    }
    P.pd.assign(P.pd_off[pd_count], 0.0f);
    std::vector<float> bsv;
    for (int g = 0; g < pd_count; ++g) {
        const uint64_t grp = P.groups[g];
        const int s = __builtin_popcountll(grp);
        if (s == 0) continue;
        int bitpos[64];
        int q = 0;
        for (int b = 0; b < 64; ++b)
            if ((grp >> b) & 1ull) bitpos[q++] = b;
        bsv.assign((size_t)s << s, 0.0f);
        for (uint64_t R = 1; R < (1ull << s); ++R) {
            if ((R & 0xFFFF) == 0 && stopped()) return true;
            uint64_t Rg = 0;
            for (int b = 0; b < s; ++b)
                if ((R >> b) & 1ull) Rg |= 1ull << bitpos[b];
            for (int j = 0; j < s; ++j) {
                if (!((R >> j) & 1ull)) continue;
                const int leaf = bitpos[j];
                bsv[R * s + j] = T.bs(leaf, scc & ~(Rg & ~(1ull << leaf)));
            }
        }
        float *pd = P.pd.data() + P.pd_off[g];
        for (int layer = 1; layer <= s; ++layer) {
            if (stopped()) return true;
            for (uint64_t R = 1; R < (1ull << s); ++R) {
                if (__builtin_popcountll(R) != layer) continue;
                float cur = 0.0f;
                for (int j = s - 1; j >= 0; --j) {
                    if (!((R >> j) & 1ull)) continue;
                    const float newG = bsv[R * s + j] + pd[R ^ (1ull << j)];
                    if (cur == 0 || newG < cur) cur = newG;
                }
                pd[R] = cur;
            }
        }
    }
    return true;
}

// Searches of several clusters on host threads (each with its own host PDB,
// all reading the shared host cost table), then their parent queries on the
// device in order.  Results go to t.spec; cluster_parents counts a search
// (distinct, expansions) only when the driver asks for its cluster, so the
// statistics are the sequential driver's.
int solve_parallel(Triplet &t, const std::vector<uint64_t> &batch) {
    HostTables base;
    host_tables(*t.s, base);
    std::vector<ClusterRun> runs(batch.size());
    std::vector<char> ok(batch.size(), 1);
    std::atomic<size_t> next{0};
    auto work = [&]() {
        HostPdb P;
        for (size_t i; (i = next.fetch_add(1)) < batch.size();) {
            if (!pdb_host(base, batch[i], t.pd_count, P)) { ok[i] = 0; continue; }
            HostTables T = base;
            T.pd = P.pd.data();
            T.groups = P.groups;
            T.pd_off = P.pd_off;
            search_cluster(T, batch[i], runs[i]);
        }
    };
    std::vector<std::thread> pool;
    const int nt = std::min<int>(t.threads, (int)batch.size());
    for (int k = 1; k < nt; ++k) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
    for (size_t i = 0; i < batch.size(); ++i) {
        if (!ok[i]) return set_err(t.c, ULG_ERR_UNSUPPORTED, "pattern-database group larger than 24 variables");
        Triplet::SpecResult sp;
        sp.nexp = runs[i].nexp;
        sp.hang = runs[i].hang;
        if (int rc = cluster_parents_of(t, runs[i], sp.op)) return rc;
        t.spec.emplace(batch[i], std::move(sp));
    }
    return ULG_OK;
}

// A pool of host threads that searches clusters ahead of the driver: the
// driver queues the cluster it needs at the front and the clusters it will
// probably ask for next behind it, and waits only for the one it needs, while
// the others keep running (a batch no longer waits for its slowest search).
// A result is counted (runs, distinct, expansions) only when the driver asks
// for its cluster, so the statistics are the sequential driver's; results
// never asked for are dropped, and searches still running at the end are
// cancelled.  Workers read only the host cost table and their own host PDBs.
struct SearchPool {
    HostTables base;
    int pd_count = 2;
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<uint64_t> queue;
    std::unordered_map<uint64_t, int> state;  // 1 queued, 2 running, 3 done
    std::unordered_map<uint64_t, std::pair<ClusterRun, bool>> done;  // run, PDB built
    std::atomic<bool> cancel{false};
    bool stop = false;
    std::vector<std::thread> workers;

    void start(const SearchState &s, int pdc, int nthreads) {
        host_tables(s, base);
        pd_count = pdc;
        for (int k = 0; k < nthreads; ++k) workers.emplace_back([this] { work(); });
    }
    void work() {
        HostPdb P;
        std::unique_lock<std::mutex> lk(mu);
        while (true) {
            cv_work.wait(lk, [&] { return stop || !queue.empty(); });
            if (stop) return;
            const uint64_t cl = queue.front();
            queue.pop_front();
            state[cl] = 2;
            lk.unlock();
            ClusterRun R;
            // a cluster dequeued after the watchdog fired is not started, and
            // a PDB build it interrupts ends the search as cancelled
            const bool ok = cancel.load(std::memory_order_relaxed) || pdb_host(base, cl, pd_count, P, &cancel);
            if (cancel.load(std::memory_order_relaxed) || P.cancelled) {
                R.cancelled = true;
            } else if (ok) {
                HostTables T = base;
                T.pd = P.pd.data();
                T.groups = P.groups;
                T.pd_off = P.pd_off;
                search_cluster(T, cl, R, &cancel);
            }
            lk.lock();
            done.emplace(cl, std::make_pair(std::move(R), ok));
            state[cl] = 3;
            cv_done.notify_all();
        }
    }
    bool known(uint64_t cl) {
        std::lock_guard<std::mutex> lk(mu);
        return state.count(cl) != 0;
    }
    size_t pending() {
        std::lock_guard<std::mutex> lk(mu);
        return queue.size();
    }
    // queue cl (front: the driver needs it now; a queued one moves up)
    void submit(uint64_t cl, bool front) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = state.find(cl);
        if (it != state.end()) {
            if (front && it->second == 1) {
                queue.erase(std::find(queue.begin(), queue.end(), cl));
                queue.push_front(cl);
            }
            return;
        }
        state[cl] = 1;
        if (front) queue.push_front(cl);
        else queue.push_back(cl);
        cv_work.notify_one();
    }
    // waits for a submitted cluster's search and hands its result over
    void take(uint64_t cl, ClusterRun &R, bool &ok) {
        std::unique_lock<std::mutex> lk(mu);
        cv_done.wait(lk, [&] { return state[cl] == 3; });
        auto it = done.find(cl);
        R = std::move(it->second.first);
        ok = it->second.second;
        done.erase(it);
        state.erase(cl);
    }
    void shutdown() {
        cancel = true;
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            queue.clear();
        }
        cv_work.notify_all();
        for (auto &th : workers) th.join();
        workers.clear();
    }
    ~SearchPool() { shutdown(); }
};

// Up to `want` distinct clusters, not yet searched, of the triples the first
// sweep reaches after (ci, cj, ck) on the current skeleton -- orientations may
// still change some of them, which only leaves a result unused.
void speculate(Triplet &t, std::vector<uint64_t> &batch, size_t want) {
    std::unordered_set<uint64_t> seen(batch.begin(), batch.end());
    for (int i = t.ci; i < t.n && batch.size() < want; ++i) {
        std::vector<int> unc;
        for (int j = 0; j < t.n; ++j)
            if (bit(t.nb[i], j)) unc.push_back(j);
        for (int j = (i == t.ci ? t.cj : 0); j < (int)unc.size() && batch.size() < want; ++j)
            for (int k = (i == t.ci && j == t.cj ? t.ck + 1 : 0); k < j && batch.size() < want; ++k) {
                int a[3] = {i, unc[j], unc[k]};
                std::sort(a, a + 3);
                const uint64_t key = ((uint64_t)a[0] << 40) + ((uint64_t)a[1] << 20) + (uint64_t)a[2];
                if (t.checked.count(key)) continue;
                const uint64_t big = t.clusters[i] | t.clusters[unc[j]] | t.clusters[unc[k]];
                if (__builtin_popcountll(big) > kMaxCluster || t.memo->count(big) || t.spec.count(big) ||
                    (t.pool && t.pool->known(big)) || !seen.insert(big).second)
                    continue;
                batch.push_back(big);
            }
    }
}

const std::vector<uint64_t> *cluster_parents(Triplet &t, uint64_t cluster) {
    ++t.runs;
    if (t.past_deadline()) return t.no_solution();
    auto it = t.memo->find(cluster);
    if (it != t.memo->end()) return &it->second;
    static const bool trace = std::getenv("ULG_TRIPLET_TRACE") != nullptr;  // per-search progress on stderr
    const auto c0 = std::chrono::steady_clock::now();
    auto sp = t.spec.find(cluster);
    if (sp == t.spec.end() && t.pool) {
        t.pool->submit(cluster, true);
        if (t.ci >= 0) {  // the first sweep: keep about two searches per thread queued
            const size_t want = 2 * (size_t)t.threads, have = t.pool->pending();
            std::vector<uint64_t> more;
            if (have < want) speculate(t, more, want - have);
            for (uint64_t m : more) t.pool->submit(m, false);
        }
        ClusterRun R;
        bool ok = false;
        t.pool->take(cluster, R, ok);
        if (R.cancelled) return t.no_solution();  // the watchdog stopped it (past the deadline)
        if (!ok) {
            t.rc = set_err(t.c, ULG_ERR_UNSUPPORTED, "pattern-database group larger than 24 variables");
            return nullptr;
        }
        Triplet::SpecResult spr;
        spr.nexp = R.nexp;
        spr.hang = R.hang;
        if ((t.rc = cluster_parents_of(t, R, spr.op))) return nullptr;
        sp = t.spec.emplace(cluster, std::move(spr)).first;
    }
    std::vector<uint64_t> op;
    int64_t nexp;
    if (sp != t.spec.end()) {
        nexp = sp->second.nexp;
        if (sp->second.hang) t.hang = true;
        t.expanded += nexp;
        op = std::move(sp->second.op);
        t.spec.erase(sp);
    } else {
        const int64_t e0 = t.expanded;
        if ((t.rc = cluster_astar(t, cluster, op))) return nullptr;
        nexp = t.expanded - e0;
    }
    if (trace)
        std::fprintf(stderr, "triplet: cluster %016llx (%d variables): %lld expansions in %.3f s\n",
                     (unsigned long long)cluster, __builtin_popcountll(cluster), (long long)nexp,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count());
    // a search the budget ran out during: the reference's loop stopped
    // without a goal (its result is not kept)
    if (t.past_deadline()) return t.no_solution();
    ++t.distinct;
    return &t.memo->emplace(cluster, std::move(op)).first->second;
}

// The context's memo for pd_count (a different pattern-database split gives
// the same optimal cost but possibly another tied DAG: start over).
std::unordered_map<uint64_t, std::vector<uint64_t>> *memo_for(SearchState &s, int pd_count) {
    if (s.triplet_pd != pd_count) {
        s.triplet_memo.clear();
        s.triplet_pd = pd_count;
    }
    return &s.triplet_memo;
}

// Look-ahead searches on host threads need the lattice tables over every
// variable (then no cluster rebuilds them) and their host copy.
void set_parallel(Triplet &t) {
    const char *e = std::getenv("ULG_TRIPLET_THREADS");
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    t.threads = e ? std::max(1, std::atoi(e)) : std::min(16, hw);
    const uint64_t all = (t.n >= 64) ? ~0ull : ((1ull << t.n) - 1ull);
    t.parallel_ok = t.threads > 1 && t.s->tables_ready && (t.s->scope & all) == all && t.s->table_vars == all &&
                    search_cost_table_host(t.c) == ULG_OK;
}

void init_skeleton(Triplet &t, const uint64_t *edges) {
    const int n = t.n;
    const uint64_t all = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    // Skeleton::get_neighbors: the file's rows, or every variable (self
    // included) without a skeleton; clusters add the variable itself (:1061-1072)
    for (int v = 0; v < n; ++v) {
        t.nb[v] = edges ? edges[v] : all;
        t.clusters[v] = t.nb[v] | (1ull << v);
    }
}

// The distinct clusters the first sweep (triplet_astar.cpp:1148-1204) asks
// for on the current skeleton, in first-request order (<= 26 variables).
std::vector<uint64_t> first_sweep_clusters(const Triplet &t) {
    std::unordered_set<uint64_t> seen;
    std::vector<uint64_t> out;
    for (int i = 0; i < t.n; ++i) {
        std::vector<int> unc;
        for (int j = 0; j < t.n; ++j)
            if (bit(t.nb[i], j)) unc.push_back(j);
        for (size_t j = 0; j < unc.size(); ++j)
            for (size_t q = 0; q < j; ++q) {
                const uint64_t big = t.clusters[i] | t.clusters[unc[j]] | t.clusters[unc[q]];
                if (__builtin_popcountll(big) > kMaxCluster || !seen.insert(big).second) continue;
                out.push_back(big);
            }
    }
    return out;
}

// process_triple (triplet_astar.cpp:811-989)
void process_triple(Triplet &t, int i, int vj, int vk) {
    if (t.rc) return;
    int a[3] = {i, vj, vk};
    std::sort(a, a + 3);
    const uint64_t big = t.clusters[i] | t.clusters[vj] | t.clusters[vk];
    if (__builtin_popcountll(big) > kMaxCluster) return;
    const uint64_t key = ((uint64_t)a[0] << 40) + ((uint64_t)a[1] << 20) + (uint64_t)a[2];
    if (!t.checked.insert(key).second) return;
    const std::vector<uint64_t> *opp = cluster_parents(t, big);
    if (!opp) return;
    const std::vector<uint64_t> &op = *opp;
    auto adjacent = [&](int x, int y) { return bit(op[x], y) || bit(op[y], x); };
    // collider c with parents p, q: p -> c <- q, then p - q if the DAG joins them
    auto collider = [&](int cc, int p, int q) {
        ++t.num_v_structures;
        t.set(p, cc, true);
        t.set(q, cc, true);
        t.set(cc, p, false);
        t.set(cc, q, false);
        t.undirected_if_free(p, q, adjacent(p, q));
        t.vstr[cc] |= (1ull << p) | (1ull << q);
    };
    if (bit(op[i], vj) && bit(op[i], vk)) collider(i, vj, vk);
    else if (bit(op[vk], i) && bit(op[vk], vj)) collider(vk, vj, i);
    else if (bit(op[vj], i) && bit(op[vj], vk)) collider(vj, vk, i);
    else {
        t.undirected_if_free(vk, vj, adjacent(vj, vk));
        t.undirected_if_free(i, vj, adjacent(vj, i));
        t.undirected_if_free(i, vk, adjacent(vk, i));
    }
}

// Meek rules 2, 3 and 4 as the reference applies them (:1297-1478), until a
// sweep orients nothing or n sweeps have run.
void meek(Triplet &t) {
    const int n = t.n;
    for (int iter = 0; iter < n; ++iter) {
        int oriented = 0;
        for (int v = 0; v < n; ++v) {  // rule 2: a -> v -> b and a - b  =>  a -> b
            uint64_t ins = 0, outs = 0;
            for (int j = 0; j < n; ++j) {
                if (t.dg(v, j) && !t.dg(j, v)) outs |= 1ull << j;
                else if (t.dg(j, v) && !t.dg(v, j)) ins |= 1ull << j;
            }
            if (!ins || !outs) continue;
            for (uint64_t pi = ins; pi; pi &= pi - 1) {
                const int p = __builtin_ctzll(pi);
                for (uint64_t co = outs; co; co &= co - 1) {
                    const int ch = __builtin_ctzll(co);
                    if (t.dg(p, ch) && t.dg(ch, p)) {
                        t.set(ch, p, false);
                        ++oriented;
                    }
                }
            }
        }
        for (int v = 0; v < n; ++v) {  // rule 3: two v-structure parents of v both undirected to w  =>  w -> v
            uint64_t und = 0;
            for (int j = 0; j < n; ++j)
                if (t.dg(v, j) && t.dg(j, v)) und |= 1ull << j;
            if (__builtin_popcountll(t.vstr[v]) < 2 || !und) continue;
            for (uint64_t wi = und; wi; wi &= wi - 1) {
                const int w = __builtin_ctzll(wi);
                int cnt = 0;
                for (uint64_t pi = t.vstr[v]; pi; pi &= pi - 1) {
                    const int p = __builtin_ctzll(pi);
                    cnt += t.dg(p, w) && t.dg(w, p);
                }
                if (cnt >= 2) {
                    t.set(v, w, false);
                    ++oriented;
                }
            }
        }
        for (int v = 0; v < n; ++v) {  // rule 4
            uint64_t ins = 0, outs = 0, und = 0;
            for (int j = 0; j < n; ++j) {
                const bool f = t.dg(v, j), b = t.dg(j, v);
                if (f && !b) outs |= 1ull << j;
                else if (b && !f) ins |= 1ull << j;
                else if (f && b) und |= 1ull << j;
            }
            if (!outs || !ins || !und) continue;
            for (uint64_t wi = und; wi; wi &= wi - 1) {
                const int w = __builtin_ctzll(wi);
                bool joined = false;
                for (uint64_t pi = ins; pi && !joined; pi &= pi - 1) {
                    const int p = __builtin_ctzll(pi);
                    joined = t.dg(w, p) && t.dg(p, w);
                }
                if (!joined) continue;
                for (uint64_t co = outs; co; co &= co - 1) {
                    const int ch = __builtin_ctzll(co);
                    if (!t.dg(w, ch) || !t.dg(ch, w)) continue;
                    ++oriented;
                    t.set(ch, w, false);
                }
            }
        }
        if (oriented == 0) break;
    }
}

}  // namespace

extern "C" int ulg_triplet_astar(ulg_ctx *c, const uint64_t *edges, int pd_count, int *directed_graph, int64_t *stats) {
    if (!c || !directed_graph || pd_count < 1) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready) return set_err(c, ULG_ERR_STATE, "ulg_triplet_astar: no parent-set lists");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = *c->search;
    const int n = s.n;
    int rc;
    Triplet t;
    t.c = c;
    t.s = &s;
    t.n = n;
    t.pd_count = pd_count;
    t.memo = memo_for(s, pd_count);
    c->out_of_time = 0;
    if (c->time_limit_ms > 0) {
        t.timed = true;
        t.deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(c->time_limit_ms);
    }
    init_skeleton(t, edges);
    set_parallel(t);
    SearchPool pool;  // its destructor cancels and joins whatever still runs
    // -r: at the deadline every running cluster search stops at its next poll
    // (t.expired for the driver's own search, the pool's cancel flag for the
    // look-ahead threads); the driver then answers "no solution" (:657-662).
    // Declared after the pool, so it is joined before the pool shuts down.
    struct Watchdog {
        std::mutex mu;
        std::condition_variable cv;
        bool stop = false;
        std::thread th;
        ~Watchdog() {
            if (!th.joinable()) return;
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            th.join();
        }
    } wd;
    if (t.timed)
        wd.th = std::thread([&t, &pool, &wd] {
            std::unique_lock<std::mutex> lk(wd.mu);
            if (!wd.cv.wait_until(lk, t.deadline, [&wd] { return wd.stop; })) {
                t.expired = true;
                pool.cancel = true;
            }
        });
    if (t.parallel_ok) {
        pool.start(s, pd_count, t.threads);
        t.pool = &pool;
        // Every cluster the first sweep will ask for is known now (on the
        // initial skeleton): queue them all, largest first (a cluster's A*
        // may expand up to 2^|cluster| nodes), so the longest searches start
        // at once instead of when the driver first names them.  Orientations
        // can change later clusters; a result nobody asks for is dropped.
        if (!std::getenv("ULG_TRIPLET_LOOKAHEAD_ONLY")) {
            std::vector<uint64_t> first = first_sweep_clusters(t);
            std::stable_sort(first.begin(), first.end(), [](uint64_t a, uint64_t b) {
                return __builtin_popcountll(a) > __builtin_popcountll(b);
            });
            for (uint64_t cl : first)
                if (!t.memo->count(cl)) pool.submit(cl, false);
        }
    }
    for (int i = 0; i < n && !t.rc; ++i) {
        const uint64_t pin = t.nb[i];
        std::vector<int> unc;
        for (int j = 0; j < n; ++j)
            if (bit(pin, j)) unc.push_back(j);
        // an isolated orphan edge i - vj (:1166-1178)
        if (unc.size() == 1 && i < unc[0] && __builtin_popcountll(t.nb[unc[0]]) == 1) {
            const int vj = unc[0];
            const uint64_t parset = 1ull << vj;
            float cost;
            uint64_t par;
            if ((rc = search_query(c, 1, &i, &parset, &cost, &par))) return rc;
            if (par == parset) {
                t.set(i, vj, true);
                t.set(vj, i, true);
            }
        }
        for (size_t j = 0; j < unc.size() && !t.rc; ++j) {
            const int vj = unc[j];
            for (size_t k = 0; k < j && !t.rc; ++k) {
                const int vk = unc[k];
                t.ci = i;
                t.cj = (int)j;
                t.ck = (int)k;
                process_triple(t, i, vj, vk);
                if (!bit(t.nb[vj], vk) && (t.dg(vj, vk) || t.dg(vk, vj))) t.add_edge(vj, vk);
            }
        }
    }
    t.ci = -1;  // no look-ahead past the first sweep
    // unfaithful edges: oriented pairs the skeleton lacks (:1256-1290)
    int delta = 1;
    while (delta > 0 && !t.rc) {
        delta = 0;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < i; ++j) {
                if (!((t.dg(i, j) || t.dg(j, i)) && !bit(t.nb[i], j))) continue;
                ++delta;
                t.add_edge(i, j);
                if (t.pool) {
                    // the clusters this edge's triples ask for are fixed until
                    // the next add_edge: queue them all, in asking order
                    for (int k = 0; k < n; ++k) {
                        if (k == i || k == j || !(bit(t.clusters[i], k) || bit(t.clusters[j], k))) continue;
                        int a[3] = {i, j, k};
                        std::sort(a, a + 3);
                        const uint64_t key = ((uint64_t)a[0] << 40) + ((uint64_t)a[1] << 20) + (uint64_t)a[2];
                        const uint64_t big = t.clusters[i] | t.clusters[j] | t.clusters[k];
                        if (__builtin_popcountll(big) > kMaxCluster || t.checked.count(key) || t.memo->count(big) ||
                            t.spec.count(big))
                            continue;
                        t.pool->submit(big, false);
                    }
                }
                for (int k = 0; k < n; ++k)
                    if (k != i && k != j && (bit(t.clusters[i], k) || bit(t.clusters[j], k))) process_triple(t, i, j, k);
            }
    }
    if (t.rc) return t.rc;
    meek(t);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) directed_graph[i * n + j] = t.dg(i, j) ? 1 : 0;
    if (stats) {
        stats[0] = t.runs;
        stats[1] = t.distinct;
        stats[2] = t.expanded;
    }
    if (t.hang) return set_err(c, ULG_ERR_STATE, "ulg_triplet_astar: the reference heap's __down_heap would not terminate here");
    return ULG_OK;
}

// The distinct clusters the driver's first sweep (triplet_astar.cpp:1148-1204)
// asks A* for on the initial skeleton, in first-request order, without the
// searches themselves: triples of a variable and two of its neighbours whose
// cluster union has at most 26 variables.  Orientations found during the
// sweep can add skeleton edges (and so clusters) that this list lacks; the
// driver searches those itself.  Used to shard the searches over ranks.
extern "C" int ulg_triplet_clusters(ulg_ctx *c, const uint64_t *edges, uint64_t *clusters, int64_t cap,
                                    int64_t *count) {
    if (!c || !count || (cap > 0 && !clusters)) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready)
        return set_err(c, ULG_ERR_STATE, "ulg_triplet_clusters: no parent-set lists");
    Triplet t;
    t.n = c->search->n;
    init_skeleton(t, edges);
    const std::vector<uint64_t> first = first_sweep_clusters(t);
    const int64_t k = (int64_t)first.size();
    for (int64_t i = 0; i < k && i < cap; ++i) clusters[i] = first[i];
    *count = k;
    return k > cap && cap > 0 ? set_err(c, ULG_ERR_ARG, "ulg_triplet_clusters: cap too small") : ULG_OK;
}

// One re-opening exact-order A* per cluster (clusters already in the memo
// are not searched again); parents[i * n + v] = v's optimal parent set in
// cluster i's DAG.  Results enter the memo ulg_triplet_astar reads.
extern "C" int ulg_triplet_solve(ulg_ctx *c, const uint64_t *clusters, int64_t nc, int pd_count, uint64_t *parents,
                                 int64_t *stats) {
    if (!c || nc < 0 || (nc > 0 && !clusters) || pd_count < 1) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready)
        return set_err(c, ULG_ERR_STATE, "ulg_triplet_solve: no parent-set lists");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = *c->search;
    Triplet t;
    t.c = c;
    t.s = &s;
    t.n = s.n;
    t.pd_count = pd_count;
    t.memo = memo_for(s, pd_count);
    const uint64_t all = (t.n >= 64) ? ~0ull : ((1ull << t.n) - 1ull);
    for (int64_t i = 0; i < nc; ++i)
        if ((clusters[i] & ~all) || __builtin_popcountll(clusters[i]) > kMaxCluster)
            return set_err(c, ULG_ERR_ARG, "ulg_triplet_solve: cluster outside the variables or above 26 variables");
    set_parallel(t);
    if (t.parallel_ok) {  // every cluster not searched yet, on host threads
        std::vector<uint64_t> batch;
        std::unordered_set<uint64_t> seen;
        for (int64_t i = 0; i < nc; ++i)
            if (!t.memo->count(clusters[i]) && seen.insert(clusters[i]).second) batch.push_back(clusters[i]);
        if (!batch.empty() && (t.rc = solve_parallel(t, batch))) return t.rc;
    }
    for (int64_t i = 0; i < nc; ++i) {
        const std::vector<uint64_t> *op = cluster_parents(t, clusters[i]);
        if (!op) return t.rc;
        if (parents) std::memcpy(parents + i * t.n, op->data(), sizeof(uint64_t) * t.n);
    }
    if (stats) {
        stats[0] = t.runs;
        stats[1] = t.distinct;
        stats[2] = t.expanded;
    }
    if (t.hang) return set_err(c, ULG_ERR_STATE, "ulg_triplet_solve: the reference heap's __down_heap would not terminate here");
    return ULG_OK;
}

// Diagnostics (tests/test_gpu_triplet.py): one host PDB build of the look-ahead
// pool's form (pdb_host) over `cluster`, with the pool's cancel flag preset
// when cancel_preset != 0.  out[0] = built, out[1] = P.cancelled, out[2] =
// entries built, out[3] = the entries equal to the device PDB's over the same
// cluster (search_build_pdb, which the driver's own searches use).
extern "C" int ulg_diag_pdb_host(ulg_ctx *c, uint64_t cluster, int pd_count, int cancel_preset, int64_t *out) {
    if (!c || !out || pd_count < 1) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready)
        return set_err(c, ULG_ERR_STATE, "ulg_diag_pdb_host: no parent-set lists");
    ULG_HIP(c, hipSetDevice(c->device));
    SearchState &s = *c->search;
    int rc;
    if ((rc = search_ensure_scope(c, cluster)) || (rc = search_cost_table_host(c)) ||
        (rc = search_build_pdb(c, pd_count, 0, cluster)))
        return rc;
    HostTables base;
    host_tables(s, base);
    HostPdb P;
    std::atomic<bool> cancel{cancel_preset != 0};
    const bool ok = pdb_host(base, cluster, pd_count, P, &cancel);
    out[0] = ok;
    out[1] = P.cancelled;
    out[2] = ok && !P.cancelled ? (int64_t)P.pd.size() : 0;
    int64_t same = 0;
    if (ok && !P.cancelled && base.pd && P.pd_off == base.pd_off)
        for (size_t i = 0; i < P.pd.size(); ++i) same += std::memcmp(&P.pd[i], base.pd + i, 4) == 0;
    out[3] = same;
    return ULG_OK;
}

// Seed the memo with other ranks' results (same lists, same pd_count).
extern "C" int ulg_triplet_memo_put(ulg_ctx *c, const uint64_t *clusters, int64_t nc, int pd_count,
                                    const uint64_t *parents) {
    if (!c || nc < 0 || (nc > 0 && (!clusters || !parents)) || pd_count < 1) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready)
        return set_err(c, ULG_ERR_STATE, "ulg_triplet_memo_put: no parent-set lists");
    SearchState &s = *c->search;
    auto *memo = memo_for(s, pd_count);
    for (int64_t i = 0; i < nc; ++i)
        (*memo)[clusters[i]] = std::vector<uint64_t>(parents + i * s.n, parents + (i + 1) * s.n);
    return ULG_OK;
}
