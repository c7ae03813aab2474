// search_gpu.hip -- order-graph search on the GPU (ULG_ASTAR_GPU).
//
// The order graph of run_astar_on_one_scc (astar/astar_main.cpp:216-546) is
// layered by |S|: every edge S -> S u {leaf} goes from layer d to d+1 with
// cost getScore(leaf, S) (the reference adds it as g(u) + leaf_score, :327).
// Instead of a priority queue the GPU sweeps the layers: layer d+1 is one
// launch in which every node T "pulls" its cost from the d+1 predecessors
// T \ {leaf} of layer d (colex-indexed dense layers, no hashing, no atomics):
//     g(T) = min_leaf fl(g(T \ leaf) + bs(leaf, T \ leaf)),   leaf(T) = argmin
// subject to the reference's skeleton filter (a leaf may only follow a
// non-empty set that contains one of its neighbours, astar_main.cpp:305-313).
// That is the same shortest-path problem A* solves, so the goal cost is the
// optimal order cost; every node of the component is expanded once, which
// makes this the expansions/s path.  The DAG it returns is an optimal one
// (Markov equivalent to the exact-order result when the optimum is unique up
// to equivalence); the bit-exact reference DAG is ULG_ASTAR_EXACT's job.
#include <algorithm>
#include <cfloat>
#include <cstring>

#include "search_internal.h"

using namespace ulg;

namespace {

constexpr int kB = 256;
constexpr int kMaxM = 32;  // nodes of a searched component (2^32 nodes is already 4 GB of leaf bytes)

struct LayerArgs {
    SearchDev d;
    const uint64_t *binom;   // [33][33] C(a, b)
    const int *comp_vars;    // compact bit -> variable
    const uint64_t *edges;   // skeleton rows (may be null)
    int skeleton;            // apply the neighbour filter
    int symmetric;           // skeleton rows symmetric: reachable == connected (see layer_pull_kernel)
    int m;                   // component size
    int layer;               // layer of the nodes computed by this launch (>= 1)
    uint64_t count;          // C(m, layer)
    const float *gprev;      // layer - 1
    float *gcur;             // layer
    uint8_t *leaf;           // leaf bytes of this layer
    unsigned long long *reached;  // kCounters striped counters of reached nodes (null: the goal layer)
    const float *w;          // sweep table (SearchState::d_sweep_w) or null
    uint64_t w_half;         // 2^(m-1): one variable's slice group
    uint64_t w_layer;        // sum_{q < layer-1} C(m-1, q): the slice of the predecessors' layer
};

constexpr int kCounters = 256;

__device__ __forceinline__ uint64_t Bn(const uint64_t *b, int a, int k) { return b[a * 33 + k]; }

// kW: the costs come from the sweep table -- the predecessor T \ a_j's cost
// for leaf a_j sits at w[a_j][layer-1][rank of T \ a_j with a_j's position
// closed], one contiguous slice per (variable, layer), so a launch's cost
// reads stay inside its layer's slices (about a MALL's worth at C3) instead
// of spreading over the whole binary-indexed lattice.  Only for launches
// without the skeleton filter.
template <bool kW>
__global__ void __launch_bounds__(kB) layer_pull_kernel(LayerArgs a) {
    __shared__ uint64_t binom[33 * 33];
    __shared__ int cv[kMaxM];
    __shared__ uint64_t edg[64];
    // only the rows and columns this layer reads: C(c, i) for c < m, i <= layer
    {
        const int cols = a.layer + 1;
        for (int e = threadIdx.x; e < a.m * cols; e += kB) {
            const int r = e / cols, i = e - r * cols;
            binom[r * 33 + i] = a.binom[r * 33 + i];
        }
    }
    for (int i = threadIdx.x; i < a.m; i += kB) cv[i] = a.comp_vars[i];
    if (a.symmetric)
        for (int i = threadIdx.x; i < 64; i += kB) edg[i] = a.edges[i];
    __syncthreads();
    const uint64_t r = (uint64_t)blockIdx.x * kB + threadIdx.x;
    const int L = a.layer;
    if (r >= a.count) return;
    // unrank T (colex over the component's compact bits)
    uint64_t Tc = 0;
    {
        uint64_t rr = r;
        int c = a.m - 1;
        for (int i = L; i >= 1; --i) {
            while (Bn(binom, c, i) > rr) --c;
            Tc |= 1ull << c;
            rr -= Bn(binom, c, i);
            --c;
        }
    }
    uint64_t Tg = 0;
    for (uint64_t x = Tc; x; x &= x - 1) Tg |= 1ull << cv[__builtin_ctzll(x)];
    // With symmetric rows a node is reachable iff T induces a connected
    // subgraph: the filter lets a leaf follow P only if one of its neighbours
    // is in P, so every reachable T grows connected, and a connected T can be
    // grown from any of its vertices.  A disconnected T has no reached
    // predecessor it may follow, so it is settled here without the L
    // predecessor reads (most of the lattice on a sparse skeleton).
    bool connected = true;
    if (a.symmetric && L > 1) {
        uint64_t seen = Tg & (0 - Tg), fr = seen;
        while (fr) {
            uint64_t nb = 0;
            for (uint64_t y = fr; y; y &= y - 1) nb |= edg[__builtin_ctzll(y)];
            fr = nb & Tg & ~seen;
            seen |= fr;
        }
        connected = seen == Tg;
    }
    // rank(T \ a_j) = sum_{i<j} C(a_i, i+1) + sum_{i>j} C(a_i, i)   (a_0 < a_1 < ...)
    // the same rank in the universe without a_j (elements above a_j move down
    // one): sum_{i<j} C(a_i, i+1) + sum_{i>j} C(a_i - 1, i)
    uint64_t suffix = 0, suffixc = 0;
    if (connected) {
        int i = 0;
        for (uint64_t x = Tc; x; x &= x - 1, ++i)
            if (i >= 1) {
                const int ai = __builtin_ctzll(x);
                suffix += Bn(binom, ai, i);
                if (kW) suffixc += Bn(binom, ai - 1, i);
            }
    }
    uint64_t prefix = 0;
    float best = FLT_MAX;
    int bestj = 255;
    bool reached = false;
    uint64_t x = Tc;
    for (int j = 0; j < (connected ? L : 0); ++j) {
        const int aj = __builtin_ctzll(x);
        x &= x - 1;  // x now holds a_{j+1}, ...
        if (kW) {
            const float gp = a.gprev[prefix + suffix];
            if (gp < FLT_MAX) {
                reached = true;
                const float cand = gp + a.w[(uint64_t)aj * a.w_half + a.w_layer + prefix + suffixc];
                if (cand < best || bestj == 255) {
                    best = cand;
                    bestj = j;
                }
            }
        } else {
            const int leaf = cv[aj];
            const uint64_t P = Tg & ~(1ull << leaf);
            bool ok = !(a.skeleton && P != 0 && (P & a.edges[leaf]) == 0);
            if (ok) {
                const float gp = a.gprev[prefix + suffix];
                if (gp < FLT_MAX) {
                    reached = true;
                    const float cand = gp + bs_cost(a.d, leaf, P);
                    if (cand < best || bestj == 255) {
                        best = cand;
                        bestj = j;
                    }
                }
            }
        }
        // advance to j+1: a_{j+1} leaves the suffix, a_j joins the prefix
        if (x) {
            const int an = __builtin_ctzll(x);
            suffix -= Bn(binom, an, j + 1);
            if (kW) suffixc -= Bn(binom, an - 1, j + 1);
        }
        prefix += Bn(binom, aj, j + 1);
    }
    a.gcur[r] = reached ? best : FLT_MAX;
    a.leaf[r] = (uint8_t)(reached ? bestj : 255);
    if (a.reached) {
        // nodes of this layer that are reached -- and so expanded, below the goal layer
        const unsigned long long b = __ballot(reached);
        if ((threadIdx.x & 63) == __ffsll((long long)__ballot(true)) - 1 && b)
            atomicAdd(&a.reached[blockIdx.x % kCounters], (unsigned long long)__popcll(b));
    }
}

// Sweep table of one component: thread f of variable slot j (blockIdx.y)
// holds getScore(v_j, P) for the f-th (m-1)-bit set in (layer, colex) order,
// P mapped back to the variables with v_j's position opened.  Blocks are
// dispatched j-major, so the running blocks read one variable's lattice
// (64 MB at C3) at a time.
__global__ void __launch_bounds__(kB) sweep_w_kernel(SearchDev d, const uint64_t *gbinom, const uint64_t *loffm1,
                                                     const int *comp_vars, int m, uint64_t half, float *w) {
    __shared__ uint64_t binom[33 * 33];
    __shared__ uint64_t lo[kMaxM + 1];
    __shared__ int cv[kMaxM];
    for (int e = threadIdx.x; e < m * 33; e += kB) binom[e] = gbinom[e];
    for (int i = threadIdx.x; i <= m; i += kB) lo[i] = loffm1[i];
    for (int i = threadIdx.x; i < m; i += kB) cv[i] = comp_vars[i];
    __syncthreads();
    const uint64_t f = (uint64_t)blockIdx.x * kB + threadIdx.x;
    const int j = blockIdx.y;
    if (f >= half) return;
    int p = 0;
    while (p + 1 < m && lo[p + 1] <= f) ++p;
    uint64_t rr = f - lo[p], x = 0;
    int c = m - 2;
    for (int i = p; i >= 1; --i) {
        while (Bn(binom, c, i) > rr) --c;
        x |= 1ull << c;
        rr -= Bn(binom, c, i);
        --c;
    }
    const uint64_t Pc = ((x >> j) << (j + 1)) | (x & ((1ull << j) - 1ull));
    uint64_t Pg = 0;
    for (uint64_t y = Pc; y; y &= y - 1) Pg |= 1ull << cv[__builtin_ctzll(y)];
    w[(uint64_t)j * half + f] = bs_cost(d, cv[j], Pg);
}

// walk the leaf pointers from the goal back to the root (one thread)
__global__ void reconstruct_kernel(const uint8_t *leaf, const uint64_t *layer_off, const uint64_t *binom, int m,
                                   int *chain) {
    uint64_t T = (m >= 64) ? ~0ull : ((1ull << m) - 1ull);  // compact goal
    for (int d = m; d >= 1; --d) {
        uint64_t rank = 0;
        int i = 0;
        uint64_t x = T;
        while (x) {
            const int b = __builtin_ctzll(x);
            x &= x - 1;
            ++i;
            rank += binom[b * 33 + i];
        }
        const int j = leaf[layer_off[d] + rank];
        if (j == 255) { chain[d - 1] = -1; return; }
        // j-th element of T
        x = T;
        for (int t = 0; t < j; ++t) x &= x - 1;
        const int bit = __builtin_ctzll(x);
        chain[d - 1] = bit;
        T &= ~(1ull << bit);
    }
}

}  // namespace

namespace ulg {

namespace {
int components_gpu(const uint64_t *edges, int n, std::vector<uint64_t> &out) {
    out.clear();
    uint64_t visited = 0;
    for (int v = 0; v < n; ++v) {
        if ((visited >> v) & 1ull) continue;
        uint64_t comp = 1ull << v;
        visited |= comp;
        std::vector<int> st{v};
        while (!st.empty()) {
            const int cur = st.back();
            st.pop_back();
            for (int i = 0; i < n; ++i)
                if (!((visited >> i) & 1ull) && ((edges[cur] >> i) & 1ull)) {
                    visited |= 1ull << i;
                    comp |= 1ull << i;
                    st.push_back(i);
                }
        }
        out.push_back(comp);
    }
    return (int)out.size();
}
}  // namespace

int astar_gpu(ulg_ctx *c, const uint64_t *edges, uint64_t *vpar, int *order, float *goal_cost, int64_t *expanded) {
    SearchState &s = *c->search;
    const int n = s.n;
    const uint64_t all = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    std::vector<uint64_t> comps;
    if (edges) components_gpu(edges, n, comps);
    else comps.push_back(all);
    // binomials C(a, b), a, b <= 32
    std::vector<uint64_t> bn(33 * 33, 0);
    for (int a = 0; a <= 32; ++a)
        for (int b = 0; b <= 32; ++b) bn[a * 33 + b] = binom64(a, b);
    DevBuf<uint64_t> d_bn, d_edges, d_layer_off;
    DevBuf<int> d_cv, d_chain;
    DevBuf<float> d_g0, d_g1;
    DevBuf<uint8_t> d_leaf;
    DevBuf<unsigned long long> d_acc;
    auto cleanup = [&]() {
        release(d_bn); release(d_edges); release(d_layer_off); release(d_cv); release(d_chain);
        release(d_g0); release(d_g1); release(d_leaf); release(d_acc);
    };
    int rc;
    if ((rc = ensure(c, d_bn, bn.size())) || (rc = ensure(c, d_edges, 64)) || (rc = ensure(c, d_cv, kMaxM)) ||
        (rc = ensure(c, d_chain, kMaxM)) || (rc = ensure(c, d_acc, kCounters))) {
        cleanup();
        return rc;
    }
    hipError_t e = hipMemcpyAsync(d_bn.p, bn.data(), bn.size() * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && edges) e = hipMemcpyAsync(d_edges.p, edges, (size_t)n * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d_acc.p, 0, kCounters * 8, c->stream);
    if (e != hipSuccess) { cleanup(); return set_err(c, ULG_ERR_HIP, hipGetErrorString(e)); }
    const SearchDev dv = s.dev();
    bool symmetric = edges != nullptr;  // off-diagonal rows mirror each other
    for (int i = 0; i < n && symmetric; ++i)
        for (int j = 0; j < n; ++j)
            if (i != j && (((edges[i] >> j) ^ (edges[j] >> i)) & 1ull)) {
                symmetric = false;
                break;
            }
    bool fail = false;
    for (uint64_t comp : comps) {
        const int m = __builtin_popcountll(comp);
        if (m > kMaxM) { cleanup(); return set_err(c, ULG_ERR_UNSUPPORTED, "ulg_astar(GPU): component larger than 32 variables"); }
        std::vector<int> cv;
        for (int b = 0; b < n; ++b)
            if ((comp >> b) & 1ull) cv.push_back(b);
        std::vector<uint64_t> loff(m + 2, 0);
        uint64_t maxl = 1;
        for (int d = 0; d <= m; ++d) {
            loff[d + 1] = loff[d] + binom64(m, d);
            maxl = std::max<uint64_t>(maxl, binom64(m, d));
        }
        if ((rc = ensure(c, d_g0, maxl)) || (rc = ensure(c, d_g1, maxl)) || (rc = ensure(c, d_leaf, loff[m + 1])) ||
            (rc = ensure(c, d_layer_off, (size_t)m + 2))) {
            cleanup();
            return rc;
        }
        e = hipMemcpyAsync(d_cv.p, cv.data(), (size_t)m * 4, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(d_layer_off.p, loff.data(), (size_t)(m + 2) * 8, hipMemcpyHostToDevice, c->stream);
        // root: g = 0 (Node(0.0f, 0.0f, ancestors, leaf), astar_main.cpp:236)
        const float zero = 0.0f;
        if (e == hipSuccess) e = hipMemcpyAsync(d_g0.p, &zero, 4, hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) { cleanup(); return set_err(c, ULG_ERR_HIP, hipGetErrorString(e)); }
        float *gprev = d_g0.p, *gcur = d_g1.p;
        // a skeleton complete on the component filters nothing (a non-empty
        // P always meets the leaf's row) and leaves every subset connected:
        // the launches skip the filter and the connectivity test
        bool complete = true;
        for (uint64_t x = edges ? comp : 0ull; x; x &= x - 1) {
            const int b = __builtin_ctzll(x);
            if (comp & ~(edges[b] | (1ull << b))) complete = false;
        }
        const int filt = edges && !complete ? 1 : 0;
        // sweep table for launches without the filter (full / complete skeleton)
        const uint64_t half = m >= 1 ? (1ull << (m - 1)) : 1ull;
        std::vector<uint64_t> loffm1(kMaxM + 1, 0);
        for (int p = 0; p < m; ++p) loffm1[p + 1] = loffm1[p] + binom64(m - 1, p);
        bool use_w = !filt && m >= 2 && c->sweep_table != 0;
        if (use_w && !(s.sweep_ready && s.sweep_comp == comp)) {
            s.sweep_ready = false;
            size_t free_b = 0, tot_b = 0;
            e = hipMemGetInfo(&free_b, &tot_b);
            const uint64_t need = (uint64_t)m * half;
            if (e != hipSuccess || need * 4 + ((size_t)1 << 30) > free_b + (size_t)s.d_sweep_w.cap * 4) {
                use_w = false;  // no room: the lattice-read launches
            } else {
                DevBuf<uint64_t> d_lo;
                if ((rc = ensure(c, s.d_sweep_w, (size_t)need)) || (rc = ensure(c, d_lo, kMaxM + 1))) {
                    release(d_lo);
                    cleanup();
                    return rc;
                }
                e = hipMemcpyAsync(d_lo.p, loffm1.data(), (kMaxM + 1) * 8, hipMemcpyHostToDevice, c->stream);
                if (e == hipSuccess) {
                    prof_begin(c, "search_sweep_w");
                    sweep_w_kernel<<<dim3((unsigned)((half + kB - 1) / kB), (unsigned)m), kB, 0, c->stream>>>(
                        dv, d_bn.p, d_lo.p, d_cv.p, m, half, s.d_sweep_w.p);
                    prof_end(c);
                    e = hipGetLastError();
                }
                if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
                release(d_lo);
                if (e != hipSuccess) { cleanup(); return set_err(c, ULG_ERR_HIP, hipGetErrorString(e)); }
                s.sweep_ready = true;
                s.sweep_comp = comp;
            }
        }
        for (int d = 1; d <= m; ++d) {
            const uint64_t cnt = binom64(m, d);
            LayerArgs a{dv, d_bn.p, d_cv.p, d_edges.p, filt, symmetric && filt ? 1 : 0, m, d, cnt, gprev, gcur,
                        d_leaf.p + loff[d], d < m ? d_acc.p : nullptr,
                        use_w ? s.d_sweep_w.p : nullptr, half, loffm1[d - 1]};
            prof_begin(c, "search_layer_pull");
            if (use_w) layer_pull_kernel<true><<<(unsigned)((cnt + kB - 1) / kB), kB, 0, c->stream>>>(a);
            else layer_pull_kernel<false><<<(unsigned)((cnt + kB - 1) / kB), kB, 0, c->stream>>>(a);
            prof_end(c);
            std::swap(gprev, gcur);
        }
        reconstruct_kernel<<<1, 1, 0, c->stream>>>(d_leaf.p, d_layer_off.p, d_bn.p, m, d_chain.p);
        e = hipGetLastError();
        float g = 0.0f;
        std::vector<int> chain(m);
        if (e == hipSuccess) e = hipMemcpyAsync(&g, gprev, 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(chain.data(), d_chain.p, (size_t)m * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) { cleanup(); return set_err(c, ULG_ERR_HIP, hipGetErrorString(e)); }
        if (!(g < FLT_MAX) || std::find(chain.begin(), chain.end(), -1) != chain.end()) { fail = true; continue; }
        // reconstruction as reconstructSolution: leaf order and getParents(remaining)
        std::vector<int> total(n, 0), qv(m);
        std::vector<uint64_t> qs(m), opt(n, 0), qp(m);
        std::vector<float> qc(m);
        uint64_t remaining = comp;
        for (int i = m - 1; i >= 0; --i) {
            const int leaf = cv[chain[i]];
            total[i] = leaf;
            qv[i] = leaf;
            qs[i] = remaining;
            remaining &= ~(1ull << leaf);
        }
        if ((rc = search_query(c, m, qv.data(), qs.data(), qc.data(), qp.data()))) { cleanup(); return rc; }
        for (int i = 0; i < m; ++i) opt[i] = qp[i];
        for (int v = 0; v < n; ++v) vpar[v] = 0;
        for (int v = 0; v < n; ++v) vpar[total[v]] = opt[v];
        for (int v = 0; v < n; ++v) order[v] = total[v];
        *goal_cost = g;
    }
    std::vector<unsigned long long> acc(kCounters, 0);
    e = hipMemcpyAsync(acc.data(), d_acc.p, kCounters * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    prof_collect(c);
    cleanup();
    if (e != hipSuccess) return set_err(c, ULG_ERR_HIP, hipGetErrorString(e));
    int64_t total_reached = (int64_t)comps.size();  // every component's root (layer 0)
    for (unsigned long long x : acc) total_reached += (int64_t)x;
    *expanded = total_reached;
    if (fail) return set_err(c, ULG_ERR_STATE, "ulg_astar(GPU): a component has no goal");
    return ULG_OK;
}

}  // namespace ulg
