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
    int xcd;                 // contiguous runs of nodes per XCD (layer_pull_w32_kernel)
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
                                                     const int *comp_vars, int m, uint64_t half, float *w,
                                                     const int *jlist) {
    __shared__ uint64_t binom[33 * 33];
    __shared__ uint64_t lo[kMaxM + 1];
    __shared__ int cv[kMaxM];
    for (int e = threadIdx.x; e < m * 33; e += kB) binom[e] = gbinom[e];
    for (int i = threadIdx.x; i <= m; i += kB) lo[i] = loffm1[i];
    for (int i = threadIdx.x; i < m; i += kB) cv[i] = comp_vars[i];
    __syncthreads();
    const uint64_t f = (uint64_t)blockIdx.x * kB + threadIdx.x;
    const int j = jlist ? jlist[blockIdx.y] : (int)blockIdx.y;  // slice blockIdx.y holds position j
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
    w[(uint64_t)blockIdx.y * half + f] = bs_cost(d, cv[j], Pg);
}

// The same slices when every v_j's lattice is exactly over comp \ {v_j}
// (D_v = the rest of the component, the tables' scope covers it): then slice
// entry (j, p, r) is lattice entry i of v_j with popcount(i) = p and colex
// rank r.  A block takes 2^kTileBits consecutive entries i (one high part H,
// every low part): colex rank = rank of the low part + a term of H and the
// low popcount k only, so the tile's entries land in kTileBits + 1
// contiguous runs of the slice, one per k, C(kTileBits, k) long.  The block
// reads the tile in order, permutes it in LDS into run order and writes the
// runs out contiguously (the previous form wrote each wave's 64 entries as 7
// runs of 1..20 floats: 2.6 ms for C3's 1.68 GB of slices).
constexpr int kTileBits = 12;
// the permutation of a full tile, the same for every tile: entry e (the low
// part) goes to run popcount(e) at its colex rank; run_of[r] = the run of
// run-order position r
struct TilePerm {
    uint16_t dst[1 << kTileBits];
    uint8_t run_of[1 << kTileBits];
};
constexpr TilePerm make_tile_perm() {
    TilePerm t{};
    uint32_t C[kTileBits + 1][kTileBits + 2] = {};
    for (int a = 0; a <= kTileBits; ++a) {
        C[a][0] = 1;
        for (int b = 1; b <= a; ++b) C[a][b] = C[a - 1][b - 1] + (b <= a - 1 ? C[a - 1][b] : 0);
    }
    uint32_t roff[kTileBits + 2] = {};
    for (int k = 0; k <= kTileBits; ++k) roff[k + 1] = roff[k] + C[kTileBits][k];
    for (uint32_t e = 0; e < (1u << kTileBits); ++e) {
        uint32_t rank = 0;
        int tt = 0;
        for (int b = 0; b < kTileBits; ++b)
            if ((e >> b) & 1u) {
                ++tt;
                rank += C[b][tt];
            }
        t.dst[e] = (uint16_t)(roff[tt] + rank);
    }
    for (int k = 0; k <= kTileBits; ++k)
        for (uint32_t r = roff[k]; r < roff[k + 1]; ++r) t.run_of[r] = (uint8_t)k;
    return t;
}
__constant__ TilePerm kTilePerm = make_tile_perm();

__global__ void __launch_bounds__(kB) sweep_w_tile_kernel(const uint32_t *table, const uint64_t *tb_off,
                                                          const uint64_t *gbinom, const uint64_t *loffm1,
                                                          const int *comp_vars, const int *jlist, int m,
                                                          uint64_t half, float *w) {
    __shared__ uint32_t binom[33 * 33];
    __shared__ uint32_t lo[kMaxM + 1];
    __shared__ float tile[1 << kTileBits];
    __shared__ uint32_t roff[kTileBits + 2];
    __shared__ uint32_t rbase[kTileBits + 1];
    for (int e = threadIdx.x; e < m * 33; e += kB) binom[e] = (uint32_t)gbinom[e];
    for (int i = threadIdx.x; i <= m; i += kB) lo[i] = (uint32_t)loffm1[i];
    __syncthreads();
    const int lb = m - 1 < kTileBits ? m - 1 : kTileBits;
    const uint32_t tn = 1u << lb;
    const uint64_t H = (uint64_t)blockIdx.x << lb;  // the tile's high part
    const int j = jlist ? jlist[blockIdx.y] : (int)blockIdx.y;
    const uint32_t *tv = table + tb_off[comp_vars[j]];
    float *wj = w + (uint64_t)blockIdx.y * half;
    if (threadIdx.x <= (unsigned)lb) {
        const int k = (int)threadIdx.x;  // low popcount
        uint32_t o = 0;
        for (int kk = 0; kk < k; ++kk) o += binom[lb * 33 + kk];
        roff[k] = o;
        if (k == lb) roff[lb + 1] = tn;
        uint32_t rank = 0;
        int t = k;
        for (uint64_t x = H; x; x &= x - 1) rank += binom[__builtin_ctzll(x) * 33 + (++t)];
        rbase[k] = lo[t] + rank;  // t = k + popcount(H): the slice's layer
    }
    __syncthreads();
    if (lb == kTileBits) {
        for (uint32_t e = threadIdx.x; e < tn; e += kB) tile[kTilePerm.dst[e]] = ord_cost(tv[H + e]);
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < tn; e += kB) {
            const int k = kTilePerm.run_of[e];
            wj[rbase[k] + (e - roff[k])] = tile[e];
        }
        return;
    }
    for (uint32_t e = threadIdx.x; e < tn; e += kB) {  // a component of <= kTileBits + 1 variables
        uint32_t rank = 0;
        int t = 0;
        for (uint32_t x = e; x; x &= x - 1) rank += binom[__builtin_ctz(x) * 33 + (++t)];
        tile[roff[t] + rank] = ord_cost(tv[H + e]);
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < tn; e += kB) {
        int k = 0;
        while (roff[k + 1] <= e) ++k;
        wj[rbase[k] + (e - roff[k])] = tile[e];
    }
}

// ---- sweep with the tables sharded by variable (n >= 31) --------------
// Rank r holds the best-score tables (and sweep slices) of its own variables
// only.  Per layer every rank computes, for every node T, the best candidate
// over the leaves it owns as the key (ordkey(cost) << 8 | leaf position), the
// caller MIN-all-reduces the keys over the ranks (the smallest cost, then the
// smallest leaf position: the single-GPU sweep's first-strict-minimum rule),
// and commit turns the reduced keys into the layer's g and leaf bytes.
constexpr uint64_t kUnreachedKey = 0xFFFFFFFFFFull;  // above every (ordkey << 8 | j)

struct ShardArgs {
    const uint64_t *binom;  // [33][33]
    const int *wslot;       // [m]: slice of compact position j, -1 if not owned
    int m, layer;
    uint64_t count;
    const float *gprev;
    const float *w;
    uint64_t w_half, w_layer;
    uint64_t *keys;
};

__global__ void __launch_bounds__(kB) layer_shard_kernel(ShardArgs a) {
    __shared__ uint64_t binom[33 * 33];
    __shared__ int ws[kMaxM];
    {
        const int cols = a.layer + 1;
        for (int e = threadIdx.x; e < a.m * cols; e += kB) {
            const int r = e / cols, i = e - r * cols;
            binom[r * 33 + i] = a.binom[r * 33 + i];
        }
    }
    for (int i = threadIdx.x; i < a.m; i += kB) ws[i] = a.wslot[i];
    __syncthreads();
    const uint64_t r = (uint64_t)blockIdx.x * kB + threadIdx.x;
    const int L = a.layer;
    if (r >= a.count) return;
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
    uint64_t suffix = 0, suffixc = 0;
    {
        int i = 0;
        for (uint64_t x = Tc; x; x &= x - 1, ++i)
            if (i >= 1) {
                const int ai = __builtin_ctzll(x);
                suffix += Bn(binom, ai, i);
                suffixc += Bn(binom, ai - 1, i);
            }
    }
    uint64_t prefix = 0, best = kUnreachedKey;
    uint64_t x = Tc;
    for (int j = 0; j < L; ++j) {
        const int aj = __builtin_ctzll(x);
        x &= x - 1;
        const int sl = ws[aj];
        if (sl >= 0) {
            const float gp = a.gprev[prefix + suffix];
            if (gp < FLT_MAX) {
                const float cand = gp + a.w[(uint64_t)sl * a.w_half + a.w_layer + prefix + suffixc];
                const uint64_t k = ((uint64_t)ordkey(cand) << 8) | (uint64_t)j;
                best = k < best ? k : best;
            }
        }
        if (x) {
            const int an = __builtin_ctzll(x);
            suffix -= Bn(binom, an, j + 1);
            suffixc -= Bn(binom, an - 1, j + 1);
        }
        prefix += Bn(binom, aj, j + 1);
    }
    a.keys[r] = best;
}

__global__ void __launch_bounds__(kB) shard_commit_kernel(const uint64_t *keys, uint64_t count, float *g, uint8_t *leaf,
                                                          unsigned long long *reached) {
    const uint64_t r = (uint64_t)blockIdx.x * kB + threadIdx.x;
    bool hit = false;
    if (r < count) {
        const uint64_t k = keys[r];
        hit = k != kUnreachedKey;
        g[r] = hit ? ord_cost((uint32_t)(k >> 8)) : FLT_MAX;
        leaf[r] = hit ? (uint8_t)(k & 0xffull) : (uint8_t)255;
    }
    const unsigned long long b = __ballot(hit);
    if (reached && (threadIdx.x & 63) == 0 && b) atomicAdd(&reached[blockIdx.x % kCounters], (unsigned long long)__popcll(b));
}

// The sweep-slice launch in 32-bit index arithmetic: on a component of
// m <= 32 variables every colex rank of a layer, C(m, L) <= C(32, 16) < 2^32,
// and every slice offset below 2^(m-1) fit in 32 bits, so the unrank and the
// per-leaf rank updates are single VALU ops (the 64-bit form spends ~1000 VALU
// instructions per node, PMC pass profiles/r2/pmc_r2.json).  Same results as
// layer_pull_kernel<true>.
constexpr int kPullPer = 1;  // nodes per thread, kB apart (4 measured slower: 1.53 -> 2.06 ms per C3 sweep)
__global__ void __launch_bounds__(kB) layer_pull_w32_kernel(LayerArgs a) {
    __shared__ uint32_t binom[33 * 33];
    {
        const int cols = a.layer + 1;
        for (int e = threadIdx.x; e < a.m * cols; e += kB) {
            const int r = e / cols, i = e - r * cols;
            binom[r * 33 + i] = (uint32_t)a.binom[r * 33 + i];
        }
    }
    __syncthreads();
    const int L = a.layer;
    // block b runs on XCD b % 8; with xcd, XCD x takes the x-th contiguous
    // eighth of the layer (colex-near nodes share predecessors and slice runs
    // in that XCD's L2)
    uint32_t bl = blockIdx.x;
    if (a.xcd) {
        const uint32_t nb = gridDim.x, x = bl & 7u, kk = bl >> 3, q = nb >> 3, rr = nb & 7u;
        bl = x * q + (x < rr ? x : rr) + kk;
    }
    for (int k = 0; k < kPullPer; ++k) {
    const uint32_t r = (bl * kPullPer + k) * kB + threadIdx.x;
    if ((uint64_t)r >= a.count) return;
    uint32_t Tc = 0;
    {
        uint32_t rr = r;
        int c = a.m - 1;
        for (int i = L; i >= 1; --i) {
            while (binom[c * 33 + i] > rr) --c;
            Tc |= 1u << c;
            rr -= binom[c * 33 + i];
            --c;
        }
    }
    uint32_t suffix = 0, suffixc = 0;
    {
        int i = 0;
        for (uint32_t x = Tc; x; x &= x - 1, ++i)
            if (i >= 1) {
                const int ai = __builtin_ctz(x);
                suffix += binom[ai * 33 + i];
                suffixc += binom[(ai - 1) * 33 + i];
            }
    }
    const uint32_t wl = (uint32_t)a.w_layer;
    uint32_t prefix = 0;
    float best = FLT_MAX;
    int bestj = 255;
    bool reached = false;
    uint32_t x = Tc;
    for (int j = 0; j < L; ++j) {
        const int aj = __builtin_ctz(x);
        x &= x - 1;
        const float gp = a.gprev[prefix + suffix];
        if (gp < FLT_MAX) {
            reached = true;
            const float cand = gp + a.w[(uint64_t)aj * a.w_half + (wl + prefix + suffixc)];
            if (cand < best || bestj == 255) {
                best = cand;
                bestj = j;
            }
        }
        if (x) {
            const int an = __builtin_ctz(x);
            suffix -= binom[an * 33 + j + 1];
            suffixc -= binom[(an - 1) * 33 + j + 1];
        }
        prefix += binom[aj * 33 + j + 1];
    }
    a.gcur[r] = reached ? best : FLT_MAX;
    a.leaf[r] = (uint8_t)(reached ? bestj : 255);
    if (a.reached) {
        const unsigned long long b = __ballot(reached);
        if ((threadIdx.x & 63) == __ffsll((long long)__ballot(true)) - 1 && b)
            atomicAdd(&a.reached[blockIdx.x % kCounters], (unsigned long long)__popcll(b));
    }
    }
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

// every variable of comp has a lattice over exactly the rest of comp
bool sweep_scatter_ok(const SearchState &s, uint64_t comp) {
    if (!s.tables_ready || (comp & ~s.scope)) return false;
    for (uint64_t x = comp; x; x &= x - 1) {
        const int v = __builtin_ctzll(x);
        if (!((s.table_vars >> v) & 1ull) || s.support[v] != (comp & ~(1ull << v))) return false;
    }
    return true;
}

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
    // the sweep's buffers persist in the search state (no allocation per call)
    DevBuf<uint64_t> &d_bn = s.gs_bn, &d_edges = s.gs_edges, &d_layer_off = s.gs_layer_off;
    DevBuf<int> &d_cv = s.gs_cv, &d_chain = s.gs_chain;
    DevBuf<float> &d_g0 = s.gs_g0, &d_g1 = s.gs_g1;
    DevBuf<uint8_t> &d_leaf = s.gs_leaf;
    DevBuf<unsigned long long> &d_acc = s.gs_acc;
    auto cleanup = [&]() {};
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
                    if (sweep_scatter_ok(s, comp))
                        sweep_w_tile_kernel<<<dim3((unsigned)(half >> std::min(m - 1, kTileBits)), (unsigned)m), kB, 0,
                                              c->stream>>>(s.d_table.p, s.d_tb_off.p, d_bn.p, d_lo.p, d_cv.p, nullptr,
                                                           m, half, s.d_sweep_w.p);
                    else
                        sweep_w_kernel<<<dim3((unsigned)((half + kB - 1) / kB), (unsigned)m), kB, 0, c->stream>>>(
                            dv, d_bn.p, d_lo.p, d_cv.p, m, half, s.d_sweep_w.p, nullptr);
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
                        use_w ? s.d_sweep_w.p : nullptr, half, loffm1[d - 1], c->sweep_xcd};
            prof_begin(c, "search_layer_pull");
            if (use_w && c->sweep_table == 1)
                layer_pull_w32_kernel<<<(unsigned)((cnt + kB * kPullPer - 1) / (kB * kPullPer)), kB, 0, c->stream>>>(a);
            else if (use_w) layer_pull_kernel<true><<<(unsigned)((cnt + kB - 1) / kB), kB, 0, c->stream>>>(a);
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

// ---- variable-sharded sweep -------------------------------------------------
namespace {
std::vector<uint64_t> layer_offsets(int m) {
    std::vector<uint64_t> loff(m + 2, 0);
    for (int d = 0; d <= m; ++d) loff[d + 1] = loff[d] + binom64(m, d);
    return loff;
}
}  // namespace

int sweep_shard_begin(ulg_ctx *c, uint64_t own, int64_t *max_nodes) {
    SearchState &s = *c->search;
    const int n = s.n;
    const uint64_t all = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    if (n < 2 || n > kMaxM) return set_err(c, ULG_ERR_UNSUPPORTED, "ulg_sweep_shard_begin: 2..32 variables");
    if (own == 0 || (own & ~all)) return set_err(c, ULG_ERR_ARG, "ulg_sweep_shard_begin: bad variable mask");
    s.shard_active = false;
    // this rank's tables (every stored set of its variables, over every variable)
    int rc = search_build_tables(c, all, own);
    if (rc) return rc;
    s.sweep_ready = false;  // d_sweep_w now holds this rank's slices
    const int m = n;
    const uint64_t half = 1ull << (m - 1);
    std::vector<int> wslot(m, -1), jlist;
    for (int v = 0; v < m; ++v)
        if ((own >> v) & 1ull) {
            wslot[v] = (int)jlist.size();
            jlist.push_back(v);
        }
    const int nown = (int)jlist.size();
    std::vector<uint64_t> bn(33 * 33, 0);
    for (int a = 0; a <= 32; ++a)
        for (int b = 0; b <= 32; ++b) bn[a * 33 + b] = binom64(a, b);
    const std::vector<uint64_t> loff = layer_offsets(m);
    std::vector<uint64_t> loffm1(kMaxM + 1, 0);
    for (int p = 0; p < m; ++p) loffm1[p + 1] = loffm1[p] + binom64(m - 1, p);
    uint64_t maxl = 1;
    for (int d = 0; d <= m; ++d) maxl = std::max<uint64_t>(maxl, binom64(m, d));
    std::vector<int> cv(m);
    for (int v = 0; v < m; ++v) cv[v] = v;
    DevBuf<uint64_t> d_lo;
    DevBuf<int> d_jl;
    if ((rc = ensure(c, s.d_sweep_w, (size_t)((uint64_t)nown * half))) || (rc = ensure(c, d_lo, kMaxM + 1)) ||
        (rc = ensure(c, d_jl, (size_t)nown)) || (rc = ensure(c, s.shard_bn, bn.size())) ||
        (rc = ensure(c, s.shard_loff, loff.size())) || (rc = ensure(c, s.shard_wslot, (size_t)m)) ||
        (rc = ensure(c, s.shard_cv, (size_t)m)) || (rc = ensure(c, s.shard_chain, kMaxM)) ||
        (rc = ensure(c, s.shard_g0, (size_t)maxl)) || (rc = ensure(c, s.shard_g1, (size_t)maxl)) ||
        (rc = ensure(c, s.shard_leaf, (size_t)loff[m + 1])) || (rc = ensure(c, s.shard_acc, kCounters))) {
        release(d_lo);
        release(d_jl);
        return rc;
    }
    hipError_t e = hipMemcpyAsync(d_lo.p, loffm1.data(), (kMaxM + 1) * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_jl.p, jlist.data(), (size_t)nown * 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.shard_bn.p, bn.data(), bn.size() * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.shard_loff.p, loff.data(), loff.size() * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.shard_wslot.p, wslot.data(), (size_t)m * 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.shard_cv.p, cv.data(), (size_t)m * 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s.shard_acc.p, 0, kCounters * 8, c->stream);
    const float zero = 0.0f;  // root: g = 0 (astar_main.cpp:236)
    if (e == hipSuccess) e = hipMemcpyAsync(s.shard_g0.p, &zero, 4, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        prof_begin(c, "search_sweep_w");
        bool scatter = true;
        for (uint64_t x = own; x; x &= x - 1) {
            const int v = __builtin_ctzll(x);
            if (s.support[v] != (all & ~(1ull << v))) scatter = false;
        }
        if (scatter)
            sweep_w_tile_kernel<<<dim3((unsigned)(half >> std::min(m - 1, kTileBits)), (unsigned)nown), kB, 0,
                                  c->stream>>>(s.d_table.p, s.d_tb_off.p, s.shard_bn.p, d_lo.p, s.shard_cv.p, d_jl.p, m,
                                               half, s.d_sweep_w.p);
        else
            sweep_w_kernel<<<dim3((unsigned)((half + kB - 1) / kB), (unsigned)nown), kB, 0, c->stream>>>(
                s.dev(), s.shard_bn.p, d_lo.p, s.shard_cv.p, m, half, s.d_sweep_w.p, d_jl.p);
        prof_end(c);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    release(d_lo);
    release(d_jl);
    if (e != hipSuccess) return set_err(c, ULG_ERR_HIP, hipGetErrorString(e));
    prof_collect(c);
    s.shard_own = own;
    s.shard_layer = 0;
    s.shard_active = true;
    *max_nodes = (int64_t)maxl;
    return ULG_OK;
}

int sweep_shard_layer(ulg_ctx *c, int layer, uint64_t *keys) {
    SearchState &s = *c->search;
    const int m = s.n;
    if (!s.shard_active || layer != s.shard_layer + 1 || layer > m)
        return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_layer: layers go 1..n, each after the previous commit");
    const uint64_t cnt = binom64(m, layer);
    const float *gprev = (layer & 1) ? s.shard_g0.p : s.shard_g1.p;  // layer d's g lives in g[d & 1]
    uint64_t wl = 0;
    for (int p = 0; p < layer - 1; ++p) wl += binom64(m - 1, p);
    ShardArgs a{s.shard_bn.p, s.shard_wslot.p, m, layer, cnt, gprev, s.d_sweep_w.p, 1ull << (m - 1), wl, keys};
    prof_begin(c, "search_shard_layer");
    layer_shard_kernel<<<(unsigned)((cnt + kB - 1) / kB), kB, 0, c->stream>>>(a);
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    ULG_HIP(c, hipStreamSynchronize(c->stream));  // the caller's collective reads the keys next
    prof_collect(c);
    return ULG_OK;
}

int sweep_shard_commit(ulg_ctx *c, int layer, const uint64_t *keys) {
    SearchState &s = *c->search;
    const int m = s.n;
    if (!s.shard_active || layer != s.shard_layer + 1 || layer > m)
        return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_commit: commit the layer just computed");
    const uint64_t cnt = binom64(m, layer);
    float *gcur = (layer & 1) ? s.shard_g1.p : s.shard_g0.p;
    const std::vector<uint64_t> loff = layer_offsets(m);
    prof_begin(c, "search_shard_commit");
    shard_commit_kernel<<<(unsigned)((cnt + kB - 1) / kB), kB, 0, c->stream>>>(
        keys, cnt, gcur, s.shard_leaf.p + loff[layer], layer < m ? s.shard_acc.p : nullptr);
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    s.shard_layer = layer;
    return ULG_OK;
}

int sweep_shard_end(ulg_ctx *c, uint64_t *vpar, int *order, float *goal_cost, int64_t *expanded) {
    SearchState &s = *c->search;
    const int n = s.n, m = n;
    if (!s.shard_active || s.shard_layer != m) return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_end: layers not done");
    reconstruct_kernel<<<1, 1, 0, c->stream>>>(s.shard_leaf.p, s.shard_loff.p, s.shard_bn.p, m, s.shard_chain.p);
    ULG_HIP(c, hipGetLastError());
    float g = 0.0f;
    std::vector<int> chain(m);
    std::vector<unsigned long long> acc(kCounters, 0);
    const float *ggoal = (m & 1) ? s.shard_g1.p : s.shard_g0.p;
    ULG_HIP(c, hipMemcpyAsync(&g, ggoal, 4, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipMemcpyAsync(chain.data(), s.shard_chain.p, (size_t)m * 4, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipMemcpyAsync(acc.data(), s.shard_acc.p, kCounters * 8, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    s.shard_active = false;
    if (!(g < FLT_MAX) || std::find(chain.begin(), chain.end(), -1) != chain.end())
        return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_end: no goal");
    std::vector<int> total(n, 0), qv(m);
    std::vector<uint64_t> qs(m), qp(m);
    std::vector<float> qc(m);
    uint64_t remaining = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    for (int i = m - 1; i >= 0; --i) {
        const int leaf = chain[i];
        total[i] = leaf;
        qv[i] = leaf;
        qs[i] = remaining;
        remaining &= ~(1ull << leaf);
    }
    int rc = search_query(c, m, qv.data(), qs.data(), qc.data(), qp.data());
    if (rc) return rc;
    for (int v = 0; v < n; ++v) vpar[v] = 0;
    for (int i = 0; i < m; ++i) vpar[total[i]] = qp[i];
    for (int v = 0; v < n; ++v) order[v] = total[v];
    *goal_cost = g;
    int64_t reached = 1;  // the root
    for (unsigned long long x : acc) reached += (int64_t)x;
    *expanded = reached;
    return ULG_OK;
}

}  // namespace ulg

extern "C" {

int ulg_sweep_shard_begin(ulg_ctx *c, uint64_t own, int64_t *max_layer_nodes) {
    if (!c || !max_layer_nodes) return ULG_ERR_ARG;
    if (!c->search || !c->search->lists_ready) return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_begin: no parent-set lists");
    ULG_HIP(c, hipSetDevice(c->device));
    return ulg::sweep_shard_begin(c, own, max_layer_nodes);
}

int ulg_sweep_shard_layer(ulg_ctx *c, int layer, uint64_t *keys_dev) {
    if (!c || !keys_dev) return ULG_ERR_ARG;
    if (!c->search) return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_layer: no search state");
    ULG_HIP(c, hipSetDevice(c->device));
    return ulg::sweep_shard_layer(c, layer, keys_dev);
}

int ulg_sweep_shard_commit(ulg_ctx *c, int layer, const uint64_t *keys_dev) {
    if (!c || !keys_dev) return ULG_ERR_ARG;
    if (!c->search) return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_commit: no search state");
    ULG_HIP(c, hipSetDevice(c->device));
    return ulg::sweep_shard_commit(c, layer, keys_dev);
}

int ulg_sweep_shard_end(ulg_ctx *c, uint64_t *vpar, int *order, float *goal_cost, int64_t *expanded) {
    if (!c || !vpar || !order || !goal_cost || !expanded) return ULG_ERR_ARG;
    if (!c->search) return set_err(c, ULG_ERR_STATE, "ulg_sweep_shard_end: no search state");
    ULG_HIP(c, hipSetDevice(c->device));
    return ulg::sweep_shard_end(c, vpar, order, goal_cost, expanded);
}

}  // extern "C"
