// search_exact.h -- building blocks of the exact-order host search shared by
// ulg_astar (search_host.cpp) and ulg_triplet_astar (triplet_host.cpp): the
// node record, the host view of the GPU-built best-score lattice and pattern
// databases, the generated-node index and the reference's heap
// (priority_queue/priority_queue-inl.h:19-234, base/node.h:124-135).
#pragma once
#include <cfloat>
#include <cmath>
#include <vector>

#include "exact_heap.h"
#include "search_internal.h"

namespace ulg {
namespace exact {



inline bool g_have_bmi2 = __builtin_cpu_supports("bmi2");

__attribute__((target("bmi2"))) inline uint64_t pext_bmi2(uint64_t x, uint64_t m) { return __builtin_ia32_pext_di(x, m); }
__attribute__((target("bmi2"))) inline uint64_t pdep_bmi2(uint64_t x, uint64_t m) { return __builtin_ia32_pdep_di(x, m); }
inline uint64_t pdep64(uint64_t x, uint64_t m) {
    uint64_t r = 0;
    for (uint64_t b = m; b; b &= b - 1, x >>= 1)
        if (x & 1ull) r |= b & (0 - b);
    return r;
}

// Host view of the best-score lattice: cost per subset of D_v.
struct HostTables {
    const float *cost;
    const uint64_t *tb_off;
    const uint64_t *support;
    std::vector<int> hole;  // D_v == all \ {hole}: pext is a shift
    uint64_t all;
    int n;
    const float *pd;
    std::vector<uint64_t> groups;
    std::vector<uint64_t> pd_off;

    inline uint64_t index(int v, uint64_t S) const {
        const uint64_t D = support[v];
        S &= D;
        const int h = hole[v];
        if (h >= 0) return ((S >> (h + 1)) << h) | (S & ((1ull << h) - 1ull));
        return g_have_bmi2 ? pext_bmi2(S, D) : pext64(S, D);
    }
    inline float bs(int v, uint64_t S) const { return cost[tb_off[v] + index(v, S)]; }
    inline void prefetch_bs(int v, uint64_t S) const { __builtin_prefetch(&cost[tb_off[v] + index(v, S)]); }
    inline uint64_t gidx(uint64_t vs, uint64_t grp) const { return g_have_bmi2 ? pext_bmi2(vs, grp) : pext64(vs, grp); }
    // StaticPatternDatabase::h (static_pattern_database.cpp:145-174)
    inline float h(uint64_t S, bool *complete) const {
        const uint64_t remaining = ~S & all;
        float hv = 0.0f;
        for (size_t g = 0; g < groups.size(); ++g) {
            const uint64_t vs = groups[g] & remaining;
            const float val = pd[pd_off[g] + gidx(vs, groups[g])];
            if (vs == remaining) {
                *complete = true;
                return val;
            }
            hv += val;
        }
        return hv;
    }
};

// generatedNodes (NodeMap) over the subsets of one scope: a dense array
// indexed by pext(S, scope) while 2^|scope| x 4 B stays small (one cached
// read per probe, no hashing), else open addressing.
struct SubsetIndex;

// open addressing u64 -> node index
struct NodeIndex {
    std::vector<uint64_t> keys;
    std::vector<uint32_t> vals;
    uint64_t mask = 0, size = 0;
    static constexpr uint64_t kEmpty = ~0ull;
    void init(uint64_t cap) {
        uint64_t c = 1024;
        while (c < cap * 2) c <<= 1;
        keys.assign(c, kEmpty);
        vals.assign(c, 0);
        mask = c - 1;
        size = 0;
    }
    static inline uint64_t mix(uint64_t x) {
        x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
        return x;
    }
    inline int64_t find(uint64_t k) const {
        uint64_t i = mix(k) & mask;
        while (true) {
            const uint64_t kk = keys[i];
            if (kk == k) return vals[i];
            if (kk == kEmpty) return -1;
            i = (i + 1) & mask;
        }
    }
    void grow() {
        std::vector<uint64_t> ok;
        std::vector<uint32_t> ov;
        ok.swap(keys);
        ov.swap(vals);
        init((ok.size()));
        for (size_t i = 0; i < ok.size(); ++i)
            if (ok[i] != kEmpty) insert(ok[i], ov[i]);
    }
    inline void insert(uint64_t k, uint32_t v) {
        if ((size + 1) * 2 > keys.size()) grow();
        uint64_t i = mix(k) & mask;
        while (keys[i] != kEmpty && keys[i] != k) i = (i + 1) & mask;
        if (keys[i] == kEmpty) ++size;
        keys[i] = k;
        vals[i] = v;
    }
};

struct SubsetIndex {
    static constexpr int kDenseBits = 27;  // 512 MB of u32
    uint64_t scope = 0;
    bool dense = false;
    std::vector<uint32_t> slots;
    NodeIndex hash;
    void init(uint64_t the_scope) {
        scope = the_scope;
        dense = __builtin_popcountll(scope) <= kDenseBits;
        if (dense) slots.assign((size_t)1 << __builtin_popcountll(scope), UINT32_MAX);
        else hash.init(1 << 16);
    }
    inline uint64_t slot(uint64_t S) const { return g_have_bmi2 ? pext_bmi2(S, scope) : pext64(S, scope); }
    inline int64_t find(uint64_t S) const {
        if (!dense) return hash.find(S);
        const uint32_t v = slots[slot(S)];
        return v == UINT32_MAX ? -1 : (int64_t)v;
    }
    inline void insert(uint64_t S, uint32_t v) {
        if (dense) slots[slot(S)] = v;
        else hash.insert(S, v);
    }
    inline void prefetch(uint64_t S) const {
        if (dense) __builtin_prefetch(&slots[slot(S)]);
    }
};

// HostTables over the SearchState's current tables and pattern database
// (call again after every search_build_pdb: the pd pointers move).
void host_tables(const SearchState &s, HostTables &T);

}  // namespace exact
}  // namespace ulg
