// search_exact.h -- building blocks of the exact-order host search shared by
// ulg_astar (search_host.cpp) and ulg_triplet_astar (triplet_host.cpp): the
// node record, the host view of the GPU-built best-score lattice and pattern
// databases, the generated-node index and the reference's heap
// (priority_queue/priority_queue-inl.h:19-234, base/node.h:124-135).
#pragma once
#include <cfloat>
#include <cmath>
#include <vector>

#include "search_internal.h"

namespace ulg {
namespace exact {

struct Node {
    float g, h;
    uint64_t sub;
    uint8_t leaf;
    int32_t pq;
};

inline bool g_have_bmi2 = __builtin_cpu_supports("bmi2");

__attribute__((target("bmi2"))) inline uint64_t pext_bmi2(uint64_t x, uint64_t m) { return __builtin_ia32_pext_di(x, m); }

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

// PriorityQueue with the reference's heap algorithms and pqPos bookkeeping.
// Heap entries carry their node's f = g + h and layer, so a comparison reads
// the (mostly contiguous) heap array instead of two random Node records.
// Invariant: every entry's f is its node's current g + h -- what the
// reference's comparator reads through the node pointer.  A decrease-key
// refreshes the entry at the node's recorded position; when that position is
// stale (the reference's __down_heap does not record moves), the node's own
// entry is found by a scan and refreshed, and the stale slot is sifted as the
// reference sifts it.
struct HeapEnt {
    float f;
    int32_t layer;
    uint32_t idx;
};

struct Heap {
    std::vector<HeapEnt> a;
    std::vector<Node> *nodes;
    bool hang = false;

    inline HeapEnt ent(uint32_t x) const {
        const Node &N = (*nodes)[x];
        return HeapEnt{N.g + N.h, __builtin_popcountll(N.sub) & 0xff, x};
    }
    // CompareNodeStar: true if x has LOWER priority than y
    static inline bool cns(const HeapEnt &A, const HeapEnt &B) {
        const float diff = A.f - B.f;
        if (std::fabs(diff) < FLT_EPSILON) return (B.layer - A.layer) > 0;
        return diff > 0;
    }
    inline void setpos(const HeapEnt &e, int64_t p) { (*nodes)[e.idx].pq = (int32_t)p; }
    void push_hole(int64_t hole, int64_t top, HeapEnt value) {
        int64_t parent = (hole - 1) / 2;
        while (hole > top && cns(a[parent], value)) {
            a[hole] = a[parent];
            setpos(a[hole], hole);
            hole = parent;
            parent = (hole - 1) / 2;
        }
        a[hole] = value;
        setpos(value, hole);
    }
    void push(uint32_t x) {
        const HeapEnt e = ent(x);
        a.push_back(e);
        push_hole((int64_t)a.size() - 1, 0, e);
    }
    void adjust(int64_t hole, int64_t len, HeapEnt value) {
        const int64_t top = hole;
        int64_t second = hole;
        // the moved nodes' pq writes are deferred (in order) behind write
        // prefetches: nothing reads pq during the sift
        uint32_t mv_idx[64];
        int64_t mv_pos[64];
        int nm = 0;
        while (second < (len - 1) / 2) {
            // the grandchildren (4 contiguous entries): the heap outgrows the
            // caches, and this descent is a chain of dependent loads
            const int64_t gc = 4 * second + 3;
            if (gc + 3 < len) {
                __builtin_prefetch(&a[gc]);
                __builtin_prefetch(&a[gc + 3]);
            }
            second = 2 * (second + 1);
            if (cns(a[second], a[second - 1])) second--;
            a[hole] = a[second];
            __builtin_prefetch(&(*nodes)[a[hole].idx], 1);
            mv_idx[nm] = a[hole].idx;
            mv_pos[nm++] = hole;
            hole = second;
        }
        if ((len & 1) == 0 && second == (len - 2) / 2) {
            second = 2 * (second + 1);
            a[hole] = a[second - 1];
            mv_idx[nm] = a[hole].idx;
            mv_pos[nm++] = hole;
            hole = second - 1;
        }
        for (int i = 0; i < nm; ++i) (*nodes)[mv_idx[i]].pq = (int32_t)mv_pos[i];
        push_hole(hole, top, value);
    }
    uint32_t pop() {
        const uint32_t ret = a[0].idx;
        const int64_t last = (int64_t)a.size() - 1;
        const HeapEnt value = a[last];
        a[last] = a[0];
        adjust(0, last, value);
        a.pop_back();
        return ret;
    }
    void update(uint32_t x) {
        const int64_t pos = (*nodes)[x].pq;
        const float fx = (*nodes)[x].g + (*nodes)[x].h;
        // the reference reads whatever node sits at the recorded position
        // (capacity memory included, as the vector keeps it)
        HeapEnt value = a.data()[pos];
        if (value.idx == x && pos < (int64_t)a.size()) {
            value.f = fx;
            a[pos].f = fx;
        } else {
            for (HeapEnt &e : a)
                if (e.idx == x) e.f = fx;
            value.f = (*nodes)[value.idx].g + (*nodes)[value.idx].h;
        }
        const int64_t parent = (pos - 1) / 2;
        if (pos > 0 && cns(a[parent], value)) {
            int64_t par = (pos - 1) / 2, index = pos;
            while (index > 0 && cns(a[par], value)) {
                a[index] = a[par];
                setpos(a[index], index);
                index = par;
                par = (par - 1) / 2;
            }
            if (pos != index) {
                a[index] = value;
                setpos(value, index);
            }
        } else {
            // __down_heap as written: follows the left child only and does not
            // record the moved value's position (priority_queue-inl.h:176-208)
            const int64_t len = (int64_t)a.size();
            int64_t index = pos, left = 2 * index + 1, right = 2 * index + 2, largest = len, guard = 0;
            while (index < len) {
                if ((right >= len) || ((left < len) && cns(a[right], a[left]))) largest = left;
                if (largest < len && cns(value, a[largest])) {
                    if (largest == index || ++guard > 128) { hang = true; break; }  // the reference would spin
                    a[index] = a[largest];
                    setpos(a[largest], index);
                    index = largest;
                    left = index * 2 + 1;
                    right = index * 2 + 2;
                } else
                    break;
            }
            if (pos != index) a[index] = value;
        }
    }
};

// HostTables over the SearchState's current tables and pattern database
// (call again after every search_build_pdb: the pd pointers move).
void host_tables(const SearchState &s, HostTables &T);

}  // namespace exact
}  // namespace ulg
