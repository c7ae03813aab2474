// exact_heap.h -- the reference's priority queue for the exact-order A*
// replays, in plain C++ (no HIP): used by search_host.cpp / triplet_host.cpp
// and by the sanitizer build's differential check (host/heap_check.cpp).
//
// Both heaps reproduce PriorityQueue (priority_queue/priority_queue.cpp:36-64)
// over libstdc++'s heap algorithms as the reference modified them
// (priority_queue/priority_queue-inl.h:19-234): push_heap/__adjust_heap with
// pqPos bookkeeping, update = __up_heap or the left-child-only __down_heap
// that does not record the moved value's position, and the comparator
// CompareNodeStar (base/node.h:124-135: |f_a - f_b| < FLT_EPSILON -> the
// deeper node first, else the smaller f).
#pragma once
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

namespace ulg {
namespace exact {

struct Node {
    float g, h;
    uint64_t sub;
    uint8_t leaf;
    int32_t pq;
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
    // The reference's std::vector<Node*> keeps popped slots in its capacity,
    // and update() can read one through a stale pqPos.  Here the buffer only
    // grows and `len` is the logical size, so such a read is a read of our own
    // initialised memory (the value the slot last held), never past the end.
    std::vector<HeapEnt> a;
    int64_t len = 0;
    std::vector<Node> *nodes;
    bool hang = false;
    int64_t scans = 0;  // decrease-keys whose recorded position was stale

    inline HeapEnt ent(uint32_t x) const {
        const Node &N = (*nodes)[x];
        return HeapEnt{N.g + N.h, __builtin_popcountll(N.sub) & 0xff, x};
    }
    // CompareNodeStar: true if x has LOWER priority than y
    static inline bool cns(const HeapEnt &A, const HeapEnt &B) {
        const float diff = A.f - B.f;
        const bool tie = std::fabs(diff) < FLT_EPSILON;
        return (tie & ((B.layer - A.layer) > 0)) | (!tie & (diff > 0));
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
    bool empty() const { return len == 0; }
    void push(uint32_t x) {
        const HeapEnt e = ent(x);
        if (len == (int64_t)a.size()) a.push_back(e);
        else a[len] = e;
        ++len;
        push_hole(len - 1, 0, e);
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
            second -= (int64_t)cns(a[second], a[second - 1]);
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
        const int64_t last = len - 1;
        const HeapEnt value = a[last];
        a[last] = a[0];
        adjust(0, last, value);
        --len;
        return ret;
    }
    void update(uint32_t x) {
        const int64_t pos = (*nodes)[x].pq;
        const float fx = (*nodes)[x].g + (*nodes)[x].h;
        // the reference reads whatever node sits at the recorded position
        // (a popped slot included, as the vector's capacity keeps it); a pqPos
        // only ever names a slot the heap has held
        if (pos < 0 || pos >= (int64_t)a.size()) {
            hang = true;  // cannot happen: report instead of reading out of bounds
            return;
        }
        HeapEnt value = a[pos];
        if (value.idx == x && pos < len) {
            value.f = fx;
            a[pos].f = fx;
        } else {
            ++scans;
            for (int64_t i = 0; i < len; ++i)
                if (a[i].idx == x) a[i].f = fx;
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

// ---- dense form ------------------------------------------------------------
// Node homes at recs[slot] (slot = pext(S, scope)), heap entries (f, slot);
// same algorithms as Heap.
struct DenseRec {
    float g, h;
    int32_t pq;     // 0: not generated, -1: closed (the reference's -2), p + 1: heap position p
    uint8_t leaf;
    uint8_t pad[3];
};
static_assert(sizeof(DenseRec) == 16, "DenseRec is one quarter cache line");

// slot (< 2^27) and layer (|S|, the comparator's depth) in one word, so a
// comparison never touches the node record or counts bits
struct DEnt {
    float f;
    uint32_t key;  // slot | layer << 27
    static constexpr uint32_t kSlotMask = (1u << 27) - 1u;
    inline uint32_t slot() const { return key & kSlotMask; }
    inline uint32_t layer() const { return key >> 27; }
};

// Physical layouts of the dense heap's logical positions p (the reference's
// implicit binary heap: children 2p+1, 2p+2).  The algorithms read and write
// logical positions only, so a layout changes where an entry lives, never
// which entry a position holds: the pop order and the pqPos values are the
// reference's in every layout.
//
// FlatLayout: position p at a[p] (the buffer starts 8 B into a line, so two
// siblings share 16 aligned bytes).
struct FlatLayout {
    static constexpr bool kBlocked = false;
    static inline int64_t phys(int64_t p) { return p; }
};
// PairBlockLayout (round 6, review item 7): every node q at an even depth
// owns one 64-B line holding its two children and four grandchildren (slots
// 0-1 and 2-5; 6-7 unused), the lines in BFS order of their owners; the root
// is alone in line 0.  A descent then reads one line per two levels instead
// of one per level, and the line it needs next is known one block ahead:
// the block of the even-depth node it stands on.
struct PairBlockLayout {
    static constexpr bool kBlocked = true;
    // the line of the block owned by even-depth node i (1-based)
    static inline int64_t block_line(uint64_t i) {
        const int dq = 63 - __builtin_clzll(i);  // even
        return 1 + (int64_t)((((uint64_t)1 << dq) - 1) / 3 + (i - ((uint64_t)1 << dq)));
    }
    static inline int64_t phys(int64_t p) {
        const uint64_t i = (uint64_t)p + 1;
        if (i == 1) return 0;
        const int d = 63 - __builtin_clzll(i);
        if (d & 1) return 8 * block_line(i >> 1) + (int64_t)(i & 1);
        return 8 * block_line(i >> 2) + 2 + (int64_t)(i & 3);
    }
    // physical entries for logical positions [0, n)
    static inline int64_t capacity(int64_t n) { return n <= 1 ? 8 : phys(n - 1) + 8; }
};

template <class Lay>
struct DenseHeapT {
    using Layout = Lay;
    DEnt *a = nullptr;  // buffer (grows to at most 2^m + 1 logical entries; never shrinks)
    bool pf5 = false;   // pop: prefetch five levels ahead as well as four (flat layout)
    bool pfdeep = false;  // blocked layout: also the grandchildren's blocks (two more levels)
    int64_t len = 0, hwm = 0;
    DenseRec *recs = nullptr;
    bool hang = false;
    int64_t scans = 0;

    inline DEnt &A(int64_t p) const { return a[Lay::phys(p)]; }
    // CompareNodeStar, evaluated without branches: the heap descent picks a
    // child per level on it, and that choice is a coin flip for a predictor
    static inline bool cns(const DEnt &X, const DEnt &Y) {
        const float diff = X.f - Y.f;
        const bool tie = std::fabs(diff) < FLT_EPSILON;
        const bool deeper = Y.layer() > X.layer();
        const bool worse = diff > 0.0f;
        return (tie & deeper) | (!tie & worse);
    }
    inline DEnt ent(uint32_t x) const {
        return DEnt{recs[x].g + recs[x].h, x | ((uint32_t)__builtin_popcount(x) << 27)};
    }
    inline void setpos(const DEnt &e, int64_t p) { recs[e.slot()].pq = (int32_t)(p + 1); }
    void push_hole(int64_t hole, int64_t top, DEnt value) {
        int64_t parent = (hole - 1) / 2;
        while (hole > top && cns(A(parent), value)) {
            A(hole) = A(parent);
            setpos(A(hole), hole);
            hole = parent;
            parent = (hole - 1) / 2;
        }
        A(hole) = value;
        setpos(value, hole);
    }
    void push(uint32_t x) {
        const DEnt e = ent(x);
        A(len) = e;
        ++len;
        hwm = std::max(hwm, len);
        push_hole(len - 1, 0, e);
    }
    inline void prefetch_descent(int64_t second, int64_t n) const {
        if constexpr (!Lay::kBlocked) {
            // four levels ahead: the 16 great-great-grandchildren of the hole
            // are 128 contiguous bytes
            const int64_t g4 = 16 * second + 15;
            if (g4 + 15 < n) {
                __builtin_prefetch(&a[g4]);
                __builtin_prefetch(&a[g4 + 15]);
            }
            if (pf5) {  // and five levels ahead: 32 entries, 256 B
                const int64_t g5 = 32 * second + 31;
                if (g5 + 31 < n) {
                    __builtin_prefetch(&a[g5]);
                    __builtin_prefetch(&a[g5 + 8]);
                    __builtin_prefetch(&a[g5 + 16]);
                    __builtin_prefetch(&a[g5 + 31]);
                }
            }
        } else {
            // the hole at an even depth owns the next block (its children and
            // grandchildren): the one line the next two levels read
            const uint64_t i = (uint64_t)second + 1;
            if (!((63 - __builtin_clzll(i)) & 1) && 2 * second + 1 < n) {
                __builtin_prefetch(&a[8 * Lay::block_line(i)]);
                if (pfdeep && 8 * second + 7 < n)  // the four grandchildren own the blocks after it
                    for (uint64_t gc = 4 * i; gc < 4 * i + 4; ++gc) __builtin_prefetch(&a[8 * Lay::block_line(gc)]);
            }
        }
    }
    void adjust(int64_t hole, int64_t n, DEnt value) {
        const int64_t top = hole;
        int64_t second = hole;
        uint32_t mv_slot[64];
        int64_t mv_pos[64];
        int nm = 0;
        while (second < (n - 1) / 2) {
            prefetch_descent(second, n);
            second = 2 * (second + 1);
            second -= (int64_t)cns(A(second), A(second - 1));
            A(hole) = A(second);
            __builtin_prefetch(&recs[A(hole).slot()], 1);
            mv_slot[nm] = A(hole).slot();
            mv_pos[nm++] = hole;
            hole = second;
        }
        if ((n & 1) == 0 && second == (n - 2) / 2) {
            second = 2 * (second + 1);
            A(hole) = A(second - 1);
            mv_slot[nm] = A(hole).slot();
            mv_pos[nm++] = hole;
            hole = second - 1;
        }
        for (int i = 0; i < nm; ++i) recs[mv_slot[i]].pq = (int32_t)(mv_pos[i] + 1);
        push_hole(hole, top, value);
    }
    uint32_t pop() {
        const uint32_t ret = A(0).slot();
        const int64_t last = len - 1;
        const DEnt value = A(last);
        A(last) = A(0);
        adjust(0, last, value);
        --len;
        return ret;
    }
    void update(uint32_t x) {
        const int64_t pos = (int64_t)recs[x].pq - 1;
        const float fx = recs[x].g + recs[x].h;
        if (pos < 0 || pos >= hwm) {
            hang = true;  // cannot happen: a pqPos only names a slot the heap has held
            return;
        }
        DEnt value = A(pos);
        if (value.slot() == x && pos < len) {
            value.f = fx;
            A(pos).f = fx;
        } else {
            ++scans;
            for (int64_t i = 0; i < len; ++i)
                if (A(i).slot() == x) A(i).f = fx;
            value.f = recs[value.slot()].g + recs[value.slot()].h;
        }
        const int64_t parent = (pos - 1) / 2;
        if (pos > 0 && cns(A(parent), value)) {
            int64_t par = (pos - 1) / 2, index = pos;
            while (index > 0 && cns(A(par), value)) {
                A(index) = A(par);
                setpos(A(index), index);
                index = par;
                par = (par - 1) / 2;
            }
            if (pos != index) {
                A(index) = value;
                setpos(value, index);
            }
        } else {
            // __down_heap as written (priority_queue-inl.h:176-208)
            int64_t index = pos, left = 2 * index + 1, right = 2 * index + 2, largest = len, guard = 0;
            while (index < len) {
                if ((right >= len) || ((left < len) && cns(A(right), A(left)))) largest = left;
                if (largest < len && cns(value, A(largest))) {
                    if (largest == index || ++guard > 128) { hang = true; break; }
                    A(index) = A(largest);
                    setpos(A(largest), index);
                    index = largest;
                    left = index * 2 + 1;
                    right = index * 2 + 2;
                } else
                    break;
            }
            if (pos != index) A(index) = value;
        }
    }
};
using DenseHeap = DenseHeapT<FlatLayout>;
using BlockedHeap = DenseHeapT<PairBlockLayout>;

}  // namespace exact
}  // namespace ulg
