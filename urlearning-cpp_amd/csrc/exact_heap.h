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

struct DenseHeap {
    DEnt *a = nullptr;  // buffer (grows to at most 2^m + 1 entries; never shrinks)
    bool pf5 = false;   // pop: prefetch five levels ahead as well as four
    int64_t len = 0, hwm = 0;
    DenseRec *recs = nullptr;
    bool hang = false;
    int64_t scans = 0;

    // CompareNodeStar, evaluated without branches: the heap descent picks a
    // child per level on it, and that choice is a coin flip for a predictor
    static inline bool cns(const DEnt &A, const DEnt &B) {
        const float diff = A.f - B.f;
        const bool tie = std::fabs(diff) < FLT_EPSILON;
        const bool deeper = B.layer() > A.layer();
        const bool worse = diff > 0.0f;
        return (tie & deeper) | (!tie & worse);
    }
    inline DEnt ent(uint32_t x) const {
        return DEnt{recs[x].g + recs[x].h, x | ((uint32_t)__builtin_popcount(x) << 27)};
    }
    inline void setpos(const DEnt &e, int64_t p) { recs[e.slot()].pq = (int32_t)(p + 1); }
    void push_hole(int64_t hole, int64_t top, DEnt value) {
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
        const DEnt e = ent(x);
        a[len] = e;
        ++len;
        hwm = std::max(hwm, len);
        push_hole(len - 1, 0, e);
    }
    void adjust(int64_t hole, int64_t n, DEnt value) {
        const int64_t top = hole;
        int64_t second = hole;
        uint32_t mv_slot[64];
        int64_t mv_pos[64];
        int nm = 0;
        while (second < (n - 1) / 2) {
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
            second = 2 * (second + 1);
            second -= (int64_t)cns(a[second], a[second - 1]);
            a[hole] = a[second];
            __builtin_prefetch(&recs[a[hole].slot()], 1);
            mv_slot[nm] = a[hole].slot();
            mv_pos[nm++] = hole;
            hole = second;
        }
        if ((n & 1) == 0 && second == (n - 2) / 2) {
            second = 2 * (second + 1);
            a[hole] = a[second - 1];
            mv_slot[nm] = a[hole].slot();
            mv_pos[nm++] = hole;
            hole = second - 1;
        }
        for (int i = 0; i < nm; ++i) recs[mv_slot[i]].pq = (int32_t)(mv_pos[i] + 1);
        push_hole(hole, top, value);
    }
    uint32_t pop() {
        const uint32_t ret = a[0].slot();
        const int64_t last = len - 1;
        const DEnt value = a[last];
        a[last] = a[0];
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
        DEnt value = a[pos];
        if (value.slot() == x && pos < len) {
            value.f = fx;
            a[pos].f = fx;
        } else {
            ++scans;
            for (int64_t i = 0; i < len; ++i)
                if (a[i].slot() == x) a[i].f = fx;
            value.f = recs[value.slot()].g + recs[value.slot()].h;
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
            // __down_heap as written (priority_queue-inl.h:176-208)
            int64_t index = pos, left = 2 * index + 1, right = 2 * index + 2, largest = len, guard = 0;
            while (index < len) {
                if ((right >= len) || ((left < len) && cns(a[right], a[left]))) largest = left;
                if (largest < len && cns(value, a[largest])) {
                    if (largest == index || ++guard > 128) { hang = true; break; }
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

}  // namespace exact
}  // namespace ulg
