// heap_check -- differential check of the two replays of the reference's
// priority queue (csrc/exact_heap.h): Heap (node records in generation order,
// used by the indexed exact search and triplet_astar) and DenseHeap (node
// homes at pext(S, scope), used by the dense exact search), the latter in its
// flat and its pair-block physical layout (BlockedHeap).  All must make
// the same moves on the same push / pop / decrease-key sequence, including
// the float ties the CompareNodeStar epsilon rule (base/node.h:124-135) and
// the left-child-only __down_heap (priority_queue-inl.h:176-208) act on.
// Built with AddressSanitizer + UBSan by `make sanitize` (tests/test_sanitize.py).
//
//   heap_check [seed] [ops] [bits]
#include <cstdio>
#include <cstdlib>
#include <random>
#include <unordered_map>
#include <vector>

#include "../csrc/exact_heap.h"

using namespace ulg::exact;

int main(int argc, char **argv) {
    const unsigned seed = argc > 1 ? (unsigned)std::atoi(argv[1]) : 1u;
    const long ops = argc > 2 ? std::atol(argv[2]) : 200000;
    const int bits = argc > 3 ? std::atoi(argv[3]) : 12;
    const uint32_t nslots = 1u << bits;
    std::mt19937_64 rng(seed);

    long pops = 0, updates = 0, pushes = 0, rounds = 0;
    int64_t scans = 0;
    long op = 0;
    while (op < ops) {
        // one round: fresh heaps over the 2^bits subsets until every node is closed
        std::vector<Node> nodes;
        Heap h;
        h.nodes = &nodes;
        std::vector<DenseRec> recs(nslots, DenseRec{0.0f, 0.0f, 0, 0, {0, 0, 0}});
        std::vector<DEnt> buf(nslots + 2);
        DenseHeap d;
        d.recs = recs.data();
        d.a = buf.data() + 1;
        // the blocked layout on its own records (the same values, its own pqPos)
        std::vector<DenseRec> recs2(nslots, DenseRec{0.0f, 0.0f, 0, 0, {0, 0, 0}});
        std::vector<DEnt> buf2((size_t)PairBlockLayout::capacity((int64_t)nslots + 2));
        BlockedHeap bl;
        bl.recs = recs2.data();
        bl.a = buf2.data();
        bl.pfdeep = (seed & 1) != 0;

        std::unordered_map<uint32_t, uint32_t> idx_of;  // slot -> index into nodes
        std::vector<uint32_t> open_slots;
        std::vector<char> state(nslots, 0);  // 0 new, 1 open, 2 closed
        // f values of two kinds: a coarse grid with exact ties, and a cluster
        // spaced below FLT_EPSILON, where "tied" is not transitive and the
        // heap can hold a near-tie chain that __down_heap then moves along
        const bool cluster = (rounds & 1) != 0;
        auto val = [&](int range) {
            if (cluster) return 0.1f + (float)(rng() % 8) * 5e-8f;
            return (float)(rng() % range) * 0.5f + ((rng() % 8) == 0 ? 1e-8f : 0.0f);
        };
        long closed = 0;
        for (; op < ops && closed < (long)nslots; ++op) {
            const int kind = (int)(rng() % 10);
            if (kind < 5) {  // push a new node
                const uint32_t x = (uint32_t)(rng() % nslots);
                if (state[x] != 0) continue;
                const float g = val(64), hh = cluster ? 0.0f : val(16);
                idx_of[x] = (uint32_t)nodes.size();
                nodes.push_back(Node{g, hh, x, 0, 0});
                h.push(idx_of[x]);
                recs[x].g = g;
                recs[x].h = hh;
                d.push(x);
                recs2[x].g = g;
                recs2[x].h = hh;
                bl.push(x);
                state[x] = 1;
                open_slots.push_back(x);
                ++pushes;
            } else if (kind < 8) {  // pop
                if (h.len == 0) continue;
                const uint32_t a = nodes[h.pop()].sub;
                const uint32_t b = d.pop();
                const uint32_t b2 = bl.pop();
                if (a != b || b != b2) {
                    std::printf("FAIL op %ld: pop %u vs %u vs %u (blocked)\n", op, a, b, b2);
                    return 1;
                }
                nodes[idx_of[a]].pq = -2;
                recs[b].pq = -1;
                recs2[b].pq = -1;
                state[a] = 2;
                ++closed;
                ++pops;
            } else {  // decrease-key of an open node
                if (open_slots.empty()) continue;
                const size_t k = rng() % open_slots.size();
                const uint32_t x = open_slots[k];
                if (state[x] != 1) {
                    open_slots[k] = open_slots.back();
                    open_slots.pop_back();
                    continue;
                }
                const float g = recs[x].g - (cluster ? 5e-8f : 0.5f) * (float)(1 + rng() % 4);
                nodes[idx_of[x]].g = g;
                recs[x].g = g;
                recs2[x].g = g;
                h.update(idx_of[x]);
                d.update(x);
                bl.update(x);
                ++updates;
            }
            if (h.hang != d.hang || d.hang != bl.hang || d.len != bl.len) {
                std::printf("FAIL op %ld: hang flags differ\n", op);
                return 1;
            }
            if (h.hang) break;
            if (h.len != d.len) {
                std::printf("FAIL op %ld: sizes %lld vs %lld\n", op, (long long)h.len, (long long)d.len);
                return 1;
            }
            if (op % 97 == 0)
                for (int64_t i = 0; i < h.len; ++i)
                    if (nodes[h.a[i].idx].sub != d.a[i].slot() || h.a[i].f != d.a[i].f ||
                        bl.A(i).slot() != d.a[i].slot() || bl.A(i).f != d.a[i].f) {
                        std::printf("FAIL op %ld: heap slot %lld differs\n", op, (long long)i);
                        return 1;
                    }
        }
        for (uint32_t x = 0; x < nslots; ++x)
            if (state[x] == 1 && (nodes[idx_of[x]].pq + 1 != recs[x].pq || recs2[x].pq != recs[x].pq)) {
                std::printf("FAIL: pqPos of %u: %d vs %d\n", x, nodes[idx_of[x]].pq, recs[x].pq - 1);
                return 1;
            }
        scans += h.scans;
        ++rounds;
        if (h.hang) break;
    }
    std::printf("heap_check ok: seed %u, %ld rounds, %ld pushes, %ld pops, %ld decrease-keys, %lld stale-position scans\n",
                seed, rounds, pushes, pops, updates, (long long)scans);
    return 0;
}
