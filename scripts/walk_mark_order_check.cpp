// When may walk_sliced (cbic_dev.h) mark an expanded node `checked`?
// find_best_subset_score (BIC_OLS.cpp:125-172) inserts T2 into `checked`
// after each call of its expansion loop.  This check replays the recursion
// on random present / hi bitsets for layers 2..8, both phases, three ways --
// the reference's order (after every call), after the first call only,
// once before the calls, and walk_sliced's flattened M == 2 level (the
// callees' single tests in one loop, one insert at the end) -- and counts the decisions (a hi key reached) that
// differ from the reference's order.  Round 6: "after the
// first call only" never differs (the later inserts are no-ops); "before the
// calls" differs in ~0.2 % of cases, because the recursion can re-enter T2
// through two variable-0 toggles (zero padding) and the reference expands it
// again there.
//
//   g++ -O2 -std=c++17 -o scripts/bin/walk_mark_order_check scripts/walk_mark_order_check.cpp
//   scripts/bin/walk_mark_order_check 200000
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

static inline bool tb(const uint64_t *w, uint32_t t) { return (w[t >> 6] >> (t & 63)) & 1ull; }
static inline void cb(uint64_t *w, uint32_t t) { w[t >> 6] &= ~(1ull << (t & 63)); }

enum Mode { kEvery, kFirst, kBefore, kFlat2 };

struct Walk {
    uint64_t hi[8], open[8];
    bool alive, dom;
    Mode mode;
    void run(uint32_t T, uint32_t pv, bool act, int M, int lo, int hi_) {
        for (int idx = lo; idx < hi_; ++idx) {
            act &= alive;
            if (!act) return;
            const uint32_t u = (pv >> (4 * idx)) & 15u, T2 = T ^ (1u << u);
            if (tb(hi, T2)) {
                dom = true;
                alive = false;
                act = false;
            }
            if (M > 1) {
                bool x = act && tb(open, T2);
                if (!x) continue;
                if (mode == kBefore) cb(open, T2);
                if (mode == kFlat2 && M == 2) {
                    // walk_sliced's M == 2 form: the callees' one test each,
                    // in one loop, and one insert at the end
                    const bool x0 = x;
                    int j = 0;
                    for (int i = 0; i < M; ++i) {
                        const uint32_t pi = (pv >> (4 * i)) & 15u;
                        if (pi == u) continue;
                        ++j;
                        if (j > 1) x &= alive;
                        if (!x) break;
                        if (tb(hi, T2 ^ (1u << pi))) {
                            dom = true;
                            alive = false;
                        }
                    }
                    if (x0 && j > 0) cb(open, T2);  // only when a call ran
                    continue;
                }
                uint32_t npv = 0;
                int j = 0;
                for (int i = 0; i < M; ++i) {
                    const uint32_t pi = (pv >> (4 * i)) & 15u;
                    if (pi == u) continue;
                    npv |= pi << (4 * j);
                    ++j;
                    run(T2, npv, x, M - 1, j == 1 ? 0 : j - 1, j == 1 ? (M - 1 < 2 ? M - 1 : 2) : j);
                    if (mode == kEvery || mode == kFlat2 || (mode == kFirst && j == 1)) cb(open, T2);
                    x &= alive;
                    if (!x) break;
                }
            }
        }
    }
};

int main(int argc, char **argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 100000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<> U(0.0, 1.0);
    long tot = 0, hits = 0, diff_first = 0, diff_before = 0, diff_flat2 = 0;
    for (int L = 2; L <= 8; ++L)
        for (int ph = 0; ph < 2; ++ph) {
            const int Q = ph == 0 ? L : L + 1;
            const uint32_t P = ph == 0 ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
            uint32_t pv = 0;
            for (int i = 0; i < L; ++i) pv |= (uint32_t)(i + (ph == 0 ? 0 : 1)) << (4 * i);
            for (long c = 0; c < n; ++c) {
                // keys: the subsets of the Q local bits with at most L members,
                // P (and P + {0}) excluded; present with density p, hi among
                // the present ones with density q, open = absent
                const double p = 0.05 + 0.9 * U(rng), q = 0.3 * U(rng);
                Walk w{};
                for (uint32_t t = 0; t < (1u << Q); ++t) {
                    if (t == P || (ph == 1 && t == (P | 1u)) || __builtin_popcount(t) > L) continue;
                    if (U(rng) < p) {
                        if (U(rng) < q) w.hi[t >> 6] |= 1ull << (t & 63);
                    } else {
                        w.open[t >> 6] |= 1ull << (t & 63);
                    }
                }
                Walk a = w, b = w, d = w, f = w;
                a.alive = b.alive = d.alive = f.alive = true;
                a.mode = kEvery;
                b.mode = kFirst;
                d.mode = kBefore;
                f.mode = kFlat2;
                a.run(P, pv, true, L, 0, L);
                b.run(P, pv, true, L, 0, L);
                d.run(P, pv, true, L, 0, L);
                f.run(P, pv, true, L, 0, L);
                ++tot;
                hits += a.dom;
                diff_first += a.dom != b.dom;
                diff_before += a.dom != d.dom;
                diff_flat2 += a.dom != f.dom;
            }
        }
    std::printf("cases %ld, reference-order hits %ld; decisions differing: first call only %ld, before the calls %ld, "
                "flat second-deepest level %ld\n",
                tot, hits, diff_first, diff_before, diff_flat2);
    return diff_first != 0 || diff_flat2 != 0;
}
