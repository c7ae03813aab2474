// Offline study of the bit-sliced walk launches (round 6, review item 1):
// replays walk_sliced (cbic_dev.h) on the queues a C3 call dumped
// (ULG_WALK_CLOCK + ULG_WALK_QUEUE_DUMP, cbic.hip dump_walk_queue), checks the
// replay's decisions against the ones the GPU wrote, and prints the union
// points of the waves of several schedules -- a wave's time is about its union
// points x ~630 cycles, and a launch lasts as long as its longest wave.
//
//   g++ -O2 -std=c++17 -o scripts/bin/walk_sched_study scripts/walk_sched_study.cpp
//   scripts/bin/walk_sched_study gpurun_out/<tag>/wc/queue_L6_p1.bin 6 1 [K]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

struct Set {
    uint32_t slot;
    uint32_t tsbits;
    uint64_t hi[8], open[8];
    uint32_t decision;  // table bits the GPU left
};

static int L_, PH_, W_;
static const bool clear_early = std::getenv("STUDY_CLEAR_EARLY") != nullptr;

static inline bool tb(const uint64_t *w, uint32_t t) { return (w[t >> 6] >> (t & 63)) & 1ull; }
static inline void cb(uint64_t *w, uint32_t t) { w[t >> 6] &= ~(1ull << (t & 63)); }

// A group of up to 64*8 sets walked as one union tree (walk_sliced), masks as
// bit vectors over the group's members.
struct Group {
    std::vector<Set *> s;
    std::vector<uint64_t> open;  // per set: its own open words (copied, cleared by the walk)
    std::vector<char> alive, dom;
    long pts = 0;
    bool any_act(const std::vector<char> &act) const {
        for (char a : act)
            if (a) return true;
        return false;
    }
    void walk(uint32_t T, uint32_t pv, std::vector<char> act, int M, int lo, int hi) {
        for (int idx = lo; idx < hi; ++idx) {
            for (size_t k = 0; k < s.size(); ++k) act[k] &= alive[k];
            if (!any_act(act)) return;
            ++pts;
            const uint32_t u = (pv >> (4 * idx)) & 15u, T2 = T ^ (1u << u);
            for (size_t k = 0; k < s.size(); ++k)
                if (act[k] && tb(s[k]->hi, T2)) {
                    dom[k] = 1;
                    alive[k] = 0;
                    act[k] = 0;
                }
            if (M > 1) {
                std::vector<char> x(s.size());
                bool anyx = false;
                for (size_t k = 0; k < s.size(); ++k) {
                    x[k] = act[k] && tb(&open[k * 8], T2);
                    anyx |= x[k];
                }
                if (!anyx) continue;
                // STUDY_CLEAR_EARLY: checked.insert(T2) once, before the
                // calls (nothing below T2 reads T2's open bit)
                if (clear_early)
                    for (size_t k = 0; k < s.size(); ++k)
                        if (x[k]) cb(&open[k * 8], T2);
                uint32_t npv = 0;
                int j = 0;
                for (int i = 0; i < M; ++i) {
                    const uint32_t pi = (pv >> (4 * i)) & 15u;
                    if (pi == u) continue;
                    npv |= pi << (4 * j);
                    ++j;
                    walk(T2, npv, x, M - 1, j == 1 ? 0 : j - 1, j == 1 ? (M - 1 < 2 ? M - 1 : 2) : j);
                    bool any2 = false;
                    for (size_t k = 0; k < s.size(); ++k) {
                        if (x[k] && !clear_early) cb(&open[k * 8], T2);
                        x[k] &= alive[k];
                        any2 |= x[k];
                    }
                    if (!any2) break;
                }
            }
        }
    }
    long run() {
        open.assign(s.size() * 8, 0);
        for (size_t k = 0; k < s.size(); ++k)
            for (int w = 0; w < W_; ++w) open[k * 8 + w] = s[k]->open[w];
        alive.assign(s.size(), 1);
        dom.assign(s.size(), 0);
        pts = 0;
        const bool v0 = PH_ == 0;
        const uint32_t P = v0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
        uint32_t pv = 0;
        for (int i = 0; i < L_; ++i) pv |= (uint32_t)(i + (v0 ? 0 : 1)) << (4 * i);
        walk(P, pv, std::vector<char>(s.size(), 1), L_, 0, L_);
        return pts;
    }
};

// The superset walk_may_hit computes (cbic_dev.h): the nodes the walk can test.
static int tested_popcount(const Set &st) {
    const int Q = PH_ == 0 ? L_ : L_ + 1;
    const uint32_t root = PH_ == 0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
    const uint32_t nsub = 1u << Q;
    std::vector<char> present(nsub), tested(nsub), reach(nsub);
    // present = not open-or-absent... the queue keeps hi and open only; open =
    // absent & cover & not checked, so use open as the "absent" proxy here
    for (uint32_t t = 0; t < nsub; ++t) present[t] = !tb(st.open, t);
    auto absent = [&](uint32_t t) { return t != root && !(PH_ == 1 && t == (root | 1u)) && !present[t]; };
    for (int b = (PH_ == 0 ? 0 : 1); b <= (PH_ == 0 ? L_ - 1 : L_); ++b) {
        const uint32_t t = root ^ (1u << b);
        tested[t] = 1;
        reach[t] = absent(t);
    }
    auto closure = [&]() {
        for (uint32_t t = 0; t < nsub; ++t)
            if (reach[t]) {
                tested[t ^ 1u] = 1;
                if (absent(t ^ 1u)) reach[t ^ 1u] = 1;
            }
    };
    closure();
    for (int e = (PH_ == 0 ? L_ - 1 : L_); e >= 1; --e) {
        for (uint32_t t = 0; t < nsub; ++t)
            if (reach[t] && ((t >> e) & 1u)) {
                const uint32_t c = t ^ (1u << e);
                tested[c] = 1;
                if (absent(c)) reach[c] = 1;
            }
        closure();
    }
    int n = 0;
    for (uint32_t t = 0; t < nsub; ++t) n += tested[t] && absent(t);
    return n;
}

// The per-lane form (round 6): one set per lane, the recursion as an explicit
// state machine (RET, CALL, TEST per iteration, the lane's frames in LDS on
// the device).  Returns the iterations the lane needs; dom = hit.
static long lane_walk(const Set &st, bool &dom, long &tests) {
    uint64_t open[8];
    for (int w = 0; w < W_; ++w) open[w] = st.open[w];
    const bool v0 = PH_ == 0;
    struct Fr { uint32_t T, pv, M, idx, hiEnd, u, i, j, npv; };
    Fr fr[8];
    int d = 0;
    Fr c{};
    c.T = v0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
    for (int i = 0; i < L_; ++i) c.pv |= (uint32_t)(i + (v0 ? 0 : 1)) << (4 * i);
    c.M = L_;
    c.idx = 0;
    c.hiEnd = L_;
    enum { TEST, CALL, RET } state = TEST;
    long it = 0;
    dom = false;
    tests = 0;
    while (true) {
        ++it;
        if (state == RET) {
            if (d == 0) break;  // exhausted: stored
            open[c.T >> 6] &= ~(1ull << (c.T & 63));
            c = fr[--d];
            state = CALL;
        }
        if (state == CALL) {
            uint32_t i = c.i;
            while (i < c.M && ((c.pv >> (4 * i)) & 15u) == c.u) ++i;
            if (i == c.M) {
                ++c.idx;
                state = TEST;
            } else {
                c.npv |= ((c.pv >> (4 * i)) & 15u) << (4 * c.j);
                ++c.j;
                c.i = i + 1;
                fr[d++] = c;
                Fr ch{};
                ch.T = c.T ^ (1u << c.u);
                ch.pv = c.npv;
                ch.M = c.M - 1;
                ch.idx = c.j == 1 ? 0 : c.j - 1;
                ch.hiEnd = c.j == 1 ? (ch.M < 2 ? ch.M : 2) : c.j;
                c = ch;
                state = TEST;
            }
        }
        if (state == TEST) {
            if (c.idx >= c.hiEnd) {
                state = RET;
                continue;
            }
            const uint32_t u = (c.pv >> (4 * c.idx)) & 15u, T2 = c.T ^ (1u << u);
            ++tests;
            if (tb(st.hi, T2)) {
                dom = true;
                break;
            }
            if (c.M > 1 && tb(open, T2)) {
                c.u = u;
                c.i = 0;
                c.j = 0;
                c.npv = 0;
                state = CALL;
            } else {
                ++c.idx;
            }
        }
    }
    return it;
}

static long sched_max(std::vector<Set *> order, int per_wave, long *sum = nullptr) {
    long mx = 0, tot = 0;
    for (size_t i = 0; i < order.size(); i += per_wave) {
        Group g;
        for (size_t j = i; j < std::min(order.size(), i + per_wave); ++j) g.s.push_back(order[j]);
        const long p = g.run();
        mx = std::max(mx, p);
        tot += p;
    }
    if (sum) *sum = tot;
    return mx;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s queue.bin L phase [K]\n", argv[0]);
        return 2;
    }
    L_ = std::atoi(argv[2]);
    PH_ = std::atoi(argv[3]);
    const int K = argc > 4 ? std::atoi(argv[4]) : 4;
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    uint64_t hdr[2];
    if (std::fread(hdr, 8, 2, f) != 2) return 1;
    const uint64_t nseg = hdr[0];
    W_ = (int)hdr[1];
    std::vector<std::vector<Set>> segs(nseg);
    for (uint64_t sgi = 0; sgi < nseg; ++sgi) {
        uint64_t n;
        if (std::fread(&n, 8, 1, f) != 1) return 1;
        std::vector<uint64_t> e(n * (1 + 2 * W_));
        std::vector<uint32_t> d(n);
        if (n && (std::fread(e.data(), 8, e.size(), f) != e.size() || std::fread(d.data(), 4, n, f) != n)) return 1;
        for (uint64_t i = 0; i < n; ++i) {
            Set st{};
            const uint64_t *x = &e[i * (1 + 2 * W_)];
            st.slot = (uint32_t)x[0];
            st.tsbits = (uint32_t)(x[0] >> 32);
            for (int w = 0; w < W_; ++w) {
                st.hi[w] = x[1 + w];
                st.open[w] = x[1 + W_ + w];
            }
            st.decision = d[i];
            segs[sgi].push_back(st);
        }
    }
    std::fclose(f);
    std::vector<Set *> all;
    for (auto &s : segs)
        for (auto &x : s) all.push_back(&x);
    // 1. each set alone: its own walk's points; decisions vs the GPU's
    std::vector<long> single(all.size());
    long bad = 0;
    for (size_t i = 0; i < all.size(); ++i) {
        Group g;
        g.s.push_back(all[i]);
        single[i] = g.run();
        const float ts = __builtin_bit_cast(float, all[i]->tsbits);
        const uint32_t want = g.dom[0] ? 0xFFFFFFFFu : __builtin_bit_cast(uint32_t, -ts);
        bad += want != all[i]->decision;
    }
    std::vector<long> srt = single;
    std::sort(srt.begin(), srt.end());
    auto q = [&](double p) { return srt.empty() ? 0 : srt[std::min(srt.size() - 1, (size_t)(p * srt.size()))]; };
    std::printf("L%d p%d: %zu queued sets in %llu segments, decisions differing from the GPU's: %ld\n", L_, PH_,
                all.size(), (unsigned long long)nseg, bad);
    std::printf("single-set walk points: p50 %ld p90 %ld p99 %ld p99.9 %ld max %ld mean %.1f\n", q(0.5), q(0.9),
                q(0.99), q(0.999), srt.empty() ? 0 : srt.back(),
                srt.empty() ? 0.0 : std::accumulate(srt.begin(), srt.end(), 0.0) / srt.size());
    // 2. the shipped grouping: per segment, 64*K consecutive entries per wave
    long mx = 0, tot = 0, waves = 0;
    for (auto &s : segs) {
        std::vector<Set *> o;
        for (auto &x : s) o.push_back(&x);
        long sum;
        mx = std::max(mx, sched_max(o, 64 * K, &sum));
        tot += sum;
        waves += (o.size() + 64 * K - 1) / (64 * K);
    }
    std::printf("shipped (segment order, %d sets/wave): waves %ld, max union points %ld, sum %ld\n", 64 * K, waves,
                mx, tot);
    // 3. predicted length = popcount of the closure's tested absent nodes
    std::vector<int> pred(all.size());
    for (size_t i = 0; i < all.size(); ++i) pred[i] = tested_popcount(*all[i]);
    {
        // correlation, and the longest walks' predicted ranks
        std::vector<size_t> ix(all.size());
        std::iota(ix.begin(), ix.end(), 0);
        std::sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return single[a] > single[b]; });
        std::printf("longest 10 walks: points/pred:");
        for (size_t i = 0; i < std::min<size_t>(10, ix.size()); ++i) std::printf(" %ld/%d", single[ix[i]], pred[ix[i]]);
        std::vector<int> ps = pred;
        std::sort(ps.begin(), ps.end());
        std::printf("\npred quantiles: p50 %d p90 %d p99 %d max %d\n", ps[ps.size() / 2], ps[ps.size() * 9 / 10],
                    ps[ps.size() * 99 / 100], ps.back());
    }
    // 4. schedules by predicted length: the top `iso` predicted walks in waves
    //    of `small` sets, the rest sorted by prediction in waves of 64*K
    for (int small : {1, 4, 16, 64}) {
        for (double frac : {0.001, 0.005, 0.02, 0.1}) {
            std::vector<Set *> o = all;
            std::vector<size_t> ix(all.size());
            std::iota(ix.begin(), ix.end(), 0);
            std::stable_sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return pred[a] > pred[b]; });
            const size_t iso = (size_t)(frac * all.size());
            std::vector<Set *> top, rest;
            for (size_t i = 0; i < ix.size(); ++i) (i < iso ? top : rest).push_back(all[ix[i]]);
            long s1, s2;
            const long m1 = sched_max(top, small, &s1), m2 = sched_max(rest, 64 * K, &s2);
            std::printf("pred-sorted: top %.1f%% (%zu) in waves of %d -> max %ld (%zu waves); rest %d/wave -> max %ld "
                        "(%zu waves)\n",
                        100 * frac, iso, small, m1, (iso + small - 1) / small, 64 * K, m2,
                        (rest.size() + 64 * K - 1) / (64 * K));
        }
    }
    // 6. the per-lane form: decisions, tests == union points of one set,
    //    iterations per lane; a wave of 64 lanes takes its longest lane
    {
        std::vector<long> its(all.size());
        long bad2 = 0, badp = 0;
        for (size_t i = 0; i < all.size(); ++i) {
            bool dom;
            long tests;
            its[i] = lane_walk(*all[i], dom, tests);
            const float ts = __builtin_bit_cast(float, all[i]->tsbits);
            const uint32_t want = dom ? 0xFFFFFFFFu : __builtin_bit_cast(uint32_t, -ts);
            bad2 += want != all[i]->decision;
            badp += tests != single[i];
        }
        std::vector<long> srt2 = its;
        std::sort(srt2.begin(), srt2.end());
        std::printf("per-lane: decisions differing %ld, test counts differing from the union walk's %ld; iterations "
                    "p50 %ld p99 %ld max %ld, sum %ld\n",
                    bad2, badp, srt2[srt2.size() / 2], srt2[srt2.size() * 99 / 100], srt2.back(),
                    std::accumulate(srt2.begin(), srt2.end(), 0L));
        for (int per : {64}) {
            long mx2 = 0, tot2 = 0, nw = 0;
            for (size_t i = 0; i < all.size(); i += per) {
                long m = 0;
                for (size_t j = i; j < std::min(all.size(), i + per); ++j) m = std::max(m, its[j]);
                mx2 = std::max(mx2, m);
                tot2 += m;
                ++nw;
            }
            std::printf("per-lane, queue order, %d sets/wave: waves %ld, max iterations %ld, sum of wave maxima %ld\n",
                        per, nw, mx2, tot2);
            std::vector<size_t> ix(all.size());
            std::iota(ix.begin(), ix.end(), 0);
            std::stable_sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return pred[a] > pred[b]; });
            mx2 = tot2 = 0;
            for (size_t i = 0; i < ix.size(); i += per) {
                long m = 0;
                for (size_t j = i; j < std::min(ix.size(), i + per); ++j) m = std::max(m, its[ix[j]]);
                mx2 = std::max(mx2, m);
                tot2 += m;
            }
            std::printf("per-lane, predicted-length order, %d sets/wave: max iterations %ld, sum of wave maxima %ld\n",
                        per, mx2, tot2);
        }
    }
    // 7. groupings by walk-tree similarity: sets sorted by a key of their
    //    open bits (the nodes the walk may expand), 64*K per wave
    {
        auto popc_lvl = [&](const Set &x, int lvl) {  // open bits of the nodes with popcount == lvl
            uint64_t k = 0;
            const int Q = L_ + 1;
            int nb = 0;
            for (uint32_t t = 0; t < (1u << Q); ++t)
                if (__builtin_popcount(t) == lvl) {
                    if (tb(x.open, t)) k |= 1ull << nb;
                    if (++nb == 64) break;
                }
            return k;
        };
        const int top = PH_ == 0 ? L_ - 1 : L_;
        for (int depth = 1; depth <= 3; ++depth) {
            std::vector<size_t> ix(all.size());
            std::iota(ix.begin(), ix.end(), 0);
            std::vector<std::vector<uint64_t>> key(all.size());
            for (size_t i = 0; i < all.size(); ++i)
                for (int d = 0; d < depth; ++d) key[i].push_back(popc_lvl(*all[i], top - d));
            std::stable_sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return key[a] < key[b]; });
            std::vector<Set *> o;
            for (size_t i : ix) o.push_back(all[i]);
            for (int per : {64, 64 * K}) {
                long sum;
                const long m = sched_max(o, per, &sum);
                std::printf("sorted by open bits of the top %d levels, %d sets/wave: max union %ld, waves %zu, sum %ld\n",
                            depth, per, m, (o.size() + per - 1) / per, sum);
            }
        }
        // the full open words
        std::vector<size_t> ix(all.size());
        std::iota(ix.begin(), ix.end(), 0);
        std::stable_sort(ix.begin(), ix.end(), [&](size_t a, size_t b) {
            for (int w = W_ - 1; w >= 0; --w)
                if (all[a]->open[w] != all[b]->open[w]) return all[a]->open[w] < all[b]->open[w];
            return false;
        });
        std::vector<Set *> o;
        for (size_t i : ix) o.push_back(all[i]);
        for (int per : {64, 64 * K}) {
            long sum;
            const long m = sched_max(o, per, &sum);
            std::printf("sorted by the open words, %d sets/wave: max union %ld, waves %zu, sum %ld\n", per, m,
                        (o.size() + per - 1) / per, sum);
        }
    }
    // 8. sorted by the open words within each segment only (a per-segment
    //    sort in LDS by the walk launch), 64*K or 64 sets per wave
    for (int per : {64, 128, 64 * K}) {
        long mx = 0, tot = 0, nw = 0;
        std::vector<long> wu;
        for (auto &sg : segs) {
            std::vector<Set *> o;
            for (auto &x : sg) o.push_back(&x);
            std::stable_sort(o.begin(), o.end(), [&](Set *a, Set *b) {
                for (int w = W_ - 1; w >= 0; --w)
                    if (a->open[w] != b->open[w]) return a->open[w] < b->open[w];
                return false;
            });
            for (size_t i = 0; i < o.size(); i += per) {
                Group g;
                for (size_t j = i; j < std::min(o.size(), i + per); ++j) g.s.push_back(o[j]);
                const long p = g.run();
                wu.push_back(p);
                mx = std::max(mx, p);
                tot += p;
                ++nw;
            }
        }
        std::sort(wu.begin(), wu.end());
        std::printf("per-segment sort by open words, %d sets/wave: waves %ld, max union %ld, p99 %ld, p90 %ld, sum %ld\n",
                    per, nw, mx, wu[wu.size() * 99 / 100], wu[wu.size() * 9 / 10], tot);
    }
    // 9. a counting sort by B bits of the open words: the bits of the
    //    first-level nodes (P minus one element, the walk's first tests) and
    //    then the next levels, most significant first; queue order within a key
    {
        const int Q = L_ + 1;
        const uint32_t root = PH_ == 0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
        // node order: by popcount descending (closest to the root first), then t
        std::vector<uint32_t> nodes;
        for (int pc = Q; pc >= 1; --pc)
            for (uint32_t t = 0; t < (1u << Q); ++t)
                if (__builtin_popcount(t) == pc && t != root && t != (root | 1u) && (t & ~(root | 1u)) == 0)
                    nodes.push_back(t);
        for (int B : {6, 8, 10, 12, 14, 16, 20}) {
            std::vector<size_t> ix(all.size());
            std::iota(ix.begin(), ix.end(), 0);
            std::vector<uint32_t> key(all.size());
            for (size_t i = 0; i < all.size(); ++i) {
                uint32_t k = 0;
                for (int b2 = 0; b2 < B && b2 < (int)nodes.size(); ++b2) k = (k << 1) | (uint32_t)tb(all[i]->open, nodes[b2]);
                key[i] = k;
            }
            std::stable_sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return key[a] < key[b]; });
            std::vector<Set *> o;
            for (size_t i : ix) o.push_back(all[i]);
            for (int per : {64 * K}) {
                long sum;
                const long m = sched_max(o, per, &sum);
                std::printf("counting sort by %d open bits (levels from the root), %d sets/wave: max union %ld, sum %ld\n",
                            B, per, m, sum);
            }
        }
    }
    // 10. buckets by the first-level open bits (6 at layer 6): the buckets
    //     with at least H open children walked 64 (or 16) per wave, the rest
    //     64*K2 per wave; queue order within a bucket
    {
        const int Q = L_ + 1;
        const uint32_t root = PH_ == 0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
        std::vector<uint32_t> first;
        for (int b2 = (PH_ == 0 ? 0 : 1); b2 <= (PH_ == 0 ? L_ - 1 : L_); ++b2) first.push_back(root ^ (1u << b2));
        (void)Q;
        for (int H : {3, 4, 5, 6}) {
            for (int hp : {16, 64}) {
                for (int K2 : {4, 8}) {
                    std::vector<Set *> heavy, light;
                    std::vector<std::pair<uint32_t, Set *>> lk;
                    for (Set *x : all) {
                        uint32_t k = 0;
                        int nopen = 0;
                        for (uint32_t t : first) {
                            k = (k << 1) | (uint32_t)tb(x->open, t);
                            nopen += tb(x->open, t);
                        }
                        if (nopen >= H) heavy.push_back(x);
                        else lk.push_back({k, x});
                    }
                    std::stable_sort(lk.begin(), lk.end(), [](auto &a, auto &b) { return a.first < b.first; });
                    for (auto &p2 : lk) light.push_back(p2.second);
                    long s1, s2;
                    const long m1 = sched_max(heavy, hp, &s1), m2 = sched_max(light, 64 * K2, &s2);
                    std::printf("buckets: >=%d open children (%zu sets) %d/wave -> max %ld sum %ld (%zu waves); rest "
                                "(%zu) %d/wave, by key -> max %ld sum %ld (%zu waves)\n",
                                H, heavy.size(), hp, m1, s1, (heavy.size() + hp - 1) / hp, light.size(), 64 * K2, m2,
                                s2, (light.size() + 64 * K2 - 1) / (64 * K2));
                }
            }
        }
    }
    // 11. two queues: the heavy sets (>= H open first-level children) per
    //     segment, 64 per wave; the rest per segment in queue order, 64*K2
    {
        const uint32_t root = PH_ == 0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
        std::vector<uint32_t> first;
        for (int b2 = (PH_ == 0 ? 0 : 1); b2 <= (PH_ == 0 ? L_ - 1 : L_); ++b2) first.push_back(root ^ (1u << b2));
        for (int H : {5, 6}) {
            for (int K2 : {4, 8}) {
                long mh = 0, sh = 0, ml = 0, sl = 0, wh = 0, wl = 0;
                for (auto &sg : segs) {
                    std::vector<Set *> heavy, light;
                    for (auto &x : sg) {
                        int nopen = 0;
                        for (uint32_t t : first) nopen += tb(x.open, t);
                        (nopen >= H ? heavy : light).push_back(&x);
                    }
                    long s1, s2;
                    mh = std::max(mh, sched_max(heavy, 64, &s1));
                    ml = std::max(ml, sched_max(light, 64 * K2, &s2));
                    sh += s1;
                    sl += s2;
                    wh += (heavy.size() + 63) / 64;
                    wl += (light.size() + 64 * K2 - 1) / (64 * K2);
                }
                std::printf("two queues per segment: heavy >= %d: max %ld sum %ld (%ld waves); light %d/wave: max %ld "
                            "sum %ld (%ld waves)\n", H, mh, sh, wh, 64 * K2, ml, sl, wl);
            }
        }
    }
    // 12. the all-open key split by a secondary key (64 per wave): (a) the
    //     var-0 toggles of the first-level nodes, (b) 6 of the second-level
    //     nodes, (c) the full open words
    {
        const uint32_t root = PH_ == 0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
        std::vector<uint32_t> first;
        for (int b2 = (PH_ == 0 ? 0 : 1); b2 <= (PH_ == 0 ? L_ - 1 : L_); ++b2) first.push_back(root ^ (1u << b2));
        std::vector<Set *> heavy;
        for (Set *x : all) {
            bool allopen = true;
            for (uint32_t t : first) allopen &= tb(x->open, t);
            if (allopen) heavy.push_back(x);
        }
        auto keyA = [&](const Set *x) {
            uint32_t k = 0;
            for (uint32_t t : first) k = (k << 1) | (uint32_t)tb(x->open, t ^ 1u);
            return k;
        };
        auto keyB = [&](const Set *x) {
            uint32_t k = 0;
            int nb = 0;
            for (size_t i = 0; i < first.size() && nb < 6; ++i)
                for (size_t j = i + 1; j < first.size() && nb < 6; ++j, ++nb)
                    k = (k << 1) | (uint32_t)tb(x->open, first[i] & first[j]);
            return k;
        };
        auto keyAB = [&](const Set *x) { return (keyA(x) << 6) | keyB(x); };
        for (int mode = 0; mode < 4; ++mode) {
            std::vector<Set *> o = heavy;
            if (mode == 1) std::stable_sort(o.begin(), o.end(), [&](Set *a, Set *b) { return keyA(a) < keyA(b); });
            if (mode == 2) std::stable_sort(o.begin(), o.end(), [&](Set *a, Set *b) { return keyB(a) < keyB(b); });
            if (mode == 3) std::stable_sort(o.begin(), o.end(), [&](Set *a, Set *b) { return keyAB(a) < keyAB(b); });
            long sum;
            const long m = sched_max(o, 64, &sum);
            const char *nm[] = {"queue order", "var-0 toggles", "6 second-level", "both (12 bits)"};
            std::printf("all-open key (%zu sets), 64/wave, secondary key %s: max %ld sum %ld\n", heavy.size(), nm[mode],
                        m, sum);
        }
    }
    // 13. the other keys: by the first-level pattern only, or also by six
    //     second-level nodes; 128 / 256 sets per wave
    {
        const uint32_t root = PH_ == 0 ? ((1u << L_) - 1u) : (((1u << L_) - 1u) << 1);
        std::vector<uint32_t> first;
        for (int b2 = (PH_ == 0 ? 0 : 1); b2 <= (PH_ == 0 ? L_ - 1 : L_); ++b2) first.push_back(root ^ (1u << b2));
        auto k1 = [&](const Set *x) {
            uint32_t k = 0;
            for (size_t i = 0; i < first.size(); ++i) k |= (uint32_t)tb(x->open, first[i]) << i;
            return k;
        };
        auto k2 = [&](const Set *x) {
            uint32_t k = 0;
            int nb = 0;
            for (size_t i = 0; i < first.size() && nb < 6; ++i)
                for (size_t j = i + 1; j < first.size() && nb < 6; ++j, ++nb)
                    k = (k << 1) | (uint32_t)tb(x->open, first[i] & first[j]);
            return k;
        };
        const uint32_t full = (1u << first.size()) - 1u;
        std::vector<Set *> light;
        for (Set *x : all)
            if (k1(x) != full) light.push_back(x);
        for (int two = 0; two < 2; ++two) {
            std::vector<Set *> o = light;
            std::stable_sort(o.begin(), o.end(), [&](Set *a, Set *b) {
                const uint32_t ka = (k1(a) << 6) | (two ? k2(a) : 0u), kb = (k1(b) << 6) | (two ? k2(b) : 0u);
                return ka < kb;
            });
            for (int per : {128, 256, 512}) {
                long sum;
                const long m = sched_max(o, per, &sum);
                std::printf("not-all-open keys (%zu sets) by first-level%s, %d/wave: max %ld sum %ld\n", light.size(),
                            two ? " + six second-level bits" : "", per, m, sum);
            }
        }
    }
    // 5. oracle schedule: by true length
    {
        std::vector<size_t> ix(all.size());
        std::iota(ix.begin(), ix.end(), 0);
        std::sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return single[a] > single[b]; });
        for (int per : {1, 8, 64, 64 * K}) {
            std::vector<Set *> o;
            for (size_t i : ix) o.push_back(all[i]);
            long sum;
            const long m = sched_max(o, per, &sum);
            std::printf("true-length sorted, %d sets/wave: max %ld, waves %zu, sum %ld\n", per, m,
                        (o.size() + per - 1) / per, sum);
        }
    }
    return 0;
}
