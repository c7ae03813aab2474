// walk_may_hit_check -- runs cbic_dev.h's walk_may_hit<L, PHASE, W> (the
// scorer's walk closure, compiled for the host from the same header) on
// presence patterns read from stdin, and prints, per pattern, the set of
// local subsets it reports as testable: subset t is testable iff the closure
// says "may hit" for hi = {t}.  tests/test_walk_closure.py compares that with
// scripts/walk_closure_check.py's restatement (which is itself checked against
// the literal find_best_subset_score recursion, BIC_OLS.cpp:125-172).
//
// stdin, one pattern per line: L phase p_0 .. p_{W-1}  (W = bits_words(L),
// presence words in hex); stdout: the tested words in hex, one line each.
#include <cstdint>
#include <cstdio>

#include "../csrc/cbic_dev.h"

template <int L, int PH>
static void run(const uint64_t *pw) {
    constexpr int W = bits_words(L);
    constexpr int Q = PH == 0 ? L : L + 1;
    uint64_t pres[W], out[W] = {};
    for (int j = 0; j < W; ++j) pres[j] = pw[j];
    for (uint32_t t = 0; t < (1u << Q); ++t) {
        uint64_t hiw[W] = {};
        hiw[t >> 6] = 1ull << (t & 63);
        if (walk_may_hit<L, PH, W>(pres, hiw)) out[t >> 6] |= 1ull << (t & 63);
    }
    for (int j = 0; j < W; ++j) std::printf(j ? " %llx" : "%llx", (unsigned long long)out[j]);
    std::printf("\n");
}

template <int L>
static void dispatch(int ph, const uint64_t *pw) {
    if (ph == 0) run<L, 0>(pw);
    else run<L, 1>(pw);
}

int main() {
    int L, ph;
    while (std::scanf("%d %d", &L, &ph) == 2) {
        uint64_t pw[2] = {0, 0};
        const int W = bits_words(L);
        for (int j = 0; j < W; ++j) {
            unsigned long long x;
            if (std::scanf("%llx", &x) != 1) return 1;
            pw[j] = x;
        }
        switch (L) {
            case 1: dispatch<1>(ph, pw); break;
            case 2: dispatch<2>(ph, pw); break;
            case 3: dispatch<3>(ph, pw); break;
            case 4: dispatch<4>(ph, pw); break;
            case 5: dispatch<5>(ph, pw); break;
            case 6: dispatch<6>(ph, pw); break;
            default: return 2;
        }
    }
    return 0;
}
