// cbic_dev.h -- device building blocks of the cBIC scorer's layer kernels
// (cbic.hip).
//
// Reference semantics (ninalu/urlearning-cpp, urlearning/):
//   colex rank == Gosper enumeration index    base/typedefs.h:692-697
//   find_best_subset_score        scoring_function/BIC_OLS.cpp:125-172
//   store / prune rule                        BIC_OLS.cpp:174-276, score_calculator.cpp:111-115
//   two-phase layer order         score_calculator.cpp:78-123
#pragma once
#include <cstdint>
#include <type_traits>

#include "search_internal.h"

namespace {

using namespace ulg;

constexpr int kBlock = 256;

// How a kernel loads slab values written by other workgroups: every writer
// of a slab is an earlier launch on the same stream (a layer is complete
// before the next one starts), so plain loads see its values.
struct LdPlain {
    __device__ static __forceinline__ float ld(const float *p) { return *p; }
};

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float absent_f() { return __uint_as_float(kAbsentBits); }

// ------------------------------------------------------------------------
// Combinatorics on compact candidate indices.  colex rank of a sorted set
// {a_1 < ... < a_L} is sum_j C(a_j, j): Gosper's next-permutation walks
// exactly this order (typedefs.h:692-697), so rank == enumeration index.
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t B(const uint32_t *binom, int a, int k) { return binom[a * kBinomK + k]; }

// Element i (from the top) of the set of colex rank r is the largest c below
// the previous one with C(c, i) <= r.  A scan down the table is a chain of up
// to U dependent LDS reads per set; instead C(x, i) i! = x (x-1) .. (x-i+1)
// <= (x - (i-1)/2)^i (AM-GM) and >= (x - (i-1)/2 - 0.75)^i for i <= 8, so the
// answer lies in [e - 3, e] for e = floor((r i!)^(1/i) + (i-1)/2) + 1, and
// one round of four independent reads (e + 1 as the guard) settles it; the
// scan remains as the fallback should the float estimate ever land low.
// Ranks of the unrolled layers fit 32 bits (C(63, 8) < 2^32, and the table
// clamps C(a, b) to 32 bits anyway), so the arithmetic stays in 32-bit
// registers: the callers are the layer kernels (L <= 8) and the list write.
__device__ __forceinline__ uint64_t unrank_colex(uint64_t r64, int l, int U, const uint32_t *binom) {
    constexpr float kFact[9] = {1.f, 1.f, 2.f, 6.f, 24.f, 120.f, 720.f, 5040.f, 40320.f};
    constexpr float kInv[9] = {1.f, 1.f, 0.5f, 1.f / 3.f, 0.25f, 0.2f, 1.f / 6.f, 1.f / 7.f, 0.125f};
    uint32_t r = (uint32_t)r64;
    uint64_t mask = 0;
    int c = U - 1;
    for (int i = l; i >= 1; --i) {
        int e;
        if (i == 1 || i > 8) {
            e = i == 1 ? (int)(r < (uint32_t)c ? r : (uint32_t)c) : c;
        } else {
            const float g = exp2f(log2f((float)r * kFact[i]) * kInv[i]);  // r = 0: 0
            e = (int)(g + 0.5f * (float)(i - 1)) + 1;
            e = e < c ? e : c;
            e = e > i - 1 ? e : i - 1;  // C(i - 1, i) = 0 <= r
        }
        const bool low = e < c && B(binom, e + 1, i) <= r;  // the estimate fell short
        const uint32_t b0 = B(binom, e, i);
        const uint32_t b1 = e >= 1 ? B(binom, e - 1, i) : 0u;
        const uint32_t b2 = e >= 2 ? B(binom, e - 2, i) : 0u;
        int cc = b0 <= r ? e : (b1 <= r ? e - 1 : (b2 <= r ? e - 2 : -1));
        uint32_t bc = b0 <= r ? b0 : (b1 <= r ? b1 : b2);
        if (low || cc < 0) {
            cc = low ? c : e - 3;
            while (cc >= 0 && B(binom, cc, i) > r) --cc;
            bc = B(binom, cc, i);
        }
        mask |= 1ull << cc;
        r -= bc;
        c = cc - 1;
    }
    return mask;
}

__device__ __forceinline__ uint64_t rank_colex(uint64_t mask, const uint32_t *binom) {
    uint32_t r = 0;
    int j = 0;
    while (mask) {
        const int a = __builtin_ctzll(mask);
        mask &= mask - 1;
        ++j;
        r += B(binom, a, j);
    }
    return r;
}

// Per-lane bitset over the subsets of (P u {var 0}) in local numbering.
template <int W>
struct Bits {
    static constexpr int kWords = W;
    uint64_t w[W];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int j = 0; j < W; ++j) w[j] = 0;
    }
    __device__ __forceinline__ bool test(uint32_t i) const {
        uint64_t x = w[0];
#pragma unroll
        for (int j = 1; j < W; ++j) x = ((int)(i >> 6) == j) ? w[j] : x;
        return (x >> (i & 63)) & 1ull;
    }
    __device__ __forceinline__ void set(uint32_t i) {
        const uint64_t bit = 1ull << (i & 63);
#pragma unroll
        for (int j = 0; j < W; ++j) w[j] |= ((int)(i >> 6) == j) ? bit : 0ull;
    }
    __device__ __forceinline__ void reset(uint32_t i) {
        const uint64_t bit = 1ull << (i & 63);
#pragma unroll
        for (int j = 0; j < W; ++j) w[j] &= ((int)(i >> 6) == j) ? ~bit : ~0ull;
    }
    __device__ __forceinline__ uint64_t word(int j) const { return w[j]; }
};

// The same bitset with its words in LDS, thread-interleaved (word j of this
// thread at base[j * kBlock]).  For W >= 4 the compiler turns the register
// select chains back into indexed accesses and puts the arrays in scratch
// (global memory) -- every walk test then pays a memory round trip; LDS keeps
// the indexing cheap.
template <int W>
struct BitsLds {
    static constexpr int kWords = W;
    uint64_t *base;
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int j = 0; j < W; ++j) base[j * kBlock] = 0;
    }
    __device__ __forceinline__ bool test(uint32_t i) const { return (base[(i >> 6) * kBlock] >> (i & 63)) & 1ull; }
    __device__ __forceinline__ void set(uint32_t i) { base[(i >> 6) * kBlock] |= 1ull << (i & 63); }
    __device__ __forceinline__ void reset(uint32_t i) { base[(i >> 6) * kBlock] &= ~(1ull << (i & 63)); }
    __device__ __forceinline__ uint64_t word(int j) const { return base[j * kBlock]; }
};

// find_best_subset_score (BIC_OLS.cpp:125-172) replayed on local masks.
// pv: M entries of 4 bits (local bit numbers; entries past the filled ones
// are 0 == variable 0, the zero-initialised arma::uvec of SURVEY N3).  Only
// WHICH cached keys are visited matters: the return value is the max over
// their cached values (and 0), so the recursion records them in `visited`.
template <int M, class BS>
__device__ __forceinline__ void best_subset(uint32_t T, uint32_t pv, const BS &present, BS &checked, BS &visited) {
#pragma nounroll
    for (int idx = 0; idx < M; ++idx) {
        const uint32_t u = (pv >> (4 * idx)) & 15u;
        const uint32_t T2 = T ^ (1u << u);
        if (checked.test(T2)) continue;
        if (present.test(T2)) {
            visited.set(T2);
            continue;
        }
        if constexpr (M > 1) {
            uint32_t npv = 0;
            int j = 0;
#pragma nounroll
            for (int i = 0; i < M; ++i) {
                const uint32_t pi = (pv >> (4 * i)) & 15u;
                if (pi == u) continue;
                npv |= pi << (4 * j);
                ++j;
                best_subset<M - 1, BS>(T2, npv, present, checked, visited);
                checked.set(T2);
            }
        }
    }
}

// cover = { T : some key of hi, without var 0, is a subset of T }: drop bit 0
// of every key, then close upwards over bits 1 .. q-1 (in-word shifts for
// bits 1..5, word ORs for the bits that index words).
template <int W>
__device__ __forceinline__ void cover_words(uint64_t *w) {
    constexpr uint64_t kM[6] = {0xAAAAAAAAAAAAAAAAull, 0xCCCCCCCCCCCCCCCCull, 0xF0F0F0F0F0F0F0F0ull,
                                0xFF00FF00FF00FF00ull, 0xFFFF0000FFFF0000ull, 0xFFFFFFFF00000000ull};
#pragma unroll
    for (int j = 0; j < W; ++j) w[j] |= (w[j] & kM[0]) >> 1;
#pragma unroll
    for (int b = 1; b < 6; ++b)
#pragma unroll
        for (int j = 0; j < W; ++j) w[j] |= (w[j] & ~kM[b]) << (1 << b);
#pragma unroll
    for (int c = 1; c < W; c <<= 1)
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j & c) w[j] |= w[j ^ c];
}

// The candidate local subsets of presence_unrolled, in increasing order, as a
// compile-time list: every nonempty t of the Q local bits with at most L
// bits, except P itself, and the L-bit ones only for sets without variable 0
// (PHASE 1) that hold variable 0 (local bit 0).
constexpr int popc_c(uint32_t x) { return x ? (int)(x & 1u) + popc_c(x >> 1) : 0; }
// The keys settle_rules reads (below): P's direct children, and for a set
// without variable 0 its grandchildren, great-grandchildren and their var-0
// toggles; for a set with variable 0, P\{0} and P\{0,c}.
template <int L, int PHASE>
constexpr bool rule_key(uint32_t x) {
    if (PHASE == 1) {
        const uint32_t P1 = ((1u << L) - 1u) << 1;
        const uint32_t r = P1 & ~x;  // removed members
        if ((x & ~1u & ~P1) != 0u) return false;
        const int k = popc_c(r);
        if (x & 1u) return k >= 1 && k <= 2;  // P\{a}+{0}, P\{a,b}+{0}
        return k >= 1 && k <= 3;              // P\{a}, P\{a,b}, P\{a,b,c}
    } else {
        const uint32_t P0 = (1u << L) - 1u;
        const uint32_t r = P0 & ~x;
        if (popc_c(r) == 1) return true;      // the children
        return popc_c(r) == 2 && (r & 1u);    // P\{0,c}
    }
}
// PART 0: every key; 1: the rule keys only; 2: the rest
template <int L, int PHASE, int Q, int PART = 0>
struct PresList {
    uint32_t t[1 << Q];
    int n;
    constexpr PresList() : t{}, n(0) {
        const uint32_t Plocal = (Q == L) ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
        for (uint32_t x = 1; x < (1u << Q); ++x) {
            const int pc = popc_c(x);
            if (pc > L || x == Plocal) continue;
            if (pc == L && (PHASE == 0 || !(x & 1u))) continue;
            if (PART == 1 && !rule_key<L, PHASE>(x)) continue;
            if (PART == 2 && rule_key<L, PHASE>(x)) continue;
            t[n++] = x;
        }
    }
};

// Presence of every key with a fully unrolled subset loop: the rank of each
// subset t of the Q local bits is a compile-time sum of per-(bit, position)
// binomials preloaded into registers.  Q = L when variable 0 is in P (local
// bits = P), Q = L + 1 otherwise (P plus variable 0).  The loads go out in
// batches of NB before any of their values is used: the gather is a chain of
// independent loads, and issued one at a time (what the compiler makes of a
// load-then-test loop) every load pays the full memory latency.
//
// B32: every slot below 2^30, so a key's byte offset fits 32 bits: the rank
// sums stay in 32-bit registers and each load is a global_load with the
// table base in SGPRs and a 32-bit VGPR offset (one address register per
// pending load instead of a 64-bit pair).  !B32 (tables of 2^30 slots or
// more, the one-pass variant 1 only): 64-bit slot arithmetic.
//
// vals (non-null): each gathered key's value at vals[t] (a local array of
// 2^Q floats the caller indexes with constants only, so it stays in registers)
template <int L, int PHASE, int Q, int W, class LD = LdPlain, int NB = 16, bool B32 = true, int PART = 0>
__device__ __forceinline__ void presence_unrolled(Bits<W> &present, Bits<W> &hi, float thr, const uint32_t *binom,
                                                  uint64_t cpack, bool z, const float *table, const uint64_t *toffv,
                                                  float *vals = nullptr) {
    constexpr PresList<L, PHASE, Q, PART> PL{};
    using Slot = std::conditional_t<B32, uint32_t, uint64_t>;
    uint32_t RB[Q][L + 1];
#pragma unroll
    for (int lb = 0; lb < Q; ++lb) {
        const int ci = (int)((cpack >> (6 * lb)) & 63ull);
#pragma unroll
        for (int p = 1; p <= L; ++p) RB[lb][p] = (p <= lb + 1) ? B(binom, ci, p) : 0u;
    }
    Slot off[L + 1];
#pragma unroll
    for (int pc = 1; pc <= L; ++pc) off[pc] = (Slot)toffv[pc];
    uint32_t pw[2 * W], hw[2 * W];  // the bitsets as 32-bit halves: a constant bit touches one
#pragma unroll
    for (int j = 0; j < 2 * W; ++j) pw[j] = hw[j] = 0u;
#pragma clang loop unroll(full)
    for (int b0 = 0; b0 < PL.n; b0 += NB) {
        // opaque per batch: no rank partial sum is shared across batches, so
        // the addresses of a batch are computed just before its loads
#pragma unroll
        for (int lb = 0; lb < Q; ++lb)
#pragma unroll
            for (int p = 1; p <= L; ++p)
                if (p <= lb + 1) asm volatile("" : "+v"(RB[lb][p]));
        float v[NB];
#pragma clang loop unroll(full)
        for (int i = 0; i < NB; ++i) {
            if (b0 + i >= PL.n) break;
            const uint32_t t = PL.t[b0 + i];
            const int pc = popc_c(t);
            Slot rk = off[pc];
            int jj = 0;
#pragma unroll
            for (int b = 0; b < Q; ++b)
                if ((t >> b) & 1u) {
                    ++jj;
                    rk += RB[b][jj];
                }
            // a key with variable 0 exists only when variable 0 is a
            // candidate (z); otherwise the lane loads slot 0 and reads it as
            // absent
            if (t & 1u) rk = z ? rk : (Slot)0;
            if constexpr (B32)
                v[i] = LD::ld(reinterpret_cast<const float *>(reinterpret_cast<const char *>(table) + (rk << 2)));
            else
                v[i] = LD::ld(table + rk);
        }
#pragma clang loop unroll(full)
        for (int i = 0; i < NB; ++i) {
            if (b0 + i >= PL.n) break;
            const uint32_t t = PL.t[b0 + i];
            float x = v[i];
            if (t & 1u) x = z ? x : absent_f();
            if (vals) vals[t] = x;
            const uint32_t bit = 1u << (t & 31u);
            pw[t >> 5] |= (fbits(x) != kAbsentBits) ? bit : 0u;
            hw[t >> 5] |= (x >= thr) ? bit : 0u;  // the absent sentinel is a NaN: never >= thr
        }
        // pinned here: the IR passes would otherwise sink every test below
        // the last batch and hold all the loaded values at once
#pragma unroll
        for (int j = 0; j < 2 * W; ++j) asm volatile("" : "+v"(pw[j]), "+v"(hw[j]));
        // keep the batches apart: hoisting every load of the unrolled loop
        // would hold all 2^Q values in registers at once
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
        present.w[j] |= (uint64_t)pw[2 * j] | ((uint64_t)pw[2 * j + 1] << 32);
        hi.w[j] |= (uint64_t)hw[2 * j] | ((uint64_t)hw[2 * j + 1] << 32);
    }
}

// bitset words per lane over the subsets of L + 1 local bits
__host__ __device__ constexpr int bits_words(int L) { return (L + 1) <= 6 ? 1 : (1 << ((L + 1) - 6)); }

template <class BS>
__device__ __forceinline__ BS make_bits(uint64_t *lds_base) {
    if constexpr (std::is_same<BS, Bits<BS::kWords>>::value) {
        (void)lds_base;
        return BS{};
    } else {
        return BS{lds_base};
    }
}

// A parent set in local numbering: local bit 0 is variable 0 (compact index
// 0 when it is a candidate), local bits 1..L the other members of P in
// increasing order (all L members of P when P contains variable 0).
template <int L>
struct LocalSet {
    uint64_t cpack;   // local bit -> compact index, 6 bits each (bit 0 -> 0)
    uint32_t Plocal;  // P itself
    uint32_t pvtop;   // the top-level parent vector: P's local bits, 4 bits each
    bool v0inP;
};
// PHASE (N4): phase-0 sets hold variable 0 and exist only when it is a
// candidate (z; the host counts no phase-0 sets otherwise), phase-1 sets never
// hold it -- so the root and the top list are constants of the phase and the
// rule tests on them compile to fixed bit positions.
template <int L, int PHASE>
__device__ __forceinline__ LocalSet<L> local_set(uint64_t cm, bool z) {
    LocalSet<L> s;
    s.v0inP = PHASE == 0;
    const uint64_t E = (PHASE == 0 || z) ? (cm & ~1ull) : cm;
    s.cpack = 0;
    uint64_t rem = E;
#pragma unroll
    for (int i = 1; i <= L; ++i) {
        if (rem) {
            const uint64_t b = (uint64_t)__builtin_ctzll(rem);
            rem &= rem - 1;
            s.cpack |= b << (6 * i);
        }
    }
    s.Plocal = s.v0inP ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    s.pvtop = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) s.pvtop |= (uint32_t)(i + (s.v0inP ? 0 : 1)) << (4 * i);
    return s;
}

// Presence of every candidate key below P u {var 0} in the cache as it
// stands now (`present`), and which of them hold a value >= thr (`hi`).
// V == 1 is the form kept for tables of 2^30 slots or more (64-bit slots).
// PART (unrolled layers only): 0 every key, 1 the keys settle_rules reads, 2
// the rest (the loop form gathers every key under PART 0 and 1, none under 2).
template <int L, int PHASE, int V, class BS, class LD = LdPlain, int PART = 0>
__device__ __forceinline__ void gather_keys(BS &present, BS &hi, const LocalSet<L> &ls, float thr,
                                            const uint32_t *binom, bool z, const float *table,
                                            const uint64_t *toffv) {
    constexpr int W = BS::kWords;
    if constexpr (L <= 6 && (V & 1)) {
        presence_unrolled<L, PHASE, (PHASE == 0 ? L : L + 1), W, LD, 8, (V != 1), PART>(present, hi, thr, binom,
                                                                                        ls.cpack, z, table, toffv);
    } else if constexpr (PART == 2) {
        return;
    } else {
        const int q = ls.v0inP ? L : L + 1;
        const uint32_t full = 1u << q;
#pragma nounroll
        for (uint32_t t = 1; t < full; ++t) {
            const int pc = __builtin_popcount(t);
            bool cand = pc <= L && t != ls.Plocal && (z || !(t & 1u));
            if (pc == L) cand = cand && PHASE == 1 && (t & 1u);
            if (!cand) continue;
            uint64_t rk = 0;
            uint32_t rem = t;
            int j = 0;
            while (rem) {
                const int lb = __builtin_ctz(rem);
                rem &= rem - 1;
                ++j;
                rk += B(binom, (int)((ls.cpack >> (6 * lb)) & 63ull), j);
            }
            const float val = LD::ld(table + toffv[pc] + rk);
            if (fbits(val) != kAbsentBits) present.set(t);
            if (val >= thr) hi.set(t);
        }
    }
}

// The two-pass form's decision for a set with ts < 0 from its presence and hi
// bitsets (variant bit 4).  Returns true when P is not stored; `queued` = the
// set needs the walk.
//  * no present key >= -ts: nothing the walk visits can prune P;
//  * a present direct child >= -ts: always visited at the top;
//  * (P without var 0) a present P\{a,b} or P\{a}+{0} >= -ts
//    with P\{a} absent: P\{a} is first reached at the top
//    level (nothing below P\{a'} contains a' != 0 again), so it
//    is expanded with the full list, and its j = L-1 call tests
//    every P\{a,b}, its j = 1 call (L >= 3) the toggle of var 0.
//    Present keys never enter `checked`, so those are visited.
// ANY_KNOWN: the caller knows some key >= -ts is present (the subset maxima
// said so), so the rules may run on the rule keys alone.
template <int L, int PHASE, class BS, bool ANY_KNOWN = false>
__device__ __forceinline__ bool settle_rules(const BS &present, const BS &hi, const LocalSet<L> &ls, bool &queued) {
    constexpr int W = BS::kWords;
    bool any = ANY_KNOWN;
#pragma unroll
    for (int wj = 0; wj < W; ++wj) any |= hi.word(wj) != 0ull;
    bool dom = false;
    queued = false;
    if (!any) return false;
#pragma unroll
    for (int i = 0; i < L; ++i) dom |= hi.test(ls.Plocal ^ (1u << ((ls.pvtop >> (4 * i)) & 15u)));
    if constexpr (PHASE == 1) {
        constexpr uint32_t P1 = ((1u << L) - 1u) << 1;
#pragma unroll
        for (int ea = 1; ea <= L; ++ea) {
            const uint32_t Ta = P1 ^ (1u << ea);
            bool d2 = false;
#pragma unroll
            for (int eb = 1; eb <= L; ++eb)
                if (eb != ea) d2 |= hi.test(Ta ^ (1u << eb));
            if constexpr (L >= 3) d2 |= hi.test(Ta | 1u);
            dom |= d2 && !present.test(Ta);
        }
        // One level further: X = P\{a,b} (a < b), absent, is first
        // tested below P\{a} if that is absent (in its j = b-1
        // call), else below P\{b} if absent (in its j = a call),
        // else never.  Its expansion list holds the entries before
        // the removed one: {1..b-1}\{a} in the first case, {1..a-1}
        // in the second, plus zeros (the var-0 toggle, L >= 4).
        if constexpr (L >= 3) {
#pragma unroll
            for (int ea = 1; ea <= L; ++ea)
#pragma unroll
                for (int eb = ea + 1; eb <= L; ++eb) {
                    const uint32_t X = P1 ^ (1u << ea) ^ (1u << eb);
                    bool h1 = false, h2 = false;
#pragma unroll
                    for (int ec = 1; ec < eb; ++ec) {
                        if (ec == ea) continue;
                        const bool hc = hi.test(X ^ (1u << ec));
                        h1 |= hc;
                        if (ec < ea) h2 |= hc;
                    }
                    if constexpr (L >= 4) {
                        const bool ht = hi.test(X | 1u);
                        h1 |= ht;
                        h2 |= ht;
                    }
                    const bool pa = present.test(P1 ^ (1u << ea));
                    const bool pb = present.test(P1 ^ (1u << eb));
                    const bool hx = pa ? (!pb && h2) : h1;
                    dom |= hx && !present.test(X);
                }
        }
    } else {
        // P\{0} is the very first node tested; if absent it is
        // expanded with every list (1..j) + zeros, so each present
        // P\{0,c} is visited.
        constexpr uint32_t P0 = (1u << L) - 1u;
        bool d2 = false;
#pragma unroll
        for (int ec = 1; ec < L; ++ec) d2 |= hi.test(P0 ^ 1u ^ (1u << ec));
        dom |= d2 && !present.test(P0 ^ 1u);
    }
    queued = !dom;
    return dom;
}

// Subset maxima (variant bit 6).  hsub[slot of X] = the largest stored value
// over the nonempty subsets of X, X included (NaN: none stored).  The walk of
// P only ever visits keys in U(P) = the nonempty subsets of P u {var 0} other
// than P and P u {var 0} (checked starts as {empty}; a layer-L key with var 0
// is in the cache only in phase 1), so
//   max over U(P) = max_a hsub[P\a]                    (P with var 0, or no var 0 candidate)
//                 = max_a max(hsub[P\a], hsub[P\a+{0}]) (P without var 0, phase 1)
// and a set whose U(P) holds no key >= -ts is stored without its 2^(L+1)
// presence gathers.  Children ranks: for P = {a_1 < ... < a_L} (compact),
//   rank(P\a_i)       = sum_{j<i} C(a_j, j)   + sum_{j>i} C(a_j, j-1)
//   rank(P\a_i + {0}) = sum_{j<i} C(a_j, j+1) + sum_{j>i} C(a_j, j)   (a_1 >= 1)
template <int L, bool WITH0>
__device__ __forceinline__ void child_ranks(uint64_t cm, const uint32_t *binom, uint64_t (&rc)[L], uint64_t (&rz)[L]) {
    uint32_t e[L], d[L], f[L];
    uint64_t rem = cm;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const int aj = __builtin_ctzll(rem);
        rem &= rem - 1;
        e[j] = B(binom, aj, j + 1);
        d[j] = B(binom, aj, j);
        f[j] = WITH0 ? B(binom, aj, j + 2) : 0u;
    }
    uint32_t pe = 0, pf = 0;  // ranks of the unrolled layers fit 32 bits
#pragma unroll
    for (int i = 0; i < L; ++i) {
        uint32_t sd = 0, se = 0;
#pragma unroll
        for (int j = i + 1; j < L; ++j) {
            sd += d[j];
            se += e[j];
        }
        rc[i] = pe + sd;
        rz[i] = pf + se;
        pe += e[i];
        pf += f[i];
    }
}

// May find_best_subset_score's walk of P reach a key >= -ts?  A superset of
// every node the walk tests: below the root any first removal (a child call
// keeps the entries after the removed one), from the second removal on only
// entries before the last removed one in the list order (one level down the
// call keeps just the entries before it), and variable 0 toggled at any node
// below the root (padding zeros; in phase 0 variable 0 is also the first list
// entry).  Only absent nodes are expanded; `checked` and the hi-cover prune
// only remove tests.  If no key >= -ts lies in that superset, the walk stores
// P -- the two-pass scorer then stores it without queueing a walk
// (scripts/walk_closure_check.py checks the superset against the recursion).
// Bit t of word t >> 6 is local subset t; root = P (and, phase 1, P + {0})
// are never keys.
// (__host__ too: host/walk_may_hit_check.cpp runs this very function against
// scripts/walk_closure_check.py's restatement, tests/test_walk_closure.py)
template <int L, int PHASE, int W>
__host__ __device__ __forceinline__ bool walk_may_hit(const uint64_t (&pres)[W], const uint64_t (&hiw)[W]) {
    constexpr int Q = PHASE == 0 ? L : L + 1;
    constexpr uint32_t root = PHASE == 0 ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    constexpr uint64_t kM[6] = {0xAAAAAAAAAAAAAAAAull, 0xCCCCCCCCCCCCCCCCull, 0xF0F0F0F0F0F0F0F0ull,
                                0xFF00FF00FF00FF00ull, 0xFFFF0000FFFF0000ull, 0xFFFFFFFF00000000ull};
    auto bitw = [](uint32_t t, int j) constexpr -> uint64_t { return (int)(t >> 6) == j ? 1ull << (t & 63) : 0ull; };
    uint64_t absent[W], tested[W], reach[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        const uint64_t valid = Q >= 6 ? (j < (1 << (Q - 6)) ? ~0ull : 0ull) : (j == 0 ? (1ull << (1 << Q)) - 1ull : 0ull);
        uint64_t first = 0;  // the root's children: every element removed once
#pragma unroll
        for (int b = (PHASE == 0 ? 0 : 1); b <= (PHASE == 0 ? L - 1 : L); ++b) first |= bitw(root ^ (1u << b), j);
        const uint64_t notkey = bitw(root, j) | (PHASE == 1 ? bitw(root | 1u, j) : 0ull);
        absent[j] = ~pres[j] & valid & ~notkey;
        tested[j] = first;
        reach[j] = first & absent[j];
    }
    auto closure = [&]() {  // variable 0 toggled at every reached node
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const uint64_t c = ((reach[j] & 0x5555555555555555ull) << 1) | ((reach[j] & 0xAAAAAAAAAAAAAAAAull) >> 1);
            tested[j] |= c;
            reach[j] |= c & absent[j];
        }
    };
    closure();
#pragma unroll
    for (int e = (PHASE == 0 ? L - 1 : L); e >= 1; --e) {
        uint64_t n[W];
#pragma unroll
        for (int j = 0; j < W; ++j) {
            if (e < 6) n[j] = (reach[j] & kM[e < 6 ? e : 0]) >> (1 << (e < 6 ? e : 0));
            else n[j] = (j + (1 << (e - 6)) < W && ((j >> (e - 6)) & 1) == 0) ? reach[j + (1 << (e - 6))] : 0ull;
        }
#pragma unroll
        for (int j = 0; j < W; ++j) {
            tested[j] |= n[j];
            reach[j] |= n[j] & absent[j];
        }
        closure();
    }
    bool hit = false;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        const uint64_t notkey = bitw(root, j) | (PHASE == 1 ? bitw(root | 1u, j) : 0ull);
        hit |= (tested[j] & ~notkey & hiw[j]) != 0ull;
    }
    return hit;
}

// ---- bit-sliced walk (score_variant bit 5) ----------------------------------
// The walk's tree (T, pv, idx, i) never depends on the data: only which
// subtrees a set enters does.  So one wave walks the union tree ONCE for 64*K
// sets with scalar control flow, and every per-set test becomes a K-bit mask
// operation: lane l holds sets l*K .. l*K+K-1, and for every local subset t
// the K bits "set k has t in hi / open" sit in K-bit fields of register
// vectors indexed by the (uniform) t.  The union of K*64 walks grows slowly
// with the set count (host model over the dumped C3 patterns: 706 points for
// 64 sets, 1076 for 512), so the work per set drops by an order of
// magnitude against one set per lane.  Same decisions: each set still takes
// exactly its own walk's steps, in its order; sets never interact.
template <int L, int K_>
struct Sliced {
    static constexpr int Q = L + 1;                   // local bits (phase 0 uses L)
    static constexpr int K = K_;                      // sets per lane
    static constexpr int E = 32 / K;                  // subsets per register
    static constexpr int NV0 = (1 << Q) / E;
    static constexpr int NV = NV0 < 2 ? 2 : NV0;      // registers per bitset vector
    static constexpr uint32_t KM = (1u << K) - 1u;
    typedef uint32_t Vec __attribute__((ext_vector_type(NV)));
};

template <int L, int K>
__device__ __forceinline__ uint32_t sl_get(const typename Sliced<L, K>::Vec &v, uint32_t t) {
    using S = Sliced<L, K>;
    return (v[t / S::E] >> (S::K * (t % S::E))) & S::KM;
}
template <int L, int K>
__device__ __forceinline__ void sl_clear(typename Sliced<L, K>::Vec &v, uint32_t t, uint32_t m) {
    using S = Sliced<L, K>;
    v[t / S::E] &= ~(m << (S::K * (t % S::E)));
}
__device__ __forceinline__ bool wave_any(uint32_t x) { return __ballot(x != 0u) != 0ull; }

// The walk's open bits in LDS instead of registers: register r of the bit-
// sliced vector is word r * 64 + lane.  A test is one ds_read at a uniform
// offset and a clear one ds_and, where the register form's indexed write
// makes the compiler copy the whole vector at every recursion level (16
// v_mov_b64 per expanded node at layer 6).
// A copy of the hi bits sits HOFF words further (read-only): a node's open
// and hi words then come from one address, two LDS reads in flight together,
// instead of an indexed register read (s_set_gpr_idx) beside the LDS read.
template <int L, int K, int HOFF = Sliced<L, K>::NV * 64>
struct OpenLds {
    uint32_t *base;  // this lane's word 0
};
template <int L, int K, int HOFF>
__device__ __forceinline__ uint32_t sl_get(const OpenLds<L, K, HOFF> &v, uint32_t t) {
    using S = Sliced<L, K>;
    return (v.base[(t / S::E) * 64] >> (S::K * (t % S::E))) & S::KM;
}
template <int L, int K, int HOFF>
__device__ __forceinline__ void sl_clear(OpenLds<L, K, HOFF> &v, uint32_t t, uint32_t m) {
    using S = Sliced<L, K>;
    __hip_atomic_fetch_and(v.base + (t / S::E) * 64, ~(m << (S::K * (t % S::E))), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <class OV>
struct HiOffset {
    static constexpr int value = -1;  // no LDS copy: the registers
};
template <int L, int K, int HOFF>
struct HiOffset<OpenLds<L, K, HOFF>> {
    static constexpr int value = HOFF;
};
// the hi bits of t: from the LDS copy beside an OpenLds, else the registers
template <int L, int K, class OV>
__device__ __forceinline__ uint32_t sl_get_hi(const OV &v, const typename Sliced<L, K>::Vec &hiV, uint32_t t) {
    using S = Sliced<L, K>;
    if constexpr (HiOffset<OV>::value >= 0)
        return (v.base[(t / S::E) * 64 + HiOffset<OV>::value] >> (S::K * (t % S::E))) & S::KM;
    else
        return sl_get<L, K>(hiV, t);
}

// [idx_lo, idx_hi): the positions this call can change anything at.  The
// j-th call fb(T2, npv) of a node's inner loop sees the positions below j-1
// already tested by its earlier calls (closed, or present below -ts) and zeros
// from j on, whose child T2 ^ {0} call 1 tested at its position 1 -- so call 1
// walks positions 0..1 and call j >= 2 position j-1 only (the reference's
// remaining re-tests are no-ops; the same tests in the same order).
#ifdef ULG_GATHER_STATS
// diagnostic build: per (layer, phase) the walk's hits by recursion depth
// (slot L - M), then [15] the sets the walk stores (scripts/gather_stats.py)
__device__ unsigned long long g_wstats[2 * (kMaxL + 1) * 16];
#endif
template <int L, int K, int M, bool DIAG = false, class OV = typename Sliced<L, K>::Vec, int PH = 0>
__device__ __forceinline__ void walk_sliced(uint32_t T, uint32_t pv, uint32_t act, const typename Sliced<L, K>::Vec &hiV,
                                            OV &openV, uint32_t &alive, uint32_t &dom, uint32_t &pts, int idx_lo = 0,
                                            int idx_hi = M) {
#pragma nounroll
    for (int idx = idx_lo; idx < idx_hi; ++idx) {
        act &= alive;
        if (!wave_any(act)) break;
        if constexpr (DIAG) ++pts;
        const uint32_t u = (pv >> (4 * idx)) & 15u;
        const uint32_t T2 = T ^ (1u << u);
        // a hit ends that set's walk (the reference returns up the recursion)
        const uint32_t h = (M > 1 ? sl_get_hi<L, K>(openV, hiV, T2) : sl_get<L, K>(hiV, T2)) & act;
        dom |= h;
#ifdef ULG_GATHER_STATS
        if (h) atomicAdd(&g_wstats[(L * 2 + PH) * 16 + (L - M)], (unsigned long long)__builtin_popcount(h));
#endif
        alive &= ~h;
        act &= ~h;
        if constexpr (M > 1) {
            uint32_t x = sl_get<L, K>(openV, T2) & act;
            // The j-th call gets the first j of the caller's entries other
            // than u, zero-padded (BIC_OLS.cpp:152-160, N3).  A list is an
            // optional leading 0 (variable 0, a member of P in phase 0), then
            // distinct nonzero entries, then zero padding, and every list the
            // walk builds keeps that shape (tests/test_walk_lists.py checks
            // it and this packing over every list of layers <= 8).  So a
            // nonzero u is the one entry at idx, and u == 0 drops the leading
            // zero (if any) and the padding: a few scalar operations per
            // expanded node instead of a compare per entry and call.  (Round
            // 6: the walk launches ~20 % shorter, C3 call 0.72 -> 0.67 ms.)
            if (!wave_any(x)) continue;
            uint32_t rest;
            int cnt;
            if (u != 0u) {
                const uint32_t lo = (1u << (4 * idx)) - 1u;
                rest = (pv & lo) | ((pv >> 4) & ~lo);
                cnt = M - 1;
            } else {
                constexpr uint32_t lm = M >= 8 ? 0xFFFFFFFFu : ((1u << (4 * M)) - 1u);
                const uint32_t nz = (pv | (pv >> 1) | (pv >> 2) | (pv >> 3)) & 0x11111111u & lm;
                cnt = __builtin_popcount(nz);
                rest = (pv & 15u) == 0u ? (pv >> 4) : pv;
            }
            if constexpr (M == 2) {
                // the callees (M = 1) only test: the j-th tests T2 minus
                // entry j-1 for the sets still running.  Inlined as one loop;
                // nothing below reads T2's open bit, so one insert at the end
                // does what the insert after each call did -- when a call
                // ran: a node whose list is empty is never inserted
                // (scripts/walk_mark_order_check.cpp checks this form).
                const uint32_t x0 = x;
#pragma nounroll
                for (int j = 1; j <= cnt; ++j) {
                    x &= alive;
                    if (!wave_any(x)) break;
                    if constexpr (DIAG) ++pts;
                    const uint32_t T3 = T2 ^ (1u << ((rest >> (4 * (j - 1))) & 15u));
                    const uint32_t h3 = sl_get<L, K>(hiV, T3) & x;
#ifdef ULG_GATHER_STATS
                    if (h3) atomicAdd(&g_wstats[(L * 2 + PH) * 16 + (L - 1)], (unsigned long long)__builtin_popcount(h3));
#endif
                    dom |= h3;
                    alive &= ~h3;
                }
                if (cnt > 0) sl_clear<L, K>(openV, T2, x0);
                continue;
            }
#pragma nounroll
            for (int j = 1; j <= cnt; ++j) {
                const uint32_t npv = j >= 8 ? rest : (rest & ((1u << (4 * j)) - 1u));
                // one call site per level: two would inline the level below
                // twice, 2^(L-1) copies of the deepest one (a ~40 KB kernel)
                walk_sliced<L, K, M - 1, DIAG, OV, PH>(T2, npv, x, hiV, openV, alive, dom, pts, j == 1 ? 0 : j - 1,
                                                       j == 1 ? (M - 1 < 2 ? M - 1 : 2) : j);
                // checked.insert(T2) for the sets that ran the call.  Not
                // once before the first call: the recursion can re-enter T2
                // through two variable-0 toggles (zero padding), where the
                // reference expands it again, and marking it early changes
                // decisions (0.2 % of random bitsets,
                // scripts/walk_mark_order_check.cpp).  After call 1 the
                // later inserts are no-ops; skipping them measured no faster.
                sl_clear<L, K>(openV, T2, x);
                x &= alive;
                if (!wave_any(x)) break;
            }
        }
    }
}


// calculateScoreAndBeta's value (BIC_OLS.cpp:277-389) for one parent set of
// L variables gv[] (ascending == parent_vec order) of variable v, from the
// Gram matrix g = Z'Z (n x n, row-major, in LDS): Cholesky of G[P,P],
// y = L^-1 G[P,v], RSS = G[v,v] - |y|^2, score = N ln(RSS / N) + lambda ln(N) L
// (BIC_OLS.cpp:366), returned as float like the reference.  Every layer kernel
// uses this one operation order.
template <int L>
__device__ __forceinline__ float cbic_set_score(const double *g, int n, int v, const int (&gv)[L], double N,
                                                double lambda) {
    double Lm[L][L];
    double y[L];
    int ro[L];  // row offsets gv[i] * n (< 2^24: a full-rate 24-bit multiply)
#pragma unroll
    for (int i = 0; i < L; ++i) ro[i] = __mul24(gv[i], n);
#pragma unroll
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) Lm[i][j] = g[ro[i] + gv[j]];
#pragma unroll
    for (int i = 0; i < L; ++i) y[i] = g[ro[i] + v];
    const double cvv = g[v * n + v];
#pragma unroll
    for (int j = 0; j < L; ++j) {
        double s = Lm[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) s -= Lm[j][k] * Lm[j][k];
        const double d = sqrt(s);
        Lm[j][j] = d;
        const double inv = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < L; ++i) {
            double t = Lm[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) t -= Lm[i][k] * Lm[j][k];
            Lm[i][j] = t * inv;
        }
    }
    double yy = 0.0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        double t = y[i];
#pragma unroll
        for (int k = 0; k < i; ++k) t -= Lm[i][k] * y[k];
        t = t / Lm[i][i];
        y[i] = t;
        yy += t * t;
    }
    const double rss = cvv - yy;
    // BIC_OLS.cpp:366  num_err*log(error_L2) + lambda*log(num_err)*k - 0
    const double the_score = N * log(rss / N) + lambda * log(N) * (double)L - 0.0;
    return (float)the_score;
}

}  // namespace
