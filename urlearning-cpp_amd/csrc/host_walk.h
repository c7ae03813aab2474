// host_walk.h -- walk_wide_lds_kernel's replay of find_best_subset_score
// (BIC_OLS.cpp:125-172; the reduced form of cbic.hip) on a host
// core.  Long walks move here from the GPU (ulg_set_option "wide_host"): a
// walk is one sequential DFS, and one wave issues at most one instruction
// every 4 cycles.  Plain C++ (no HIP), so host tools can time it too.
#pragma once
#include <cstdint>

namespace ulg {

// In-word neighbours of a node at bit b of its word: positions b ^ 2^l,
// l < 6.  pext over mask[b] returns them in ascending position order -- the
// l with bit l of b set in decreasing l, then the others in increasing l --
// and perm[b] puts them back in l order.
struct NbrTables {
    uint64_t mask[64];
    uint8_t perm[64][64];
    NbrTables() {
        for (int b = 0; b < 64; ++b) {
            int order[6], k = 0;
            for (int l = 5; l >= 0; --l)
                if ((b >> l) & 1) order[k++] = l;
            for (int l = 0; l < 6; ++l)
                if (!((b >> l) & 1)) order[k++] = l;
            mask[b] = 0;
            for (int l = 0; l < 6; ++l) mask[b] |= 1ull << (b ^ (1 << l));
            for (int v = 0; v < 64; ++v) {
                uint8_t o = 0;
                for (int j = 0; j < 6; ++j) o |= (uint8_t)(((v >> j) & 1) << order[j]);
                perm[b][v] = o;
            }
        }
    }
};
inline const NbrTables &nbr_tables() {
    static const NbrTables t;
    return t;
}

constexpr int kStragDepth = 24;                // frames of a replay (cbic.hip's LDS replay has the same)
constexpr uint64_t kStragIterCap = 1ull << 32;  // iterations before a replay fails loudly

// walk_wide_lds_kernel's walk on a host core, over the same skip / hi
// bitsets (strag_fill's): the same tests in the same order, with the wave's
// neighbour ballots as loops over the q local bits.  Returns dominated (the
// walk reached a present key >= -ts); err on the kernel's error conditions.
inline bool host_walk(int L, int phase, uint64_t *skip, const uint64_t *hib, bool *err, uint64_t *iters = nullptr,
                      uint64_t *nbr_calls = nullptr) {
    const int q = phase == 0 ? L : L + 1;
    // bit l of sm / hm: skip / hi bit of N ^ {l} (the wave's ballot; bits
    // from q up read as skipped)
    const uint32_t above = q >= 32 ? 0u : ~0u << q;
    uint64_t ncalls = 0;
    // N ^ {l} for l < 6 stays in N's word (bit b ^ 2^l); for l >= 6 it is
    // bit b of the word w ^ 2^(l-6): one word read per neighbour, and six
    // neighbours from one read
    const int ql = q < 6 ? q : 6;
    // (the kernel's hi mask hm is only ever tested at the chosen entry, so
    // the host reads that one bit of hib directly instead)
    const NbrTables &nt = nbr_tables();
    auto nbr = [&](uint32_t Nn, uint32_t &sm_) {
        ++ncalls;
        const uint32_t w = Nn >> 6, b = Nn & 63u;
        const uint64_t ws = skip[w];
        uint32_t s_ = above;
        if (ql == 6) {
            s_ |= nt.perm[b][__builtin_ia32_pext_di(ws, nt.mask[b])];
        } else {
            for (int l = 0; l < ql; ++l) s_ |= (uint32_t)((ws >> (b ^ (1u << l))) & 1ull) << l;
        }
        for (int l = 6; l < q; ++l) s_ |= (uint32_t)((skip[w ^ (1u << (l - 6))] >> b) & 1ull) << l;
        sm_ = s_;
    };
    auto hi_at = [&](uint32_t t) -> bool { return (hib[t >> 6] >> (t & 63u)) & 1ull; };
    struct Frame {
        uint32_t N, rem, B, w, sm;
    } frames[kStragDepth];
    const uint32_t P = phase == 0 ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    uint32_t N = P, rem = P, B = 0, sm;
    nbr(N, sm);
    int x = 31, zr = 0, js = 0, d = 0, mS = L;
    bool pend = false, incall = false, dom = false;
    uint64_t it = 0;
    while (true) {
        if (++it > kStragIterCap) {
            *err = true;
            break;
        }
        int y = 0;
        if (pend) {
            pend = false;
            y = 0;
        } else {
            if (incall) {
                skip[N >> 6] |= 1ull << (N & 63);
                incall = false;
            }
            const uint32_t xb = x < 32 ? 1u << x : 0u;
            const uint32_t cand = rem & ~xb;
            bool found = false;
            if (d == 0) {
                const uint32_t ev = rem & ~sm;
                if (ev) {
                    y = __builtin_ctz(ev);
                    rem &= ~((2u << y) - 1u);
                    found = true;
                }
            } else if (js == 0) {
                if (cand) {
                    y = __builtin_ctz(cand);
                    rem &= ~((2u << y) - 1u);
                    B |= 1u << y;
                    found = true;
                } else if (zr && x != 0) {
                    --zr;
                    y = 0;
                    found = true;
                }
                if (found) {
                    js = 1;
                    incall = true;
                    pend = mS - 1 >= 2;
                }
            } else {
                const uint32_t ev = cand & ~sm;
                if (ev) {
                    y = __builtin_ctz(ev);
                    const uint32_t run = cand & ((2u << y) - 1u);
                    B |= run;
                    js += __builtin_popcount(run);
                    rem &= ~((2u << y) - 1u);
                    incall = true;
                    found = true;
                } else {
                    B |= cand;
                    js += __builtin_popcount(cand);
                    rem = 0;
                    if (zr && x != 0) {
                        if (sm & 1u) {
                            js += zr;
                            zr = 0;
                        } else {
                            --zr;
                            ++js;
                            y = 0;
                            incall = true;
                            found = true;
                        }
                    }
                }
            }
            if (!found) {
                if (d == 0) break;
                const int cx = x;
                const bool cmarked = js > 0;
                --d;
                const Frame &f = frames[d];
                N = f.N;
                rem = f.rem;
                B = f.B;
                sm = f.sm;
                x = (int)(f.w & 31u);
                zr = (int)((f.w >> 5) & 31u);
                js = (int)((f.w >> 10) & 31u);
                pend = (f.w >> 15) & 1u;
                incall = (f.w >> 16) & 1u;
                mS = d == 0 ? L : L - d + 1;
                if (cx != 0) {
                    if (cmarked) sm |= 1u << cx;
                } else {
                    nbr(N, sm);
                }
                continue;
            }
        }
        if ((sm >> y) & 1u) continue;
        if (y < q && hi_at(N ^ (1u << y))) {
            dom = true;
            break;
        }
        const uint32_t Sc = d == 0 ? P : B;
        const int mc = d == 0 ? L : mS - 1;
        if (d + 1 >= kStragDepth || mc < __builtin_popcount(Sc)) {
            *err = true;
            break;
        }
        frames[d] = Frame{N, rem, B,
                          (uint32_t)x | ((uint32_t)zr << 5) | ((uint32_t)js << 10) | ((uint32_t)pend << 15) |
                              ((uint32_t)incall << 16),
                          sm};
        ++d;
        N ^= 1u << y;
        x = y;
        rem = Sc;
        zr = mc - __builtin_popcount(Sc);
        B = 0;
        js = 0;
        pend = false;
        incall = false;
        mS = mc;
        nbr(N, sm);
    }
    if (iters) *iters = it;
    if (nbr_calls) *nbr_calls = ncalls;
    return dom;
}


}  // namespace ulg
