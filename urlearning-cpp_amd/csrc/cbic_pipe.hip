// cbic_pipe.hip -- one scoring call (layers 1..kmax <= 6) as ONE persistent
// launch with a device-side work queue.
//
// Reference loop: ScoreCalculator::calculateScores_internal
// (scoring_function/score_calculator.cpp:78-123): per variable, layer after
// layer in Gosper order; BIC_OLS_Function::calculateScore
// (BIC_OLS.cpp:174-276) decides each set against the sets cached so far.
//
// Dependencies.  A variable's layer L reads only its own layers < L and, for
// sets without variable 0, the layer-L sets with variable 0.  So
// every variable is a chain of stages s = 2 (L - 1) + phase (phase 0: the
// sets containing variable 0, phase 1: the rest), and different variables
// never wait for each other.  The layer kernels of cbic.hip run one stage of
// every variable per launch, so each launch waits for the slowest variable's
// stage and ends with a tail of idle CUs; here a stage of a variable is
// released the moment that variable's previous stage is decided, and the
// waves of the one launch move on to whatever stage of whatever variable is
// ready (C3: 25 chains of 12 stages).
//
// Work items (claimed by one wave each):
//   SCORE tile: 64 x R consecutive sets (colex rank) of a stage.  Layers
//     <= Ls: the one-pass form (every set decided in its lane, full
//     find_best_subset_score replay).  Layers > Ls: the two-pass form of
//     score_layer_kernel's variant 113 -- score, settle by the subset maxima,
//     gather the presence bitsets of the rest on dense lanes (the wave's
//     undecided sets pooled in LDS), settle by the two-level rules, and queue
//     the remaining sets for the walk.
//   WALK chunk: 64 x K queued sets of a stage, replayed by one wave with the
//     bit-sliced union-tree walk (walk_sliced).
// A stage is complete when all its tiles are done and every set they queued
// is walked: one 64-bit counter per (variable, stage) holds
//   tiles_done << 32 + (sets walked - sets queued)
// (the difference is signed and stays within +-2^31), so the stage completes
// exactly when the counter equals ntiles << 32, and the wave whose atomic add
// reaches that value publishes the variable's next stage.
//
// Visibility inside the launch (MI355X_MICROARCH.md, inter-workgroup
// visibility; cdna_hip_programming.md Guideline 16).  Decided values and
// subset maxima live in the work layout below: plain stores, and every item
// ends with s_waitcnt vmcnt(0) + an agent release (the XCD's dirty L2 lines
// written back) before the stage-counter add that hands them over; readers use
// plain loads, which is exact because no cache can hold a line of a stage
// before the stage is complete (see "the work layout").  Walk entries, the
// counters and the current-stage words are stored and loaded with sc1 (agent
// atomics), and a wave drains its entry stores before the fill-counter add
// that publishes them.  Read-only inputs (Gram matrix, binomials, offsets,
// stage table) are plain loads.  Every spin is bounded: a wave idle for
// `timeout` clock ticks sets the error word and leaves, and the host reports
// the stall.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "search_internal.h"
#include "cbic_dev.h"
#include "cbic_pipe.h"

namespace {

constexpr uint32_t kDone = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t ld32(const uint32_t *p) {
    return __hip_atomic_load((const gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld64(const uint64_t *p) {
    return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32(uint32_t *p, uint32_t v) {
    __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st64(uint64_t *p, uint64_t v) {
    __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// sets per lane of a walk chunk (walk_sliced_kernel's defaults: 2 up to
// layer 5, 4 at layer 6)
__host__ __device__ constexpr int pipe_k(int L) { return L <= 5 ? 2 : 4; }
// queue entry words: work slot | ts << 32, hch | table slot << 32, then W hi
// and W open words
__host__ __device__ constexpr int entry_words(int L) { return 2 + 2 * bits_words(L); }

struct PipeShared {
    const double *g;
    const uint32_t *binom;
    const uint64_t *toff;
    const int *meta;
};

// ---- stage bookkeeping -------------------------------------------------------
__device__ __forceinline__ void publish_next(const PipeArgs &a, int vi, int s) {
    const uint32_t nx = a.stages[vi * a.NS + s].next;
    st32(a.stage_of + vi, nx);
    if (nx == kDone) __hip_atomic_fetch_add((gu32 *)a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// this wave's stores are drained; add `delta` to the stage counter and, if
// that completes the stage, release the variable's next stage.  Returns
// (wave-uniform) the stage this wave released, or -1.
__device__ __forceinline__ int stage_add(const PipeArgs &a, int vi, int s, uint64_t delta, int lane) {
    drain();
    // the slab values are plain stores: write this XCD's dirty L2 lines back
    // before the counter hands them over (Guideline 16 R1 producer; the asm
    // wait after the fence, Pitfall 12)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    drain();
    int released = -1;
    if (lane == 0) {
        PipeCtr *ct = a.ctr + vi * a.NS + s;
        const uint64_t old = __hip_atomic_fetch_add((gu64 *)&ct->units, delta, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old + delta == ((uint64_t)a.stages[vi * a.NS + s].ntiles << 32)) {
            publish_next(a, vi, s);
            const uint32_t nx = a.stages[vi * a.NS + s].next;
            released = nx == kDone ? -1 : (int)nx;
        }
    }
    return __builtin_amdgcn_readfirstlane(released);
}

// ---- the work layout ------------------------------------------------------------
// Inside the launch the decided values live in a layout of their own: every
// (variable, layer, phase) stage has its own slab, starting on a 128-byte
// line, indexed by the set's rank in its phase's enumeration (sets with
// variable 0: colex rank of the other members among the candidates after
// variable 0; the rest: colex rank among those candidates, or among all of
// them when variable 0 is not one).  A cache line then holds values of one
// stage only, and nothing reads a stage's lines before the stage is
// complete -- so no L1 or L2 can hold a stale copy of a line, plain loads are
// exact, and the lines a stage writes stay in its XCD's L2 for the stages
// above (the layer kernels' slabs interleave both phases of a layer).  The
// values also go to the colex-ordered table the compaction reads after the
// launch.
struct Slabs {
    uint32_t o0[kPipeMaxL + 1], o1[kPipeMaxL + 1];  // per layer: phase 0 / phase 1 slab offsets
};
__device__ __forceinline__ void load_slabs(const PipeArgs &a, int vi, int L, Slabs &sl) {
#pragma unroll
    for (int p = 1; p <= kPipeMaxL; ++p) {
        if (p > L) break;
        sl.o0[p] = a.stages[vi * a.NS + 2 * (p - 1)].slab;
        sl.o1[p] = a.stages[vi * a.NS + 2 * (p - 1) + 1].slab;
    }
}
__device__ __forceinline__ float ldw(const float *p) { return *p; }

// address in the work layout of the local subset t of a set whose local bit
// lb is compact index (cpack >> 6 lb) & 63 (local bit 0: variable 0)
__device__ __forceinline__ uint32_t work_addr(uint32_t t, uint64_t cpack, uint32_t zz, const uint32_t *binom,
                                              const Slabs &sl) {
    uint32_t rk = 0;
    int k = 0;
    for (uint32_t rem = t & ~1u; rem; rem &= rem - 1) {
        const int lb = __builtin_ctz(rem);
        ++k;
        rk += B(binom, (int)((cpack >> (6 * lb)) & 63ull) - (int)zz, k);
    }
    const int pc = __builtin_popcount(t);
    // a select chain, not an indexed load: a runtime index into the
    // register array would put it in scratch
    uint32_t o = 0;
#pragma unroll
    for (int p = 1; p <= kPipeMaxL; ++p)
        if (p == pc) o = (t & 1u) ? sl.o0[p] : sl.o1[p];
    return o + rk;
}

// presence_unrolled (cbic_dev.h) over the work layout: the same subsets and
// batches; a subset's rank counts its members other than variable 0, their
// compact indices shifted down by one when variable 0 is a candidate
template <int L, int PHASE, int Q, int W, int NB = 16>
__device__ __forceinline__ void presence_work(Bits<W> &present, Bits<W> &hi, float thr, const uint32_t *binom,
                                              uint64_t cpack, bool z, const float *work, const Slabs &sl) {
    constexpr PresList<L, PHASE, Q> PL{};
    const uint32_t zz = z ? 1u : 0u;
    uint32_t RB[Q][L + 1];
#pragma unroll
    for (int lb = 1; lb < Q; ++lb) {
        const int ci = (int)((cpack >> (6 * lb)) & 63ull) - (int)zz;
#pragma unroll
        for (int p = 1; p <= L; ++p) RB[lb][p] = (p <= lb) ? B(binom, ci < 0 ? 0 : ci, p) : 0u;
    }
#pragma clang loop unroll(full)
    for (int b0 = 0; b0 < PL.n; b0 += NB) {
#pragma unroll
        for (int lb = 1; lb < Q; ++lb)
#pragma unroll
            for (int p = 1; p <= L; ++p)
                if (p <= lb) asm volatile("" : "+v"(RB[lb][p]));
        float v[NB];
#pragma clang loop unroll(full)
        for (int i = 0; i < NB; ++i) {
            if (b0 + i >= PL.n) break;
            const uint32_t t = PL.t[b0 + i];
            const int pc = popc_c(t);
            uint32_t rk = 0;
            int jj = 0;
#pragma unroll
            for (int b = 1; b < Q; ++b)
                if ((t >> b) & 1u) {
                    ++jj;
                    rk += RB[b][jj];
                }
            const bool ok = !(t & 1u) || z;
            v[i] = ldw(work + (ok ? ((t & 1u) ? sl.o0[pc] : sl.o1[pc]) + rk : 0u));
        }
#pragma clang loop unroll(full)
        for (int i = 0; i < NB; ++i) {
            if (b0 + i >= PL.n) break;
            const uint32_t t = PL.t[b0 + i];
            const bool ok = !(t & 1u) || z;
            if (ok && fbits(v[i]) != kAbsentBits) present.set(t);
            if (ok && v[i] >= thr) hi.set(t);  // the absent sentinel is a NaN: never >= thr
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Work addresses of P's direct subsets (layer L - 1) and, for a set without
// variable 0 when variable 0 is a candidate, of the layer-L keys P\a + {0}
// (SURVEY N4), for P = compact mask cm.
template <int L, int PH>
__device__ __forceinline__ void work_children(uint64_t cm, bool z, const uint32_t *binom, const Slabs &sl,
                                              uint32_t (&ca)[L], uint32_t (&za)[L]) {
    const int zz = z ? 1 : 0;
    if constexpr (PH == 1) {
        uint32_t d0[L], dm1[L];
        uint64_t rem = cm;
#pragma unroll
        for (int j = 0; j < L; ++j) {
            const int e = __builtin_ctzll(rem) - zz;
            rem &= rem - 1;
            d0[j] = B(binom, e, j + 1);
            dm1[j] = B(binom, e, j);
        }
        uint32_t pre = 0;
#pragma unroll
        for (int i = 0; i < L; ++i) {
            uint32_t suf = 0;
#pragma unroll
            for (int j = i + 1; j < L; ++j) suf += dm1[j];
            const uint32_t rk = pre + suf;
            ca[i] = (L > 1 ? sl.o1[L - 1 > 0 ? L - 1 : 1] : 0u) + rk;
            za[i] = sl.o0[L] + rk;
            pre += d0[i];
        }
    } else {
        // P = {var0} u {f_1 < ... < f_{L-1}} (f = compact index - 1)
        uint32_t d0[L], dm1[L];
        uint64_t rem = cm & ~1ull;
#pragma unroll
        for (int k = 0; k < L - 1; ++k) {
            const int f = __builtin_ctzll(rem) - 1;
            rem &= rem - 1;
            d0[k] = B(binom, f, k + 1);
            dm1[k] = B(binom, f, k);
        }
        if constexpr (L > 1) {
            uint32_t all = 0;
#pragma unroll
            for (int k = 0; k < L - 1; ++k) all += d0[k];
            ca[0] = sl.o1[L - 1] + all;  // P \ {var0}
            uint32_t pre = 0;
#pragma unroll
            for (int i = 0; i < L - 1; ++i) {
                uint32_t suf = 0;
#pragma unroll
                for (int k = i + 1; k < L - 1; ++k) suf += dm1[k];
                ca[i + 1] = sl.o0[L - 1] + pre + suf;  // P \ {f_i}: still holds var0
                pre += d0[i];
            }
        } else {
            ca[0] = 0;
        }
#pragma unroll
        for (int i = 0; i < L; ++i) za[i] = 0;
    }
}

// ---- one-pass tile (layers <= Ls): every set decided in its lane -----------
template <int L, int PH>
__device__ __forceinline__ int tile_onepass(const PipeArgs &a, const PipeShared &sh, int vi, int s, uint32_t tile, int lane) {
    const PipeStage &st = a.stages[vi * a.NS + s];
    const int v = sh.meta[vi * 4 + 0], m = sh.meta[vi * 4 + 1];
    const bool z = sh.meta[vi * 4 + 2] != 0;
    const uint64_t vbase = (uint64_t)vi * a.S;
    const uint8_t *cl = a.cand + vi * 64;
    constexpr int W = bits_words(L);
    Slabs sl;
    load_slabs(a, vi, L, sl);
    const uint32_t zz = z ? 1u : 0u;
    for (int r = 0; r < a.Rsmall; ++r) {
        const uint32_t idx = (tile * (uint32_t)a.Rsmall + (uint32_t)r) * 64u + (uint32_t)lane;
        if (!wave_any(idx < st.nsets)) break;
        if (idx >= st.nsets) continue;
        uint64_t cm;
        if (PH == 0) cm = (unrank_colex(idx, L - 1, m - 1, sh.binom) << 1) | 1ull;
        else if (z) cm = unrank_colex(idx, L, m - 1, sh.binom) << 1;
        else cm = unrank_colex(idx, L, m, sh.binom);
        const uint64_t rankP = rank_colex(cm, sh.binom);
        int gv[L];
        {
            uint64_t rem = cm;
#pragma unroll
            for (int i = 0; i < L; ++i) {
                const int b = __builtin_ctzll(rem);
                rem &= rem - 1;
                gv[i] = cl[b];
            }
        }
        const float ts = cbic_set_score<L>(sh.g, a.n, v, gv, a.N, a.lambda);
        float out;
        if (ts >= 0.0f) {
            const float sneg = -ts;
            out = (sneg < 0.0f) ? sneg : absent_f();
        } else {
            const LocalSet<L> ls = local_set<L>(cm, z);
            Bits<W> present, hi, checked, visited;
            present.clear();
            hi.clear();
            presence_work<L, PH, (PH == 0 ? L : L + 1), W>(present, hi, -ts, sh.binom, ls.cpack, z, a.ptab, sl);
            checked.clear();
            visited.clear();
            checked.set(0u);  // checked.insert(empty_set)
            best_subset<L, Bits<W>>(ls.Plocal, ls.pvtop, present, checked, visited);
            float best = 0.0f;
#pragma unroll
            for (int wj = 0; wj < W; ++wj) {
                uint64_t x = visited.word(wj);
                while (x) {
                    const uint32_t t = (uint32_t)(wj * 64 + __builtin_ctzll(x));
                    x &= x - 1;
                    const float val = ldw(a.ptab + work_addr(t, ls.cpack, zz, sh.binom, sl));
                    if (val > best) best = val;
                }
            }
            // BIC_OLS.cpp:234: best_subset_score + bic_threshold >= -the_score
            out = ((double)best + 0.0 >= (double)(-ts)) ? absent_f() : -ts;
        }
        const uint32_t wslot = (PH == 0 ? sl.o0[L] : sl.o1[L]) + idx;
        a.table[sh.toff[vbase + L] + rankP] = out;  // for the compaction after the launch
        a.ptab[wslot] = out;
        // subset maxima for the layers above (score_layer_kernel's one-pass form)
        uint32_t ca[L], za[L];
        work_children<L, PH>(cm, z, sh.binom, sl, ca, za);
        float hch = absent_f();
        if constexpr (L > 1) {
#pragma unroll
            for (int i = 0; i < L; ++i) hch = fmaxf(hch, ldw(a.phsub + ca[i]));
        }
        a.phsub[wslot] = fmaxf(out, hch);
    }
    return stage_add(a, vi, s, 1ull << 32, lane);
}

// ---- two-pass tile (layers > Ls) --------------------------------------------
// per-wave LDS pool of undecided sets: compact mask, slot, ts, children maximum
constexpr int kPool = kPipePool;
struct WavePool {
    uint64_t cm[kPool];
    uint32_t slot[kPool];  // work-layout slot
    float ts[kPool];
    float hch[kPool];
    uint32_t sslot[kPool];  // colex-table slot (the compaction's)
};
static_assert(sizeof(WavePool) == kPipePoolBytes, "pipe_lds sizes the pools");

template <int L, int PH>
__device__ __forceinline__ void pool_drain(const PipeArgs &a, const PipeShared &sh, int vi, int s, const WavePool &P, int off,
                           int take, int lane, uint32_t &queued, bool hsub_on, const Slabs &sl) {
    constexpr int W = bits_words(L);
    constexpr int EW = entry_words(L);
    constexpr uint32_t CH = 64u * pipe_k(L);
    const bool z = sh.meta[vi * 4 + 2] != 0;
    const bool act = lane < take;
    bool q = false, dom = false;
    Bits<W> present, hib;
    uint64_t cm = 0;
    uint32_t slot = 0, sslot = 0;
    float ts = 0.0f, hch = 0.0f;
    if (act) {
        cm = P.cm[off + lane];
        slot = P.slot[off + lane];
        sslot = P.sslot[off + lane];
        ts = P.ts[off + lane];
        hch = P.hch[off + lane];
        const LocalSet<L> ls = local_set<L>(cm, z);
        present.clear();
        hib.clear();
        presence_work<L, PH, (PH == 0 ? L : L + 1), W>(present, hib, -ts, sh.binom, ls.cpack, z, a.ptab, sl);
        dom = settle_rules<L, PH>(present, hib, ls, q);
    }
    // queue the sets that still need the walk (one reservation per wave)
    const uint64_t qm = __ballot(act && q);
    const uint32_t nq = (uint32_t)__popcll(qm);
    uint32_t base = 0;
    if (nq) {
        PipeCtr *ct = a.ctr + vi * a.NS + s;
        if (lane == 0) base = __hip_atomic_fetch_add((gu32 *)&ct->qlen, nq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        base = __shfl(base, 0);
    }
    if (act && q) {
        const uint32_t pos = base + (uint32_t)__popcll(qm & ((1ull << lane) - 1ull));
        uint64_t ow[W];
#pragma unroll
        for (int wj = 0; wj < W; ++wj) ow[wj] = hib.word(wj);
        cover_words<W>(ow);
#pragma unroll
        for (int wj = 0; wj < W; ++wj) {
            const uint64_t ce = ow[wj] & 0x5555555555555555ull;
            ow[wj] = (ce | (ce << 1)) & ~present.word(wj) & (wj == 0 ? ~1ull : ~0ull);
        }
        uint64_t *e = a.queue + a.stages[vi * a.NS + s].qoff + (uint64_t)pos * EW;
        st64(e, (uint64_t)slot | ((uint64_t)__float_as_uint(ts) << 32));
        st64(e + 1, (uint64_t)__float_as_uint(hch) | ((uint64_t)sslot << 32));
#pragma unroll
        for (int wj = 0; wj < W; ++wj) st64(e + 2 + wj, hib.word(wj));
#pragma unroll
        for (int wj = 0; wj < W; ++wj) st64(e + 2 + W + wj, ow[wj]);
    } else if (act) {
        const float o = dom ? absent_f() : -ts;
        a.table[sslot] = o;
        a.ptab[slot] = o;
        if (hsub_on) a.phsub[slot] = fmaxf(o, hch);
    }
    if (nq) {
        // the entries are written: count them into their walk chunks
        drain();
        if (lane == 0) {
            const uint32_t *f0 = nullptr;
            (void)f0;
            uint32_t lo = base, hi = base + nq;
            while (lo < hi) {
                const uint32_t c = lo / CH;
                const uint32_t end = (c + 1) * CH < hi ? (c + 1) * CH : hi;
                __hip_atomic_fetch_add((gu32 *)(a.fill + a.stages[vi * a.NS + s].foff + c), end - lo, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                lo = end;
            }
        }
    }
    queued += nq;
}

template <int L, int PH>
__device__ __forceinline__ int tile_twopass(const PipeArgs &a, const PipeShared &sh, int vi, int s, uint32_t tile, int lane,
                             WavePool &P) {
    const PipeStage &st = a.stages[vi * a.NS + s];
    const int v = sh.meta[vi * 4 + 0], m = sh.meta[vi * 4 + 1];
    const bool z = sh.meta[vi * 4 + 2] != 0;
    const uint64_t vbase = (uint64_t)vi * a.S;
    const uint8_t *cl = a.cand + vi * 64;
    // the subset maxima of the top layer's phase 1 are never read
    const bool hsub_on = !(L == a.kmax && PH == 1);
    Slabs sl;
    load_slabs(a, vi, L, sl);
    int cnt = 0;
    uint32_t queued = 0;
    const uint64_t tq0 = a.stats ? wall_clock64() : 0;
    for (int r = 0; r < a.R; ++r) {
        const uint32_t idx = (tile * (uint32_t)a.R + (uint32_t)r) * 64u + (uint32_t)lane;
        const bool valid = idx < st.nsets;
        if (!wave_any(valid)) break;
        bool need = false;
        uint64_t cm = 0;
        uint32_t slot = 0, sslot = 0;
        float ts = 0.0f, hch = absent_f();
        if (valid) {
            if (PH == 0) cm = (unrank_colex(idx, L - 1, m - 1, sh.binom) << 1) | 1ull;
            else if (z) cm = unrank_colex(idx, L, m - 1, sh.binom) << 1;
            else cm = unrank_colex(idx, L, m, sh.binom);
            const uint64_t rankP = rank_colex(cm, sh.binom);
            int gv[L];
            {
                uint64_t rem = cm;
#pragma unroll
                for (int i = 0; i < L; ++i) {
                    const int b = __builtin_ctzll(rem);
                    rem &= rem - 1;
                    gv[i] = cl[b];
                }
            }
            ts = cbic_set_score<L>(sh.g, a.n, v, gv, a.N, a.lambda);
            slot = (PH == 0 ? sl.o0[L] : sl.o1[L]) + idx;
            sslot = (uint32_t)(sh.toff[vbase + L] + rankP);
            // 1. settle by the subset maxima (score_layer_kernel, variant 113)
            uint32_t ca[L], za[L];
            work_children<L, PH>(cm, z, sh.binom, sl, ca, za);
            if constexpr (L > 1) {
#pragma unroll
                for (int i = 0; i < L; ++i) hch = fmaxf(hch, ldw(a.phsub + ca[i]));
            }
            float out;
            if (ts >= 0.0f) {
                const float sneg = -ts;
                out = (sneg < 0.0f) ? sneg : absent_f();
            } else {
                const float thr = -ts;
                float hu = hch;
                if constexpr (PH == 1) {
                    if (z) {
#pragma unroll
                        for (int i = 0; i < L; ++i) hu = fmaxf(hu, ldw(a.phsub + za[i]));
                    }
                }
                out = -ts;
                if (hu >= thr) {
                    bool dh = false;
                    if constexpr (L > 1) {
#pragma unroll
                        for (int i = 0; i < L; ++i) dh |= ldw(a.ptab + ca[i]) >= thr;
                    }
                    out = absent_f();
                    need = !dh;
                }
            }
            if (!need) {
                a.table[sslot] = out;
                a.ptab[slot] = out;
                if (hsub_on) a.phsub[slot] = fmaxf(out, hch);
            }
        }
        // 2. pool the undecided sets; gather on dense lanes
        const uint64_t nm = __ballot(valid && need);
        if (valid && need) {
            const int pos = cnt + __popcll(nm & ((1ull << lane) - 1ull));
            P.cm[pos] = cm;
            P.slot[pos] = slot;
            P.sslot[pos] = sslot;
            P.ts[pos] = ts;
            P.hch[pos] = hch;
        }
        cnt += __popcll(nm);
    }
    __builtin_amdgcn_wave_barrier();
    const uint64_t tq1 = a.stats ? wall_clock64() : 0;
    // 3. the pooled sets on dense lanes, 64 at a time
    for (int off = 0; off < cnt; off += 64)
        pool_drain<L, PH>(a, sh, vi, s, P, off, cnt - off < 64 ? cnt - off : 64, lane, queued, hsub_on, sl);
    if (a.stats) {
        const uint64_t tq2 = wall_clock64();
        drain();
        const uint64_t tq3 = wall_clock64();
        if (lane == 0) {
            __hip_atomic_fetch_add((gu64 *)(a.stats + 10), tq1 - tq0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add((gu64 *)(a.stats + 11), tq2 - tq1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add((gu64 *)(a.stats + 12), tq3 - tq2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add((gu64 *)(a.stats + 13), (uint64_t)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    return stage_add(a, vi, s, (1ull << 32) - (uint64_t)queued, lane);
}

// ---- walk chunk ----------------------------------------------------------------
template <int L, int PH>
__device__ __forceinline__ int walk_chunk(const PipeArgs &a, int vi, int s, uint32_t c, int lane) {
    constexpr int K = pipe_k(L);
    using SL = Sliced<L, K>;
    constexpr int W = bits_words(L);
    constexpr int EW = entry_words(L);
    constexpr uint32_t CH = 64u * K;
    PipeCtr *ct = a.ctr + vi * a.NS + s;
    const uint32_t ql = ld32(&ct->qlen);
    const uint32_t first = c * CH;
    const uint32_t e = (ql - first) < CH ? (ql - first) : CH;
    const uint64_t *q0 = a.queue + a.stages[vi * a.NS + s].qoff;
    const uint32_t mine = first + (uint32_t)lane * K;
    const uint32_t endq = first + e;
    typename SL::Vec hiV, openV;
#pragma unroll
    for (int r = 0; r < SL::NV; ++r) {
        hiV[r] = 0u;
        openV[r] = 0u;
    }
    uint32_t alive = 0u;
#pragma nounroll
    for (int k = 0; k < K; ++k) {
        if (mine + k >= endq) break;
        alive |= 1u << k;
        const uint64_t *en = q0 + (uint64_t)(mine + k) * EW;
        uint64_t hw[W], ow[W];
#pragma unroll
        for (int wj = 0; wj < W; ++wj) {
            hw[wj] = ld64(en + 2 + wj);
            ow[wj] = ld64(en + 2 + W + wj);
        }
#pragma unroll
        for (int r = 0; r < SL::NV0; ++r) {
            const int t0 = r * SL::E;
            constexpr uint32_t EM = (uint32_t)((1ull << SL::E) - 1ull);
            const uint32_t hb = (uint32_t)(hw[t0 >> 6] >> (t0 & 63)) & EM;
            const uint32_t ob = (uint32_t)(ow[t0 >> 6] >> (t0 & 63)) & EM;
            uint32_t hs = 0u, os = 0u;
#pragma unroll
            for (int f = 0; f < SL::E; ++f) {
                hs |= ((hb >> f) & 1u) << (SL::K * f);
                os |= ((ob >> f) & 1u) << (SL::K * f);
            }
            hiV[r] |= hs << k;
            openV[r] |= os << k;
        }
    }
    constexpr bool v0inP = PH == 0;
    constexpr uint32_t Plocal = v0inP ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    uint32_t pvtop = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) pvtop |= (uint32_t)(i + (v0inP ? 0 : 1)) << (4 * i);
    uint32_t dom = 0u, pts = 0u;
    walk_sliced<L, K, L>(Plocal, pvtop, alive, hiV, openV, alive, dom, pts);
    const bool hsub_on = !(L == a.kmax && PH == 1);
#pragma nounroll
    for (int k = 0; k < K; ++k) {
        if (mine + k >= endq) break;
        const uint64_t *en = q0 + (uint64_t)(mine + k) * EW;
        const uint64_t e0 = ld64(en), e1 = ld64(en + 1);
        const float ts = __uint_as_float((uint32_t)(e0 >> 32));
        const float hch = __uint_as_float((uint32_t)e1);
        const bool d = (dom >> k) & 1u;
        const uint32_t slot = (uint32_t)e0, sslot = (uint32_t)(e1 >> 32);
        if (slot >= a.work_slots || sslot >= a.total_slots) {  // never: an entry read before it was written
            st32(a.done + 1, 2u);
            continue;
        }
        a.table[sslot] = d ? absent_f() : -ts;
        a.ptab[slot] = d ? absent_f() : -ts;
        if (hsub_on) a.phsub[slot] = d ? hch : fmaxf(hch, -ts);
    }
    return stage_add(a, vi, s, (uint64_t)e, lane);
}

// ---- scheduling ------------------------------------------------------------------
struct Item {
    int kind;  // 0 none, 1 score tile, 2 walk chunk
    int vi, s;
    uint32_t idx;
};

// Every lane looks at one variable (the wave's rotation first): its current
// stage, a walk chunk ready to claim, a score tile left.  Walk chunks are
// preferred (they complete stages); among variables the first in rotation
// order wins.  The claim is an atomic (tile) or a CAS (chunk).
__device__ __forceinline__ Item find_work(const PipeArgs &a, int rot, int lane, bool &any_left) {
    Item it{0, 0, 0, 0};
    const int nv = a.nv;
    const int vi = lane < nv ? (rot + lane) % nv : 0;
    uint32_t s = kDone;
    if (lane < nv) s = ld32(a.stage_of + vi);
    bool walk_ok = false, score_ok = false;
    uint32_t c = 0;
    if (s != kDone) {
        const PipeStage &st = a.stages[vi * a.NS + s];
        PipeCtr *ct = a.ctr + vi * a.NS + s;
        const int L = (int)s / 2 + 1;
        if (L > a.Ls) {
            // the stage counter first: once it shows every tile done, the
            // queue length and fill counters read after it are final
            const uint64_t u = ld64(&ct->units);
            drain();
            const uint32_t T = (uint32_t)((u + 0x80000000ull) >> 32);
            const uint32_t ql = ld32(&ct->qlen);
            c = ld32(&ct->wclaim);
            drain();
            const uint32_t CH = 64u * (uint32_t)pipe_k(L);
            if ((uint64_t)c * CH < ql) {
                const uint32_t f = ld32(a.fill + st.foff + c);
                const uint32_t want = (ql - c * CH) < CH ? (ql - c * CH) : CH;
                walk_ok = f == CH || (T == st.ntiles && f == want);
            }
        }
        score_ok = ld32(&ct->claim) < st.ntiles;
    }
    any_left = __ballot(s != kDone) != 0ull;
    const uint64_t wm = __ballot(walk_ok);
    if (wm) {
        const int l = __ffsll((long long)wm) - 1;
        uint32_t won = 0;
        if (lane == l) {
            PipeCtr *ct = a.ctr + vi * a.NS + s;
            won = __hip_atomic_compare_exchange_strong((gu32 *)&ct->wclaim, &c, c + 1, __ATOMIC_RELAXED,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      ? 1u
                      : 0u;
        }
        won = __shfl(won, l);
        if (won) {
            it.kind = 2;
            it.vi = __shfl(vi, l);
            it.s = (int)__shfl(s, l);
            it.idx = __shfl(c, l);
            return it;
        }
    }
    const uint64_t sm = __ballot(score_ok);
    if (sm) {
        const int l = __ffsll((long long)sm) - 1;
        uint32_t t = 0xFFFFFFFFu, nt = 0;
        if (lane == l) {
            PipeCtr *ct = a.ctr + vi * a.NS + s;
            t = __hip_atomic_fetch_add((gu32 *)&ct->claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            nt = a.stages[vi * a.NS + s].ntiles;
        }
        t = __shfl(t, l);
        nt = __shfl(nt, l);
        if (t < nt) {
            it.kind = 1;
            it.vi = __shfl(vi, l);
            it.s = (int)__shfl(s, l);
            it.idx = t;
            return it;
        }
        it.kind = -1;  // lost the race: look again at once
    } else if (wm) {
        it.kind = -1;
    }
    return it;
}

template <int L>
__device__ __forceinline__ int run_item(const PipeArgs &a, const PipeShared &sh, const Item &it, int lane, WavePool &P) {
    const int ph = it.s & 1;
    if (it.kind == 2) {
        if constexpr (L >= 2) {
            if (ph == 0) return walk_chunk<L, 0>(a, it.vi, it.s, it.idx, lane);
            return walk_chunk<L, 1>(a, it.vi, it.s, it.idx, lane);
        }
        return -1;
    }
    if (L <= a.Ls) {
        if constexpr (L <= kPipeMaxSmall) {
            if (ph == 0) return tile_onepass<L, 0>(a, sh, it.vi, it.s, it.idx, lane);
            return tile_onepass<L, 1>(a, sh, it.vi, it.s, it.idx, lane);
        }
    } else {
        if constexpr (L >= 2) {
            if (ph == 0) return tile_twopass<L, 0>(a, sh, it.vi, it.s, it.idx, lane, P);
            return tile_twopass<L, 1>(a, sh, it.vi, it.s, it.idx, lane, P);
        }
    }
    return -1;
}

__device__ __forceinline__ int run_any(const PipeArgs &a, const PipeShared &sh, const Item &it, int lane, WavePool &P) {
    switch (it.s / 2 + 1) {
        case 1: return run_item<1>(a, sh, it, lane, P);
        case 2: return run_item<2>(a, sh, it, lane, P);
        case 3: return run_item<3>(a, sh, it, lane, P);
        case 4: return run_item<4>(a, sh, it, lane, P);
        case 5: return run_item<5>(a, sh, it, lane, P);
        case 6: return run_item<6>(a, sh, it, lane, P);
        default: return -1;
    }
}

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

// OCC: waves per SIMD the register allocation must allow (2: 197 VGPRs, no
// spills; 3: 168 VGPRs with a few spilled values) -- option pipe_occ.
template <int OCC>
__global__ void __launch_bounds__(kBlock, OCC) pipe_kernel(PipeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const PipeLds lay = pipe_lds(a.n, a.nv, a.S);
    double *g = reinterpret_cast<double *>(smem + lay.gram);
    uint32_t *binom = reinterpret_cast<uint32_t *>(smem + lay.binom);
    uint64_t *toff = reinterpret_cast<uint64_t *>(smem + lay.toff);
    int *meta = reinterpret_cast<int *>(smem + lay.meta);
    for (int i = threadIdx.x; i < a.n * a.n; i += kBlock) g[i] = a.gram[i];
    for (int i = threadIdx.x; i < 64 * kBinomK; i += kBlock) binom[i] = a.binom[i];
    for (int i = threadIdx.x; i <= a.nv * a.S; i += kBlock) toff[i] = a.tbl_off[i];
    for (int i = threadIdx.x; i < a.nv * 4; i += kBlock) meta[i] = a.meta[i];
    __syncthreads();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    WavePool &P = reinterpret_cast<WavePool *>(smem + lay.pool)[wid];
    const PipeShared sh{g, binom, toff, meta};
    // Every XCD starts its search at its own run of variables (their slabs
    // then mostly stay in that XCD's L2), and the waves of one XCD spread over
    // that run.
    const int xcc = (int)xcc_id();
    const int vlo = xcc * a.nv / 8, vhi = (xcc + 1) * a.nv / 8;
    const int own = vhi > vlo ? vhi - vlo : 1;
    const int rot = (vlo + (int)(((blockIdx.x >> 3) * 4u + (uint32_t)wid) % (uint32_t)own)) % a.nv;
    uint64_t idle_since = 0;
    int backoff = 1;
    // ULG_PIPE_STATS: wall-clock ticks and counts per activity, summed over waves
    uint64_t st_find = 0, st_idle = 0, st_t[3] = {0, 0, 0}, st_n[3] = {0, 0, 0}, st_polls = 0, st_lost = 0;
    const bool stats = a.stats != nullptr;
    while (true) {
        bool any_left = true;
        const uint64_t t0 = stats ? wall_clock64() : 0;
        Item it = find_work(a, rot, lane, any_left);
        // wave-uniform in SGPRs: the dispatch below then branches on scalars
        // and each item form keeps its own register allocation
        it.kind = __builtin_amdgcn_readfirstlane(it.kind);
        it.vi = __builtin_amdgcn_readfirstlane(it.vi);
        it.s = __builtin_amdgcn_readfirstlane(it.s);
        it.idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)it.idx);
        if (stats) {
            st_find += wall_clock64() - t0;
            ++st_polls;
        }
        if (it.kind > 0) {
            idle_since = 0;
            backoff = 1;
            Item cur = it;
            while (true) {
                const uint64_t t1 = stats ? wall_clock64() : 0;
                const int nxt = run_any(a, sh, cur, lane, P);
                if (stats) {
                    const int kk = cur.kind == 2 ? 2 : ((cur.s / 2 + 1) <= a.Ls ? 0 : 1);
                    st_t[kk] += wall_clock64() - t1;
                    ++st_n[kk];
                }
                // The wave that released a variable's next stage starts on it
                // at once (the chain's critical path, and its slabs are warm
                // in this XCD's L2); other waves join through find_work.
                if (nxt < 0 || !a.chain) break;
                uint32_t t = 0;
                if (lane == 0)
                    t = __hip_atomic_fetch_add((gu32 *)&a.ctr[cur.vi * a.NS + nxt].claim, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
                if (t >= a.stages[cur.vi * a.NS + nxt].ntiles) break;
                cur = Item{1, cur.vi, nxt, t};
            }
            continue;
        }
        if (it.kind < 0) {
            if (stats) ++st_lost;
            continue;
        }
        if (!any_left) break;  // every variable's last stage is published
        const uint64_t now = wall_clock64();
        if (idle_since == 0) idle_since = now;
        if (now - idle_since > a.timeout) {
            if (lane == 0) st32(a.done + 1, 1u);  // stalled: the host fails the call
            break;
        }
        if (ld32(a.done + 1)) break;
        // nothing to claim: back off (up to ~6 us) so idle waves do not
        // flood the counters' lines while the others work
        for (int b = 0; b < backoff; ++b) __builtin_amdgcn_s_sleep(8);
        backoff = backoff < 32 ? 2 * backoff : 32;
        if (stats) st_idle += wall_clock64() - now;
    }
    if (stats && lane == 0) {
        const uint64_t v[11] = {st_find, st_idle, st_t[0], st_t[1], st_t[2], st_n[0], st_n[1], st_n[2], st_polls, 1, 0};
        for (int i = 0; i < 10; ++i)
            __hip_atomic_fetch_add((gu64 *)(a.stats + i), v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gu64 *)(a.stats + 14), st_lost, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

namespace ulg {

int pipe_chunk_sets(int L) { return 64 * pipe_k(L); }
int pipe_entry_words(int L) { return entry_words(L); }

int pipe_prepare(ulg_ctx *c, int nv, int S, int kmax, int max_parents, const std::vector<int> &mv,
                 const std::vector<int> &meta, PipeArgs &a) {
    const int NS = 2 * kmax;
    const int Ls = std::max(1, std::min(kPipeMaxSmall, std::min(kmax, c->score_small_layers)));
    const int R = std::max(1, std::min(c->pipe_rounds, kPipePool / 64)), Rs = std::max(1, c->pipe_rounds_small);
    std::vector<PipeStage> stages((size_t)nv * NS);
    std::vector<uint32_t> first(nv, kDone);
    uint64_t qwords = 0, fills = 0;
    uint64_t wslots = 32;  // line 0: never written (the gathers' masked lanes load it)
    for (int vi = 0; vi < nv; ++vi) {
        const int m = mv[vi];
        const bool z = meta[vi * 4 + 2] != 0;
        for (int s = 0; s < NS; ++s) {
            const int L = s / 2 + 1, ph = s & 1;
            uint64_t cnt = 0;
            if (L <= max_parents) cnt = ph == 0 ? (z ? binom64(m - 1, L - 1) : 0) : (z ? binom64(m - 1, L) : binom64(m, L));
            if (cnt >= (1ull << 31)) return set_err(c, ULG_ERR_UNSUPPORTED, "pipe: stage too large");
            PipeStage &st = stages[(size_t)vi * NS + s];
            st.nsets = (uint32_t)cnt;
            const uint64_t per = 64ull * (uint64_t)(L <= Ls ? Rs : R);
            st.ntiles = (uint32_t)((cnt + per - 1) / per);
            st.qoff = qwords;
            st.foff = (uint32_t)fills;
            st.slab = (uint32_t)wslots;
            st.pad = 0;
            wslots += (cnt + 31) / 32 * 32;  // whole 128-byte lines per stage
            st.next = kDone;
            if (L > Ls && cnt > 0) {
                qwords += cnt * (uint64_t)pipe_entry_words(L);
                fills += (cnt + (uint64_t)pipe_chunk_sets(L) - 1) / (uint64_t)pipe_chunk_sets(L);
            }
        }
        uint32_t nx = kDone;
        for (int s = NS - 1; s >= 0; --s) {
            PipeStage &st = stages[(size_t)vi * NS + s];
            st.next = nx;
            if (st.nsets > 0) nx = (uint32_t)s;
        }
        first[vi] = nx;
    }
    // state: [counters nv*NS lines][fill counters][done words], zeroed every
    // call as one block padded to 16 bytes; then the initial stages
    const size_t ctr_bytes = (size_t)nv * NS * sizeof(PipeCtr);
    const size_t fill_bytes = (size_t)((fills * 4 + 15) / 16 * 16);
    c->pipe_zero_bytes = ctr_bytes + fill_bytes + 16;
    const size_t state_bytes = c->pipe_zero_bytes + (size_t)(nv * 4 + 15) / 16 * 16;
    int rc;
    if ((rc = ensure(c, c->d_pstate, state_bytes)) || (rc = ensure(c, c->d_pqueue, (size_t)std::max<uint64_t>(qwords, 1))) ||
        (rc = ensure(c, c->d_pinit, (size_t)nv)))
        return rc;
    if (2 * wslots >= 0xFFFFFFFFull) return set_err(c, ULG_ERR_UNSUPPORTED, "pipe: work layout too large");
    if ((rc = ensure(c, c->d_pwork, (size_t)(2 * wslots)))) return rc;
    std::vector<uint8_t> sbytes(stages.size() * sizeof(PipeStage));
    std::memcpy(sbytes.data(), stages.data(), sbytes.size());
    if ((rc = upload(c, c->d_pstages, c->mir_pstages, sbytes))) return rc;
    if ((rc = upload(c, c->d_pinit, c->mir_pinit, first))) return rc;
    uint8_t *base = c->d_pstate.p;
    a.stages = reinterpret_cast<const PipeStage *>(c->d_pstages.p);
    a.ctr = reinterpret_cast<PipeCtr *>(base);
    a.fill = reinterpret_cast<uint32_t *>(base + ctr_bytes);
    a.done = reinterpret_cast<uint32_t *>(base + ctr_bytes + fill_bytes);
    a.stage_of = reinterpret_cast<uint32_t *>(base + c->pipe_zero_bytes);
    a.queue = c->d_pqueue.p;
    a.gram = c->gram.p;
    a.binom = c->d_binom.p;
    a.cand = c->d_cand.p;
    a.meta = c->d_meta.p;
    a.tbl_off = c->d_tbl_off.p;
    a.table = c->table.p;
    a.ptab = c->d_pwork.p;
    a.phsub = c->d_pwork.p + wslots;
    a.N = (double)c->N;
    a.lambda = c->lambda;
    a.n = c->n;
    a.nv = nv;
    a.S = S;
    a.NS = NS;
    a.kmax = kmax;
    a.Ls = Ls;
    a.R = R;
    a.Rsmall = Rs;
    a.chain = c->pipe_chain;
    a.total_slots = (uint32_t)(c->table.cap < 0xFFFFFFFFull ? c->table.cap : 0xFFFFFFFFull);
    a.work_slots = (uint32_t)wslots;
    a.stats = nullptr;
    if (std::getenv("ULG_PIPE_STATS")) {
        if ((rc = ensure(c, c->d_pstats, 16))) return rc;
        a.stats = c->d_pstats.p;
    }
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
    a.timeout = (uint64_t)khz * 1000ull * 10ull;  // 10 s idle
    c->pipe_nv = nv;
    return ULG_OK;
}

int pipe_launch(ulg_ctx *c, const PipeArgs &a, hipStream_t st) {
    ULG_HIP(c, hipMemsetAsync(c->d_pstate.p, 0, c->pipe_zero_bytes, st));
    if (a.stats) ULG_HIP(c, hipMemsetAsync(a.stats, 0, 16 * 8, st));
    ULG_HIP(c, hipMemcpyAsync(a.stage_of, c->d_pinit.p, (size_t)a.nv * 4, hipMemcpyDeviceToDevice, st));
    const PipeLds lay = pipe_lds(a.n, a.nv, a.S);
    void (*kfn)(PipeArgs) = c->pipe_occ == 3 ? pipe_kernel<3> : pipe_kernel<2>;
    if (lay.total > 64 * 1024)
        ULG_HIP(c, hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, lay.total));
    // every workgroup resident: waves wait only for work other resident waves
    // hold, but a grid beyond residency would just queue behind them
    int per_cu = 0;
    ULG_HIP(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kBlock, (size_t)lay.total));
    if (c->pipe_cus == 0) {
        hipDeviceProp_t pr;
        ULG_HIP(c, hipGetDeviceProperties(&pr, c->device));
        c->pipe_cus = pr.multiProcessorCount;
    }
    int grid = std::max(1, per_cu) * std::max(1, c->pipe_cus);
    if (c->pipe_grid_max > 0) grid = std::min(grid, c->pipe_grid_max);  // A/B: fewer workers
    prof_begin_s(c, "score_pipe", st);
    hipLaunchKernelGGL(kfn, dim3((unsigned)grid), dim3(kBlock), (size_t)lay.total, st, a);
    prof_end_s(c, st);
    ULG_HIP(c, hipGetLastError());
    return ULG_OK;
}

void pipe_report(ulg_ctx *c) {
    if (!std::getenv("ULG_PIPE_STATS") || !c->d_pstats.p) return;
    uint64_t v[16] = {0};
    if (hipMemcpy(v, c->d_pstats.p, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return;
    const double tick = 1e-2;  // wall clock 100 MHz: us per tick
    std::fprintf(stderr,
                 "pipe_stats waves=%llu polls=%llu find_us=%.0f idle_us=%.0f | onepass n=%llu us=%.0f | twopass n=%llu "
                 "us=%.0f | walk n=%llu us=%.0f | per item us: onepass %.2f twopass %.2f walk %.2f find %.2f\n",
                 (unsigned long long)v[9], (unsigned long long)v[8], v[0] * tick, v[1] * tick,
                 (unsigned long long)v[5], v[2] * tick, (unsigned long long)v[6], v[3] * tick,
                 (unsigned long long)v[7], v[4] * tick, v[5] ? v[2] * tick / v[5] : 0.0, v[6] ? v[3] * tick / v[6] : 0.0,
                 v[7] ? v[4] * tick / v[7] : 0.0, v[8] ? v[0] * tick / v[8] : 0.0);
    std::fprintf(stderr,
                 "pipe_stats twopass per tile us: score rounds %.2f, gathers+queue %.2f, final drain %.2f; pooled sets "
                 "per tile %.1f; lost claims %llu\n",
                 v[6] ? v[10] * tick / v[6] : 0.0, v[6] ? v[11] * tick / v[6] : 0.0, v[6] ? v[12] * tick / v[6] : 0.0,
                 v[6] ? (double)v[13] / v[6] : 0.0, (unsigned long long)v[14]);
}

int pipe_check(ulg_ctx *c) {
    if (c->pipe_stall_pinned && *c->pipe_stall_pinned)
        return set_err(c, ULG_ERR_HIP, *c->pipe_stall_pinned == 2
                                           ? "ulg_cbic_score: the scoring pipeline read a walk entry before it was written"
                                           : "ulg_cbic_score: the scoring pipeline stalled (a wave waited 10 s for work)");
    return ULG_OK;
}

}  // namespace ulg
