// cbic.hip -- continuous-BIC parent-set scoring on MI355X (gfx950).
//
// Reference path (ninalu/urlearning-cpp, urlearning/):
//   BIC_OLS_Function ctor          scoring_function/BIC_OLS.cpp:30-123
//   calculateScoreAndBeta          BIC_OLS.cpp:277-389 (mlpack OLS, no intercept)
//   calculateScore                 BIC_OLS.cpp:174-276 (store / prune rule)
//   find_best_subset_score         BIC_OLS.cpp:125-172 (dominance recursion)
//   calculateScores_internal       score_calculator.cpp:54-135 (layers, Gosper)
//
// Design (MI355X-first):
//   * the data is normalised once and the FP64 Gram matrix G = Z'Z is built
//     with v_mfma_f64_16x16x4_f64 (the only dense contraction on the path);
//   * every parent set is then one lane: gather G[P,P], G[P,v] from LDS,
//     k x k Cholesky in registers, RSS = G[v,v] - |L^-1 b|^2;
//   * the dominance recursion (whose result depends on the reference's
//     zero-padded parent vector and XOR-toggle) is replayed
//     exactly on per-lane bitsets over subsets of P u {variable 0};
//   * a layer is two launches -- sets that contain variable 0, then the rest
//      -- which reproduces the sequential Gosper order;
//   * every (variable, layer) owns a dense float slab indexed by the colex
//     rank of the set inside the variable's candidate list (= the Gosper
//     enumeration index), holding the stored score or an absent sentinel.
#include <cstdio>
#include <atomic>
#include <thread>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "search_internal.h"
#include "host_walk.h"
#include "cbic_dev.h"

using namespace ulg;

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kGramRows = 1024;  // rows of Z per Gram wave (split-K chunk)


// ------------------------------------------------------------------------
// Normalisation (BIC_OLS.cpp:66-97): x - mean, divided by the sample std
// (N-1) of the centred column.  Deterministic tree reductions.
// ------------------------------------------------------------------------
__device__ double block_sum(double v, double *red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    double r = red[0];
    __syncthreads();
    return r;
}

__global__ void __launch_bounds__(kBlock) colstats_kernel(const double *raw, int64_t N, double *stat) {
    __shared__ double red[kBlock];
    const double *x = raw + (int64_t)blockIdx.x * N;
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += kBlock) s += x[i];
    const double mean = block_sum(s, red) / (double)N;
    // arma::var(x - mean): two-pass with the compensation term
    double s2 = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += kBlock) s2 += x[i] - mean;
    const double m2 = block_sum(s2, red) / (double)N;
    double a2 = 0.0, a3 = 0.0;
    for (int64_t i = threadIdx.x; i < N; i += kBlock) {
        const double t = m2 - (x[i] - mean);
        a2 += t * t;
        a3 += t;
    }
    a2 = block_sum(a2, red);
    a3 = block_sum(a3, red);
    if (threadIdx.x == 0) {
        const double var = N > 1 ? (a2 - a3 * a3 / (double)N) / (double)(N - 1) : 0.0;
        stat[2 * blockIdx.x] = mean;
        stat[2 * blockIdx.x + 1] = sqrt(var);
    }
}

// Z row-major N x npad (padded columns zero): lanes of a wave read one row.
__global__ void __launch_bounds__(kBlock) normalise_kernel(const double *raw, int64_t N, int n, int npad,
                                                           const double *stat, double *z) {
    const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= N * npad) return;
    const int64_t r = idx / npad;
    const int c = (int)(idx % npad);
    double v = 0.0;
    if (c < n) v = (raw[(int64_t)c * N + r] - stat[2 * c]) / stat[2 * c + 1];
    z[idx] = v;
}

// G = Z'Z on v_mfma_f64_16x16x4_f64.  One wave per (16x16 tile, row chunk).
// A[i][k] = Z[r0+k][I0+i], B[k][j] = Z[r0+k][J0+j]; lane l holds
// i = j = l & 15, k = l >> 4.  D: col = l & 15, row = (l >> 4) + 4 * reg.
__global__ void __launch_bounds__(64) gram_mfma_kernel(const double *z, int64_t N, int npad, int tiles,
                                                       double *partials) {
    const int chunk = blockIdx.x;
    const int tile = blockIdx.y;
    const int I0 = (tile / tiles) * 16, J0 = (tile % tiles) * 16;
    const int lane = threadIdx.x;
    const int i = lane & 15, k = lane >> 4;
    const int64_t rb = (int64_t)chunk * kGramRows;
    const int64_t re = rb + kGramRows < N ? rb + kGramRows : N;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int64_t r0 = rb; r0 < re; r0 += 4) {
        const int64_t r = r0 + k;
        double a = 0.0, b = 0.0;
        if (r < re) {
            a = z[r * npad + I0 + i];
            b = z[r * npad + J0 + i];
        }
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    double *out = partials + ((int64_t)chunk * tiles * tiles + tile) * 256;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
        const int row = (lane >> 4) + 4 * reg;
        out[row * 16 + (lane & 15)] = acc[reg];
    }
}

__global__ void __launch_bounds__(kBlock) gram_reduce_kernel(const double *partials, int chunks, int tiles, int n,
                                                             double *gram) {
    const int idx = blockIdx.x * kBlock + threadIdx.x;
    if (idx >= n * n) return;
    const int r = idx / n, c = idx % n;
    const int tile = (r / 16) * tiles + (c / 16);
    const int e = (r % 16) * 16 + (c % 16);
    double s = 0.0;
    for (int ch = 0; ch < chunks; ++ch) s += partials[((int64_t)ch * tiles * tiles + tile) * 256 + e];
    gram[idx] = s;
}


struct ScoreArgs {
    const double *gram;      // n x n row-major
    const uint32_t *binom;   // [64][kBinomK]
    const uint8_t *cand;     // [nv][64] compact index -> variable
    const int *meta;         // [nv][4]: variable, m, var0in, -
    const uint64_t *tbl_off; // [nv*S + 1] start of (vi, layer) slab
    const uint64_t *work;    // [nv + 1] prefix of this launch's sets
    float *table;
    float *hsub;                // variant bit 6: per slot, the maximum stored value over the set's
                                // nonempty subsets (the set included; NaN = none), table layout
    uint64_t *queue;            // variant bit 4: lanes left for the walk launch
    unsigned long long *qcount;
    unsigned long long *err;    // the call's error word (kErrQueue: a walk-queue segment overflowed)
    uint8_t *qkey;              // bucketed walk launches: per queue entry, its walk key
    double N;
    double lambda;
    int n, nv, S;
    int xcd;                    // remap blocks so each XCD takes a contiguous run of sets
    int hsub_out;               // write the subset maxima (0: the top layer's phase 1, never read)
};

// Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8),
// and each XCD has its own L2.  With xcd set, XCD x takes the x-th contiguous
// eighth of the launch's blocks -- the sets of a few variables, whose slabs
// then stay in that XCD's L2 -- through a bijection of [0, nb).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb, int on) {
    if (!on) return b;
    const uint32_t x = b & 7u, k = b >> 3, q = nb >> 3, r = nb & 7u;
    return x * q + (x < r ? x : r) + k;
}


// LDS carve: gram | binom | work | tbl_off | meta | candidate lists |
// recursion stack (variant bit 1)
// | LDS bitsets (3 per lane when they have >= 4 words) | the block's
// undecided sets after the subset-maxima test (variant bits 4 + 6: a count,
// then per entry compact mask, slot, ts, children maximum, variable) (16-B
// aligned)
struct LdsLayout {
    int gram, binom, work, toff, meta, cand, stack, bits, cmp, cmp2, total;
};
constexpr int kCmpEntryBytes = 8 + 4 + 4 + 4 + 4;
__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }
#ifndef ULG_LDS_ALIAS
#define ULG_LDS_ALIAS 1
#endif
__host__ __device__ inline LdsLayout lds_layout(int n, int nv, int S, int L, int V) {
    LdsLayout l;
    if (ULG_LDS_ALIAS && (V & 208) == 208 && bits_words(L) < 4) {
        // the two-pass kernels with the second compaction (variant bit 7):
        // the Gram matrix, the work prefixes and the candidate lists are
        // read only before the block's first barrier (the scores and the
        // subset-maxima settle), and the compaction entries and their words
        // are written only after it -- so they share one region.  The
        // counters, the binomials, the slab offsets and the metadata, read
        // throughout, sit in front of it.  C3 layer 6: 26.7 -> 19 KB per
        // block, 6 -> 8 blocks per CU (C5: 5 -> 8).
        const int W = bits_words(L);
        l.binom = 0;
        l.toff = align16(l.binom + 64 * kBinomK * 4);
        l.meta = align16(l.toff + (nv * S + 1) * 8);
        l.cmp = align16(l.meta + nv * 4 * 4);  // 16 bytes of counters, then the entries
        const int ra = l.cmp + 16;             // the shared region
        l.gram = ra;
        l.work = align16(l.gram + n * n * 8);
        l.cand = align16(l.work + (nv + 1) * 8);
        l.stack = l.bits = align16(l.cand + nv * 64);
        l.cmp2 = align16(ra + kBlock * kCmpEntryBytes);
        const int endc = l.cmp2 + 2 * W * kBlock * 8;
        l.total = l.stack > endc ? l.stack : endc;
        return l;
    }
    l.gram = 0;
    l.binom = align16(l.gram + n * n * 8);
    l.work = align16(l.binom + 64 * kBinomK * 4);
    l.toff = align16(l.work + (nv + 1) * 8);
    l.meta = align16(l.toff + (nv * S + 1) * 8);
    l.cand = align16(l.meta + nv * 4 * 4);
    l.stack = align16(l.cand + nv * 64);
    l.bits = l.stack;
    const int W = bits_words(L);
    l.cmp = align16(l.bits + (W >= 4 ? 3 * W * kBlock * 8 : 0));
    // variant bit 7: the second compaction carries each set's gathered
    // present / hi words (register bitsets only, W < 4)
    l.cmp2 = align16(l.cmp + ((V & 80) == 80 ? 16 + kBlock * kCmpEntryBytes : 0));
    l.total = l.cmp2 + ((V & 208) == 208 && W < 4 ? 2 * W * kBlock * 8 : 0);
    return l;
}



// The walk queue of a two-pass launch is cut into nseg = ceil(blocks /
// kSegBlocks) segments, each with its own counter on its own 128-byte line:
// one counter for the whole launch took ~23 K wave atomics in a row at C3's
// layer 6 and cost a third of the scoring kernel (318 -> 204 us without it).
// Block b queues into segment b mod nseg, so the blocks resident at any time
// spread over all counters and every segment is a cross-section of the
// launch (segments of neighbouring blocks cluster the long walks into the
// same walk waves: the layer-6 walk launch took 2x longer).  Segment s holds
// its queued sets at entries [s * kSegEntries, s * kSegEntries + count_s);
// the walk kernel takes one (segment, chunk) per wave.
constexpr int kSegBlocks = 32;
constexpr uint64_t kSegEntries = (uint64_t)kSegBlocks * kBlock;
constexpr int kSegStride = 16;  // counters 128 B apart
// A bucketed launch's header after its segment counters (zeroed with them):
// every key's set total (u32 64..191).
constexpr int kBucketHdrWords = 128;
// Bits of the call's error word (d_qcount[nqc - 1], zeroed by the prologue,
// copied beside the stored count by scan_kernel): a wide walk over its cap;
// a queue position past its segment (nothing is written there); a walk entry
// whose table slot lies past the call's slots (its decision is not written).
constexpr unsigned long long kErrWide = 1ull, kErrQueue = 2ull, kErrSlot = 4ull;
__host__ __device__ inline uint64_t seg_count(uint64_t blocks) { return (blocks + kSegBlocks - 1) / kSegBlocks; }
__device__ __forceinline__ uint64_t walk_segment() { return blockIdx.x % seg_count(gridDim.x); }

// Append a set to the walk queue (wave-aggregated: one atomic per wave on the
// segment's counter): table slot | ts bits << 32, the hi words, then the open
// words (open = absent & cover(T without var 0) & not checked; checked =
// {empty}).  queue / qcount: the segment's entries and counter.
// The walk key of a queued set (walk_bucket): which of the walk's first-level
// nodes (P minus one member, the top call's tests) it may expand, one bit per
// member -- sets with the same key start the same union walk, so a launch
// sorted by key walks ~3x fewer union points (scripts/walk_sched_study.cpp).
// When every first-level node is open (the longest, least alike walks), the
// key is 64 + the open bits of six second-level nodes (P minus two members,
// the first six pairs in order): those sets then split further (C3 layer 6
// with variable 0: the longest wave 432 -> 294 union points).
template <int L, int PHASE, int W>
__device__ __forceinline__ uint32_t walk_key(const uint64_t (&ow)[W]) {
    constexpr uint32_t root = PHASE == 0 ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    constexpr int off = PHASE == 0 ? 0 : 1;
    uint32_t key = 0;
#pragma unroll
    for (int a = 0; a < L; ++a) {
        const uint32_t t = root ^ (1u << (a + off));
        key |= (uint32_t)((ow[t >> 6] >> (t & 63u)) & 1ull) << a;
    }
    if (key == (1u << L) - 1u) {
        uint32_t sec = 0;
        int nb = 0;
#pragma unroll
        for (int a = 0; a < L; ++a)
#pragma unroll
            for (int b = a + 1; b < L; ++b) {
                if (nb < 6) {
                    const uint32_t t = root ^ (1u << (a + off)) ^ (1u << (b + off));
                    sec |= (uint32_t)((ow[t >> 6] >> (t & 63u)) & 1ull) << nb;
                }
                ++nb;
            }
        key = 64u + sec;
    }
    return key;
}

template <int L, int PHASE, class BS>
__device__ __forceinline__ void queue_walk(const BS &present, const BS &hi, uint64_t *queue,
                                           unsigned long long *qcount, unsigned long long *err, uint64_t slot,
                                           float ts, uint8_t *qkey = nullptr) {
    constexpr int W = BS::kWords;
    const unsigned long long act = __ballot(1);
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)act) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(qcount, (unsigned long long)__popcll(act));
    base = __shfl(base, leader);
    const uint64_t pos = base + (uint64_t)__popcll(act & ((1ull << lane) - 1ull));
    // a segment holds at most kSegBlocks blocks' lanes by construction
    // (seg_count); a sizing mistake becomes an error status, not a stray write
    if (pos >= kSegEntries) {
        if (err) atomicOr(err, kErrQueue);
        return;
    }
    uint64_t ow[W];
#pragma unroll
    for (int wj = 0; wj < W; ++wj) ow[wj] = hi.word(wj);
    cover_words<W>(ow);
#pragma unroll
    for (int wj = 0; wj < W; ++wj) {
        const uint64_t ce = ow[wj] & 0x5555555555555555ull;
        ow[wj] = (ce | (ce << 1)) & ~present.word(wj) & (wj == 0 ? ~1ull : ~0ull);
    }
    if constexpr (W < 4)
        if (qkey) qkey[pos] = (uint8_t)walk_key<L, PHASE, W>(ow);
    uint64_t *e = queue + pos * (uint64_t)(1 + 2 * W);
    e[0] = slot | ((uint64_t)fbits(ts) << 32);
#pragma unroll
    for (int wj = 0; wj < W; ++wj) e[1 + wj] = hi.word(wj);
#pragma unroll
    for (int wj = 0; wj < W; ++wj) e[1 + W + wj] = ow[wj];
}



#ifdef ULG_GATHER_STATS
// Diagnostic build only (scripts/gather_stats.py): per (layer, phase) counts of
// what the presence gathers of the compacted sets find.
__device__ unsigned long long g_gstats[2 * (kMaxL + 1) * 16];

// Compile-time masks over the local subsets t of a layer-L set: the keys the
// full gather reads, the keys without child i's removed member (child i =
// P minus its i-th member in compact order), the keys holding variable 0.
template <int L, int PHASE>
struct KeyMasks {
    static constexpr int Q = PHASE == 0 ? L : L + 1;
    static constexpr int W = bits_words(L);
    uint64_t key[W], miss[L][W], v0[W];
    constexpr KeyMasks() : key{}, miss{}, v0{} {
        constexpr PresList<L, PHASE, Q, 0> PL{};
        for (int i = 0; i < PL.n; ++i) key[PL.t[i] >> 6] |= 1ull << (PL.t[i] & 63);
        for (uint32_t t = 0; t < (1u << Q); ++t) {
            if (t & 1u) v0[t >> 6] |= 1ull << (t & 63);
            for (int i = 0; i < L; ++i) {
                const int b = PHASE == 1 ? i + 1 : i;
                if (!((t >> b) & 1u)) miss[i][t >> 6] |= 1ull << (t & 63);
            }
        }
    }
};

template <int L, int PHASE, class BS>
__device__ void gather_stats(const BS &present, const BS &hi, uint32_t hotA, uint32_t hotZ, bool z, bool queued) {
    constexpr int W = BS::kWords;
    constexpr KeyMasks<L, PHASE> KM{};
    uint64_t cov[W];
#pragma unroll
    for (int j = 0; j < W; ++j) cov[j] = hi.word(j);
    cover_words<W>(cov);
    unsigned long long c[16] = {};
    c[0] = 1;
    c[1] = __builtin_popcount(hotA);
    c[2] = __builtin_popcount(hotZ);
    const uint32_t sel = (PHASE == 1 && z) ? hotZ : hotA;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        uint64_t need = 0, hrel = 0;
#pragma unroll
        for (int i = 0; i < L; ++i) {
            if ((sel >> i) & 1u) need |= KM.miss[i][j];
            if ((hotA >> i) & 1u) hrel |= KM.miss[i][j] & ~KM.v0[j];
            if (PHASE == 1 && z && ((hotZ >> i) & 1u)) hrel |= KM.miss[i][j] & KM.v0[j];
        }
        need &= KM.key[j];
        hrel &= KM.key[j];
        const uint64_t pr = present.word(j) & KM.key[j], hw = hi.word(j) & KM.key[j], cv = cov[j] & KM.key[j];
        c[3] += __builtin_popcountll(pr);
        c[4] += __builtin_popcountll(hw);
        c[5] += __builtin_popcountll(need);
        c[6] += __builtin_popcountll(hrel);
        c[7] += __builtin_popcountll(cv);
        c[8] += __builtin_popcountll(pr & need);
        c[9] += __builtin_popcountll(hw & ~hrel);
        c[10] += __builtin_popcountll(cv & ~need);
        c[11] += __builtin_popcountll(KM.key[j]);
        c[13] += __builtin_popcountll((hrel | cv) & KM.key[j]);
        c[14] += __builtin_popcountll(pr & ~need);
    }
    c[12] = queued;
    unsigned long long *g = g_gstats + (L * 2 + PHASE) * 16;
#pragma unroll
    for (int i = 0; i < 15; ++i) atomicAdd(g + i, c[i]);
}
#endif

// Set r of variable vi's (layer L, phase) launch: its compact mask over the
// candidate list, colex rank, and parent variables in ascending order (==
// BIC_OLS parent_vec order).  smeta / scand / binom: the LDS copies.
template <int L>
struct SetHead {
    int v;
    bool z;
    uint64_t cm, rankP;
    int gv[L];
};
template <int L, int PHASE>
__device__ __forceinline__ SetHead<L> set_head(const int *smeta, const uint8_t *scand, const uint32_t *binom, int vi,
                                               uint64_t r) {
    SetHead<L> h;
    h.v = smeta[vi * 4 + 0];
    const int m = smeta[vi * 4 + 1];
    h.z = smeta[vi * 4 + 2] != 0;
    if (PHASE == 0) h.cm = (unrank_colex(r, L - 1, m - 1, binom) << 1) | 1ull;
    else if (h.z) h.cm = unrank_colex(r, L, m - 1, binom) << 1;
    else h.cm = unrank_colex(r, L, m, binom);
    h.rankP = rank_colex(h.cm, binom);
    const uint8_t *cl = scand + vi * 64;
    uint64_t rem = h.cm;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const int b = __builtin_ctzll(rem);
        rem &= rem - 1;
        h.gv[i] = cl[b];
    }
    return h;
}

// The one-pass form of one set (variant bit 4 clear): presence gathers, the
// walk in registers (or LDS bitsets from 4 words), the store rule, and under
// bit 6 the subset maxima.  Shared by score_layer_kernel and the fused small
// layers (score_small_kernel).
template <int L, int PHASE, int V>
__device__ __forceinline__ void one_pass_set(const ScoreArgs &a, unsigned char *smem, const LdsLayout &lay,
                                             const uint32_t *binom, const uint64_t *toff, int vi, bool z, uint64_t cm,
                                             uint64_t rankP, float ts) {
    constexpr bool HM = (V & 64) != 0;
    // the children's subset maxima (bit 6), loaded before the gathers so both
    // share one memory round trip
    float hch = absent_f();
    if constexpr (HM && L > 1) {
        const uint64_t vbase = (uint64_t)vi * a.S;
        uint64_t rc[L], rz[L];
        child_ranks<L, false>(cm, binom, rc, rz);
        float ch[L];
#pragma unroll
        for (int i = 0; i < L; ++i) ch[i] = a.hsub[toff[vbase + L - 1] + rc[i]];
#pragma unroll
        for (int i = 0; i < L; ++i) hch = fmaxf(hch, ch[i]);
    }
    // small layers (one bitset word, unrolled gathers): the gathered values
    // stay in registers, so the walk's best needs no second round trip
    constexpr int QV = PHASE == 0 ? L : L + 1;
    constexpr bool KEEPV = bits_words(L) == 1 && (V & 1) && !(V & 16) && QV <= 5;
    float out;
    bool queued = false;  // variant bit 4: left for the walk launch
    if (ts >= 0.0f) {
        // returned -ts; the caller stores it iff it is < 0 (score_calculator.cpp:111)
        const float s = -ts;
        out = (s < 0.0f) ? s : absent_f();
    } else {
        constexpr int W = bits_words(L);
        using BS = std::conditional_t<(W >= 4), BitsLds<W>, Bits<W>>;
        uint64_t *lds_bits = reinterpret_cast<uint64_t *>(smem + lay.bits) + threadIdx.x;
        const LocalSet<L> ls = local_set<L, PHASE>(cm, z);
        const uint64_t cpack = ls.cpack;
        const uint32_t Plocal = ls.Plocal;
        const uint32_t pvtop = ls.pvtop;
        const uint64_t vbase = (uint64_t)vi * a.S;

        // presence of every candidate key in the cache as it stands now
        // the first LDS bitset is `present`; `hi` and `checked` share the
        // second (only the decision-only walk uses `hi`); `visited` the third
        BS present = make_bits<BS>(lds_bits);
        BS hi = make_bits<BS>(lds_bits + (size_t)W * kBlock);
        present.clear();
        if constexpr ((V & 16) != 0) hi.clear();
        const float thr = -ts;
        float vals[KEEPV ? (1 << QV) : 1];
        if constexpr (KEEPV) {
#pragma unroll
            for (int t = 0; t < (1 << QV); ++t) vals[t] = 0.0f;
            presence_unrolled<L, PHASE, QV, W, LdPlain, 8, (V != 1), 0>(present, hi, thr, binom, ls.cpack, z, a.table,
                                                                        toff + vbase, vals);
        } else {
            gather_keys<L, PHASE, V>(present, hi, ls, thr, binom, z, a.table, toff + vbase);
        }

        if constexpr ((V & 16) != 0) {
            // decide what needs no walk; queue the rest for the walk kernel
            const bool dom = settle_rules<L, PHASE>(present, hi, ls, queued);
            if (queued) {
                const uint64_t seg = walk_segment();
                constexpr int QW = bits_words(L);
                queue_walk<L, PHASE>(present, hi, a.queue + seg * kSegEntries * (uint64_t)(1 + 2 * QW),
                                     a.qcount + seg * kSegStride, a.err, toff[vbase + L] + rankP, ts);
            }
            out = dom ? absent_f() : -ts;
        } else {
        BS checked = make_bits<BS>(lds_bits + (size_t)W * kBlock);
        BS visited = make_bits<BS>(lds_bits + (size_t)2 * W * kBlock);
        checked.clear();
        visited.clear();
        checked.set(0u);  // checked.insert(empty_set)
        best_subset<L, BS>(Plocal, pvtop, present, checked, visited);

        float best = 0.0f;
        if constexpr (KEEPV) {
            // every visited node is a present key, gathered above
            const uint64_t x = visited.word(0);
#pragma unroll
            for (int t = 0; t < (1 << QV); ++t)
                if (((x >> t) & 1ull) && vals[t] > best) best = vals[t];
        } else {
#pragma unroll
        for (int wj = 0; wj < W; ++wj) {
            uint64_t x = visited.word(wj);
            while (x) {
                const uint32_t t = (uint32_t)(wj * 64 + __builtin_ctzll(x));
                x &= x - 1;
                uint64_t rk = 0;
                uint32_t rem = t;
                int j = 0;
                while (rem) {
                    const int lb = __builtin_ctz(rem);
                    rem &= rem - 1;
                    ++j;
                    rk += B(binom, (int)((cpack >> (6 * lb)) & 63ull), j);
                }
                const float val = a.table[toff[vbase + __builtin_popcount(t)] + rk];
                if (val > best) best = val;
            }
        }
        }
        // BIC_OLS.cpp:234: best_subset_score + bic_threshold >= -the_score
        out = ((double)best + 0.0 >= (double)(-ts)) ? absent_f() : -ts;
        }
    }
    if (!queued) a.table[toff[(uint64_t)vi * a.S + L] + rankP] = out;
    // the one-pass form keeps the subset maxima for the layers above it
    if constexpr (HM)
        if (a.hsub_out) a.hsub[toff[(uint64_t)vi * a.S + L] + rankP] = fmaxf(out, hch);
}

// The rest of a queued set's gathers (the keys the rules did not read), then
// either the walk queue or, when the walk closure shows the walk cannot reach
// a key >= -ts, the store it would make.  toffv: this variable's slab offsets.
template <int L, int PHASE, int V, class BS>
__device__ __forceinline__ void walk_or_store(const ScoreArgs &a, BS &present, BS &hib, const LocalSet<L> &ls,
                                              float tk, const uint32_t *binom, bool zk, const uint64_t *toffv,
                                              uint64_t seg, uint64_t sk, float hch) {
    constexpr int W = BS::kWords;
#ifndef ULG_PROBE_NOPART2
    gather_keys<L, PHASE, V, BS, LdPlain, 2>(present, hib, ls, -tk, binom, zk, a.table, toffv);
#endif
    // no key >= -ts among the nodes the walk can test: it would store P
    // (80 % of the walked sets at C3's layer 6 end stored)
    bool may_hit = true;
    if constexpr (W < 4) {
        uint64_t pw[W], hw[W];
#pragma unroll
        for (int j = 0; j < W; ++j) {
            pw[j] = present.word(j);
            hw[j] = hib.word(j);
        }
        may_hit = walk_may_hit<L, PHASE, W>(pw, hw);
    }
    if (may_hit) {
#ifndef ULG_PROBE_NOQUEUE
        queue_walk<L, PHASE>(present, hib, a.queue + seg * kSegEntries * (uint64_t)(1 + 2 * W),
                             a.qcount + seg * kSegStride, a.err, sk, tk,
                             a.qkey ? a.qkey + seg * kSegEntries : nullptr);
#endif
        if (a.hsub_out) a.hsub[sk] = hch;  // the walk raises it to -ts if it stores P
    } else {
        a.table[sk] = -tk;
        if (a.hsub_out) a.hsub[sk] = fmaxf(-tk, hch);
    }
}

// Minimum waves per SIMD for the register allocator (the second argument of
// __launch_bounds__): the layer-6 two-pass launch without variable 0, the
// largest, at 7 (72 VGPRs; 82 had left 5 waves per SIMD): C3 188 -> 175 us,
// C5 1,405 -> 1,293 us (6: 178 / 1,302 us).  8 for every kernel (64 VGPRs)
// spilled more and slowed the phase-0 launch 210 -> 269 us.  The phase-0
// launch at 7 (72 VGPRs): 215 -> 208 us at C5; the layer-4 one-pass kernels
// at 8 (60 VGPRs, no spills): C5 81 -> 79 us.  The others keep their
// allocation.
#ifndef ULG_L6_REST_WAVES
#define ULG_L6_REST_WAVES 7
#endif
#ifndef ULG_L6_VAR0_WAVES
#define ULG_L6_VAR0_WAVES 7
#endif
#ifndef ULG_L4_WAVES
#define ULG_L4_WAVES 8
#endif
template <int L, int PHASE, int V>
constexpr int score_min_waves() {
    return (L == 6 && (V & 16) != 0) ? (PHASE == 1 ? ULG_L6_REST_WAVES : ULG_L6_VAR0_WAVES)
                                     : (L == 4 ? ULG_L4_WAVES : 1);
}
// PHASE 0: sets containing variable 0; 1: the rest.  V = variant bits (see
// ulg_set_option "score_variant"), compile-time so each form gets its own
// register allocation.
template <int L, int PHASE, int V>
__global__ void __launch_bounds__(kBlock, (score_min_waves<L, PHASE, V>())) score_layer_kernel(ScoreArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const LdsLayout lay = lds_layout(a.n, a.nv, a.S, L, V);
    double *g = reinterpret_cast<double *>(smem + lay.gram);
    uint32_t *binom = reinterpret_cast<uint32_t *>(smem + lay.binom);
    uint64_t *work = reinterpret_cast<uint64_t *>(smem + lay.work);
    uint64_t *toff = reinterpret_cast<uint64_t *>(smem + lay.toff);
    // the per-variable metadata and candidate lists too: every lane reads
    // them right after its variable is known, and from global memory those
    // would be two more dependent round trips per lane
    int *smeta = reinterpret_cast<int *>(smem + lay.meta);
    uint8_t *scand = reinterpret_cast<uint8_t *>(smem + lay.cand);
    for (int i = threadIdx.x; i < a.n * a.n; i += kBlock) g[i] = a.gram[i];
    for (int i = threadIdx.x; i < 64 * kBinomK; i += kBlock) binom[i] = a.binom[i];
    for (int i = threadIdx.x; i <= a.nv; i += kBlock) work[i] = a.work[i];
    for (int i = threadIdx.x; i <= a.nv * a.S; i += kBlock) toff[i] = a.tbl_off[i];
    for (int i = threadIdx.x; i < a.nv * 4; i += kBlock) smeta[i] = a.meta[i];
    for (int i = threadIdx.x; i < a.nv * 16; i += kBlock)
        reinterpret_cast<uint32_t *>(scand)[i] = reinterpret_cast<const uint32_t *>(a.cand)[i];
    __syncthreads();

    constexpr bool HM = (V & 64) != 0;           // subset maxima kept up to date
    constexpr bool CMP = HM && (V & 16) != 0;     // ... and the sets settled by them first
    const uint64_t gid0 = (uint64_t)xcd_block(blockIdx.x, gridDim.x, a.xcd) * kBlock + threadIdx.x;
    const bool valid = gid0 < work[a.nv];
    if (!CMP && !valid) return;
    // CMP: every lane reaches the block's barrier; a lane past the launch's
    // sets scores the last one again and writes nothing
    const uint64_t gid = valid ? gid0 : work[a.nv] - 1;
    int lo = 0, hi = a.nv;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (work[mid] <= gid) lo = mid; else hi = mid;
    }
    const int vi = lo;
    const uint64_t r = gid - work[vi];
    const SetHead<L> hd = set_head<L, PHASE>(smeta, scand, binom, vi, r);
    const bool z = hd.z;
    const uint64_t cm = hd.cm, rankP = hd.rankP;

#ifndef ULG_PROBE_NOSCORE  // ULG_PROBE_*: timing-only builds, see the two-pass section below
    const float ts = cbic_set_score<L>(g, a.n, hd.v, hd.gv, a.N, a.lambda);
#else
    const float ts = (float)(-a.N * g[hd.gv[0] * a.n + hd.gv[L - 1]] - (double)(r & 1023));
#endif

    if constexpr (CMP) {
        // 1. settle by the subset maxima: ts >= 0, no key >= -ts in U(P), or a
        //    present direct child >= -ts (always visited at the top level)
        const uint64_t vbase = (uint64_t)vi * a.S;
        const uint64_t slot = toff[vbase + L] + rankP;
        uint64_t rc[L], rz[L];
        child_ranks<L, PHASE == 1>(cm, binom, rc, rz);
        // every load of the settle issued at once (the children's maxima and
        // values, the var-0 toggles' maxima): one memory round trip instead
        // of up to three dependent ones
        float hch = absent_f();  // max over the proper nonempty subsets of P
        float hz = absent_f();   // ... and over the toggles P\a + {0}
        bool dh = false;         // a direct child >= -ts
#ifdef ULG_GATHER_STATS
        uint32_t hotA = 0u;      // children P\a_i holding a key >= -ts (hsub)
        uint32_t hotZ = 0u;      // toggled children P\a_i + {0} holding one
#endif
        {
            float ch[L], cv[L], zv[L];
            const uint32_t o1 = (uint32_t)toff[vbase + L - 1], o0 = (uint32_t)toff[vbase + L];
#pragma unroll
            for (int i = 0; i < L; ++i) {
                if constexpr (L > 1) {
                    ch[i] = a.hsub[o1 + (uint32_t)rc[i]];
                    cv[i] = a.table[o1 + (uint32_t)rc[i]];
                }
                if constexpr (PHASE == 1) zv[i] = a.hsub[(z ? o0 : 0u) + (z ? (uint32_t)rz[i] : 0u)];
            }
            const float thr = -ts;
#pragma unroll
            for (int i = 0; i < L; ++i) {
                if constexpr (L > 1) {
                    hch = fmaxf(hch, ch[i]);
                    dh |= cv[i] >= thr;
#ifdef ULG_GATHER_STATS
                    hotA |= (ch[i] >= thr) ? 1u << i : 0u;
#endif
                }
                if constexpr (PHASE == 1) {
                    hz = fmaxf(hz, zv[i]);
#ifdef ULG_GATHER_STATS
                    hotZ |= (zv[i] >= thr) ? 1u << i : 0u;
#endif
                }
            }
            if (!z) hz = absent_f();
#ifdef ULG_GATHER_STATS
            if (!z) hotZ = 0u;
#endif
        }
        bool need = false;
        float out;
        if (ts >= 0.0f) {
            const float s = -ts;
            out = (s < 0.0f) ? s : absent_f();
        } else {
            const float thr = -ts;
            const float hu = fmaxf(hch, hz);
            out = -ts;
            if (hu >= thr) {
                out = absent_f();
                need = !dh;
            }
        }
        if (valid && !need) {
            a.table[slot] = out;
            if (a.hsub_out) a.hsub[slot] = fmaxf(out, hch);
        }
// ULG_PROBE_*: timing-only builds (wrong lists, never shipped) that drop one
// part of the two-pass kernel (scripts/r5_kernel_ab.sh)
#ifdef ULG_PROBE_NOCMP  // the undecided sets are left undecided
        return;
#endif
        // 2. the rest of the block's sets, compacted in LDS, so the presence
        //    gathers (2^(L+1) reads each) run on dense waves
        unsigned int *cnt = reinterpret_cast<unsigned int *>(smem + lay.cmp);
        uint64_t *ecm = reinterpret_cast<uint64_t *>(smem + lay.cmp + 16);
        uint32_t *eslot = reinterpret_cast<uint32_t *>(ecm + kBlock);
        float *ets = reinterpret_cast<float *>(eslot + kBlock);
        float *ehch = ets + kBlock;
        int *evi = reinterpret_cast<int *>(ehch + kBlock);
        if (threadIdx.x == 0) {
            cnt[0] = 0u;
            cnt[1] = 0u;  // the second compaction's count (variant bit 7)
        }
        __syncthreads();
        if (valid && need) {
            const unsigned int k = atomicAdd(cnt, 1u);
            ecm[k] = cm;
            eslot[k] = (uint32_t)slot;
            ets[k] = ts;
            ehch[k] = hch;
#ifdef ULG_GATHER_STATS
            evi[k] = vi | (int)(hotA << 8) | (int)(hotZ << 16);
#else
            evi[k] = vi;
#endif
        }
        __syncthreads();
        constexpr int W = bits_words(L);
        using BS = std::conditional_t<(W >= 4), BitsLds<W>, Bits<W>>;
        constexpr bool CMP2 = (V & 128) != 0 && W < 4;
        if constexpr (!CMP2)
            if (threadIdx.x >= *cnt) return;
        const int k = threadIdx.x;
        const bool a1 = threadIdx.x < cnt[0];
        const uint64_t seg = walk_segment();
        // this lane's compacted set (the lanes past the count, variant bit 7
        // only, carry a dummy and gather nothing)
        const int vk = a1 ? evi[k] & 0xff : 0;
#ifdef ULG_GATHER_STATS
        const uint32_t hk = a1 ? (uint32_t)evi[k] >> 8 : 0u;  // hotA | hotZ << 8
#endif
        const bool zk = smeta[vk * 4 + 2] != 0;
        const float tk = a1 ? ets[k] : -1.0f;
        const uint64_t sk = a1 ? eslot[k] : 0u;
        const uint64_t cmk = a1 ? ecm[k] : 1ull;
        const float hk1 = a1 ? ehch[k] : absent_f();
        uint64_t *lds_bits = reinterpret_cast<uint64_t *>(smem + lay.bits) + threadIdx.x;
        const LocalSet<L> ls = local_set<L, PHASE>(cmk, zk);
        BS present = make_bits<BS>(lds_bits);
        BS hib = make_bits<BS>(lds_bits + (size_t)W * kBlock);
        present.clear();
        hib.clear();
        bool q = false;
        if (a1) {
            // the keys the two-level rules read first; the rest only for the
            // sets the rules leave to the walk (the subset maxima already
            // showed a key >= -ts is present, so the rules need no "any key"
            // test)
#ifndef ULG_PROBE_NOPART1
            gather_keys<L, PHASE, V, BS, LdPlain, 1>(present, hib, ls, -tk, binom, zk, a.table,
                                                    toff + (uint64_t)vk * a.S);
#endif
#ifndef ULG_PROBE_NORULES
            const bool dom = settle_rules<L, PHASE, BS, true>(present, hib, ls, q);
#else
            const bool dom = false;
            q = false;
#endif
#ifdef ULG_GATHER_STATS
            if constexpr (W < 4) {
                BS p2 = make_bits<BS>(lds_bits), h2 = make_bits<BS>(lds_bits);
                p2.clear();
                h2.clear();
                gather_keys<L, PHASE, V, BS, LdPlain, 0>(p2, h2, ls, -tk, binom, zk, a.table,
                                                        toff + (uint64_t)vk * a.S);
                gather_stats<L, PHASE>(p2, h2, hk & 0xffu, hk >> 8, zk, q);
            }
#endif
            if (!q) {
                const float o = dom ? absent_f() : -tk;
                a.table[sk] = o;
                if (a.hsub_out) a.hsub[sk] = fmaxf(o, hk1);
            }
        }
        if constexpr (CMP2) {
            // 3. the sets the rules leave to the walk (about a third of the
            //    compacted ones) compacted once more, with their gathered
            //    words, so the rest of the gathers, the walk closure and the
            //    queue run on dense waves: at ~30 % of the lanes every wave
            //    would still issue them
            uint64_t *c2w = reinterpret_cast<uint64_t *>(smem + lay.cmp2);  // [2W][kBlock]
            __syncthreads();  // every lane has read its first entry
            if (q) {
                const unsigned int k2 = atomicAdd(cnt + 1, 1u);
                ecm[k2] = cmk;
                eslot[k2] = (uint32_t)sk;
                ets[k2] = tk;
                ehch[k2] = hk1;
                evi[k2] = vk;
#pragma unroll
                for (int j = 0; j < W; ++j) {
                    c2w[j * kBlock + k2] = present.word(j);
                    c2w[(W + j) * kBlock + k2] = hib.word(j);
                }
            }
            __syncthreads();
            if (threadIdx.x >= cnt[1]) return;
            const int vq = evi[k];
            const bool zq = smeta[vq * 4 + 2] != 0;
            const float tq = ets[k];
            const uint64_t sq = eslot[k];
            const float hq = ehch[k];
            const LocalSet<L> lq = local_set<L, PHASE>(ecm[k], zq);
            BS pq = make_bits<BS>(lds_bits), hq_bits = make_bits<BS>(lds_bits);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                pq.w[j] = c2w[j * kBlock + k];
                hq_bits.w[j] = c2w[(W + j) * kBlock + k];
            }
            walk_or_store<L, PHASE, V, BS>(a, pq, hq_bits, lq, tq, binom, zq, toff + (uint64_t)vq * a.S, seg, sq, hq);
        } else {
            if (q)
                walk_or_store<L, PHASE, V, BS>(a, present, hib, ls, tk, binom, zk, toff + (uint64_t)vk * a.S, seg, sk,
                                               hk1);
        }
        return;
    }

    one_pass_set<L, PHASE, V>(a, smem, lay, binom, toff, vi, z, cm, rankP, ts);
}

// Layers 1..LF of every variable in ONE launch (option score_fused; the
// small layers' one-pass form, V = variant & 65).  Workgroup b takes variable
// b and runs (L, phase) in order, its kFusedThreads lanes taking the phase's
// sets kFusedThreads at a time, with a barrier between phases: a phase reads
// only its own variable's lower layers and, in phase 1, the same layer's
// var-0 sets, all written by this workgroup before the barrier
// (its waves share one CU, so the workgroup-scope fences of __syncthreads
// order the stores before the loads).  Replaces 2 LF dependent launches of
// a few waves each (layers 1-4 at C3: ~117 us whatever the variable count).
constexpr int kFusedThreads = 1024;
template <int L, int PHASE, int LF, int V>
__device__ __forceinline__ void fused_phase(const ScoreArgs &a, const uint64_t *work_all, unsigned char *smem,
                                            const LdsLayout &lay, const double *g, const uint32_t *binom,
                                            const uint64_t *toff, const int *smeta, const uint8_t *scand, int vi) {
    const uint64_t *w = work_all + ((uint64_t)L * 2 + PHASE) * (uint64_t)(a.nv + 1);
    const uint64_t cnt = w[vi + 1] - w[vi];
    ScoreArgs as = a;
    as.hsub_out = a.hsub_out || !(L == LF && PHASE == 1);
    for (uint64_t r = threadIdx.x; r < cnt; r += kFusedThreads) {
        const SetHead<L> hd = set_head<L, PHASE>(smeta, scand, binom, vi, r);
        const float ts = cbic_set_score<L>(g, a.n, hd.v, hd.gv, a.N, a.lambda);
        one_pass_set<L, PHASE, V>(as, smem, lay, binom, toff, vi, hd.z, hd.cm, hd.rankP, ts);
    }
    __syncthreads();
    if constexpr (PHASE == 0) fused_phase<L, 1, LF, V>(a, work_all, smem, lay, g, binom, toff, smeta, scand, vi);
    else if constexpr (L < LF) fused_phase<L + 1, 0, LF, V>(a, work_all, smem, lay, g, binom, toff, smeta, scand, vi);
}
// a.hsub_out: whether layer LF's phase 1 writes the subset maxima (read by a
// layer above LF); a.work unused (work_all: every (layer, phase) prefix)
template <int LF, int V>
__global__ void __launch_bounds__(kFusedThreads) score_small_kernel(ScoreArgs a, const uint64_t *work_all) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const LdsLayout lay = lds_layout(a.n, a.nv, a.S, LF, V);
    double *g = reinterpret_cast<double *>(smem + lay.gram);
    uint32_t *binom = reinterpret_cast<uint32_t *>(smem + lay.binom);
    uint64_t *toff = reinterpret_cast<uint64_t *>(smem + lay.toff);
    int *smeta = reinterpret_cast<int *>(smem + lay.meta);
    uint8_t *scand = reinterpret_cast<uint8_t *>(smem + lay.cand);
    for (int i = threadIdx.x; i < a.n * a.n; i += kFusedThreads) g[i] = a.gram[i];
    for (int i = threadIdx.x; i < 64 * kBinomK; i += kFusedThreads) binom[i] = a.binom[i];
    for (int i = threadIdx.x; i <= a.nv * a.S; i += kFusedThreads) toff[i] = a.tbl_off[i];
    for (int i = threadIdx.x; i < a.nv * 4; i += kFusedThreads) smeta[i] = a.meta[i];
    for (int i = threadIdx.x; i < a.nv * 16; i += kFusedThreads)
        reinterpret_cast<uint32_t *>(scand)[i] = reinterpret_cast<const uint32_t *>(a.cand)[i];
    __syncthreads();
    fused_phase<1, 0, LF, V>(a, work_all, smem, lay, g, binom, toff, smeta, scand, (int)blockIdx.x);
}

// Second half of a queued layer (variant bit 4): one wave (64 threads) per
// 64*K queued sets.  Entry: table slot (low 32 bits) | ts bits (high 32), W
// `hi` words, W open words (queue_walk).  walk_load gathers this lane's K
// entries into the bit-sliced hi / open vectors (register r, field f <-
// subset r*E + f, bit k of a field <- set k) and returns the alive mask.
template <int L, int K>
__device__ __forceinline__ uint32_t walk_load(const uint64_t *queue, uint64_t qn, uint64_t mine,
                                              typename Sliced<L, K>::Vec &hiV, typename Sliced<L, K>::Vec &openV) {
    using S = Sliced<L, K>;
    constexpr int W = bits_words(L);
#pragma unroll
    for (int r = 0; r < S::NV; ++r) {
        hiV[r] = 0u;
        openV[r] = 0u;
    }
    uint32_t alive = 0u;
#pragma nounroll
    for (int k = 0; k < S::K; ++k) {
        if (mine + k >= qn) break;
        alive |= 1u << k;
        const uint64_t *e = queue + (mine + k) * (uint64_t)(1 + 2 * W);
        uint64_t hw[W], ow[W];
#pragma unroll
        for (int wj = 0; wj < W; ++wj) {
            hw[wj] = e[1 + wj];
            ow[wj] = e[1 + W + wj];
        }
        // transpose: register r, field f <- subset r*E + f of set k
#pragma unroll
        for (int r = 0; r < S::NV0; ++r) {
            const int t0 = r * S::E;
            constexpr uint32_t EM = (uint32_t)((1ull << S::E) - 1ull);
            const uint32_t hb = (uint32_t)(hw[t0 >> 6] >> (t0 & 63)) & EM;
            const uint32_t ob = (uint32_t)(ow[t0 >> 6] >> (t0 & 63)) & EM;
            uint32_t hs, os;
            if constexpr (S::K == 8) {
                // 4 bits -> bytes 0..3 (non-overlapping partial products)
                hs = (hb * 0x00204081u) & 0x01010101u;
                os = (ob * 0x00204081u) & 0x01010101u;
            } else {
                hs = os = 0u;
#pragma unroll
                for (int f = 0; f < S::E; ++f) {
                    hs |= ((hb >> f) & 1u) << (S::K * f);
                    os |= ((ob >> f) & 1u) << (S::K * f);
                }
            }
            hiV[r] |= hs << k;
            openV[r] |= os << k;
        }
    }
    return alive;
}

// The decisions of this lane's sets: pruned (absent) or stored (-ts), and the
// subset maxima raised to -ts when stored (variant bit 6).
template <int K>
__device__ __forceinline__ void walk_store(const uint64_t *queue, uint64_t qn, uint64_t mine, int W, uint32_t dom,
                                           float *table, float *hsub, uint64_t nslots, unsigned long long *err) {
#pragma nounroll
    for (int k = 0; k < K; ++k) {
        if (mine + k >= qn) break;
        const uint64_t e0 = queue[(mine + k) * (uint64_t)(1 + 2 * W)];
        const float ts = __uint_as_float((uint32_t)(e0 >> 32));
        const bool d = (dom >> k) & 1u;
        if ((uint32_t)e0 >= nslots) {  // an entry no scoring lane wrote
            atomicOr(err, kErrSlot);
            continue;
        }
        table[(uint32_t)e0] = d ? absent_f() : -ts;
        if (hsub && !d) hsub[(uint32_t)e0] = fmaxf(hsub[(uint32_t)e0], -ts);
    }
}

// One wave per (queue segment, chunk of 64 * K entries), chunk-major:
// blockIdx.x = chunk * nseg + segment, so the few chunks that hold sets come
// first in dispatch order and the empty ones (a segment can hold up to
// kSegEntries sets) form the tail -- interleaved, the empty workgroups' own
// dispatch delayed the last busy waves (the layer-6 walk's span 220 -> 427 us).
template <int L, int PHASE, int K>
__global__ void __launch_bounds__(64) walk_sliced_kernel(const uint64_t *queue, const unsigned long long *qcount,
                                                         float *table, float *hsub, uint64_t *wclock, uint64_t nslots,
                                                         unsigned long long *err) {
    using S = Sliced<L, K>;
    const uint64_t t_start = wclock ? wall_clock64() : 0;
    constexpr int W = bits_words(L);
    constexpr uint32_t kChunks = (uint32_t)((kSegEntries + 64 * K - 1) / (64 * K));
    const uint32_t nseg = gridDim.x / kChunks;
    const uint32_t seg = blockIdx.x % nseg;
    const uint64_t qc = qcount[(uint64_t)seg * kSegStride];
    const uint64_t qn = qc < kSegEntries ? qc : kSegEntries;  // past it: kErrQueue is set
    const uint64_t first = (uint64_t)(blockIdx.x / nseg) * 64 * S::K;
    if (first >= qn) return;
    queue += (uint64_t)seg * kSegEntries * (uint64_t)(1 + 2 * W);
    const uint64_t mine = first + (uint64_t)threadIdx.x * S::K;
    typename S::Vec hiV, openV;
    uint32_t alive = walk_load<L, K>(queue, qn, mine, hiV, openV);
    constexpr bool v0inP = PHASE == 0;
    constexpr uint32_t Plocal = v0inP ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    uint32_t pvtop = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) pvtop |= (uint32_t)(i + (v0inP ? 0 : 1)) << (4 * i);
    uint32_t dom = 0u, pts = 0u;
    // the open bits in LDS (OpenLds): no vector copies per recursion level
    __shared__ uint32_t open_lds[2 * S::NV * 64];
    OpenLds<L, K> ol{open_lds + threadIdx.x};
#pragma unroll
    for (int r = 0; r < S::NV; ++r) {
        ol.base[r * 64] = openV[r];
        ol.base[r * 64 + S::NV * 64] = hiV[r];
    }
    if (wclock) walk_sliced<L, K, L, true, OpenLds<L, K>, PHASE>(Plocal, pvtop, alive, hiV, ol, alive, dom, pts);
    else walk_sliced<L, K, L, false, OpenLds<L, K>, PHASE>(Plocal, pvtop, alive, hiV, ol, alive, dom, pts);
#ifdef ULG_GATHER_STATS
    if (alive) atomicAdd(&g_wstats[(L * 2 + PHASE) * 16 + 15], (unsigned long long)__builtin_popcount(alive));
#endif
    if (wclock && threadIdx.x == 0) {
        // diagnostics (ULG_WALK_CLOCK): start, end, union points of this wave
        wclock[3 * blockIdx.x] = t_start;
        wclock[3 * blockIdx.x + 1] = wall_clock64();
        wclock[3 * blockIdx.x + 2] = pts;
    }
    walk_store<S::K>(queue, qn, mine, W, dom, table, hsub, nslots, err);
}

// ---- bucketed walk launches (round 6, option walk_bucket) --------------------
// A layer-5/6 launch's queued sets walked in the order of their walk key
// (walk_key): a counting sort over (key, segment) -- the scoring kernel
// writes each set's key, walk_bucket_count_kernel ranks the sets of each
// segment by key and, in its last block, lays out the keys and a table of walk
// waves, walk_bucket_scatter_kernel writes each set's queue index at its place -- and
// walk_bucket_kernel walks the table.  The sets whose every first-level node
// is open hold the longest, least alike walks: split 64 ways by six
// second-level nodes (keys 64..127), they come first in the table, 64 sets per
// wave (one per lane); every other key 64 x K per wave.  At C3's layer 6
// without variable 0 the longest wave's union walk drops from 811 to ~465
// points and the launch's union points from 311 K to ~100 K
// (scripts/walk_sched_study.cpp on the dumped queues).  Same walks, same
// decisions: only which sets share a wave changes.
constexpr int kBucketMax = 128;  // walk keys: 64 first-level patterns, the all-open one split 64 ways


// One block per kBucketSegs segments: the segments' key histogram in LDS
// (16 keys per 16-byte load), each entry's rank among the block's sets of its
// key (qaux = key << 24 | rank), and one global atomic per key for the
// block's base within the key (kbase; few blocks, so few atomics per address
// -- one block per segment serialised ~300-2300 atomics on each key's total).
// The key totals then give every key's sorted start and the list of walk
// waves (bucket_lanes), recomputed by each later kernel instead of a table.
#ifndef ULG_BUCKET_SEGS
#define ULG_BUCKET_SEGS 8
#endif
constexpr int kBucketSegs = ULG_BUCKET_SEGS;
__global__ void __launch_bounds__(256) walk_bucket_count_kernel(const unsigned long long *qseg, uint32_t nseg,
                                                                int L, const uint8_t *qkey, uint32_t *qaux,
                                                                uint32_t *kbase) {
    __shared__ unsigned int lh[kBucketMax];
    __shared__ unsigned int cst[kBucketSegs + 1];
    __shared__ unsigned int qnl[kBucketSegs];
    const uint32_t seg0 = blockIdx.x * kBucketSegs;
    const uint32_t nsb = nseg - seg0 < (uint32_t)kBucketSegs ? nseg - seg0 : (uint32_t)kBucketSegs;
    unsigned int *hdr = reinterpret_cast<unsigned int *>(const_cast<unsigned long long *>(qseg) + (uint64_t)nseg * kSegStride);
    if (threadIdx.x < kBucketMax) lh[threadIdx.x] = 0u;
    if (threadIdx.x < 64) {
        // the block's segments: their set counts and 16-entry chunk offsets
        const int lane = threadIdx.x;
        unsigned int qn = 0;
        if ((uint32_t)lane < nsb) {
            const uint64_t qc = qseg[(uint64_t)(seg0 + lane) * kSegStride];
            qn = (unsigned int)(qc < kSegEntries ? qc : kSegEntries);
            qnl[lane] = qn;
        }
        const unsigned int ch = (qn + 15u) >> 4;
        unsigned int incl = ch;
#pragma unroll
        for (int o = 1; o < kBucketSegs; o <<= 1) {
            const unsigned int t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        if (lane < kBucketSegs) cst[lane + 1] = incl;
        if (lane == 0) cst[0] = 0u;
    }
    __syncthreads();
    const unsigned int items = cst[nsb];
    for (unsigned int it = threadIdx.x; it < items; it += 256) {
        uint32_t s = 0;
        while (s + 1 < nsb && cst[s + 1] <= it) ++s;
        const uint32_t c = it - cst[s];
        const uint64_t base = (uint64_t)(seg0 + s) * kSegEntries + (uint64_t)c * 16;
        const unsigned int n = qnl[s] - c * 16 < 16u ? qnl[s] - c * 16 : 16u;
        const uint4 k4 = *reinterpret_cast<const uint4 *>(qkey + base);
        const uint32_t kw[4] = {k4.x, k4.y, k4.z, k4.w};
#pragma unroll
        for (unsigned int j = 0; j < 16; ++j) {
            if (j >= n) break;
            const uint32_t key = (kw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t r = atomicAdd(&lh[key], 1u);
            qaux[base + j] = (key << 24) | r;
        }
    }
    __syncthreads();
    if (threadIdx.x < kBucketMax) {
        const unsigned int c = lh[threadIdx.x];
        kbase[(uint64_t)blockIdx.x * kBucketMax + threadIdx.x] = c ? atomicAdd(hdr + 64 + threadIdx.x, c) : 0u;
    }
    (void)L;
}

// The keys in walk order as one wave's lanes, two per lane: order kk = 2 lane
// + h (h = 0, 1); orders 0..63 are the all-open sub-keys 64..127 (64 sets
// per wave, one per lane), orders 64..127 the other first-level patterns
// 0..63 (per_light sets per wave).  Per half: the key's set count, its first
// sorted position and its wave range [wbeg, wend) in the launch's wave list.
struct BucketLanes {
    unsigned int tot[2], st[2], wbeg[2], wend[2], pk[2];
};
__device__ __forceinline__ uint32_t bucket_key(uint32_t kk) { return kk < 64 ? 64u + kk : kk - 64u; }
__device__ __forceinline__ BucketLanes bucket_lanes(const unsigned int *hdr, uint32_t per_light) {
    const int lane = threadIdx.x & 63;
    BucketLanes b;
    unsigned int nw[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t kk = 2u * (uint32_t)lane + (uint32_t)h;
        b.tot[h] = hdr[64 + bucket_key(kk)];
        b.pk[h] = kk < 64 ? 64u : per_light;
        nw[h] = (b.tot[h] + b.pk[h] - 1) / b.pk[h];
    }
    const unsigned int t2 = b.tot[0] + b.tot[1], w2 = nw[0] + nw[1];
    unsigned int st = t2, wi = w2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned int t = __shfl_up(st, o), u = __shfl_up(wi, o);
        if (lane >= o) {
            st += t;
            wi += u;
        }
    }
    b.st[0] = st - t2;
    b.st[1] = b.st[0] + b.tot[0];
    b.wbeg[0] = wi - w2;
    b.wend[0] = b.wbeg[0] + nw[0];
    b.wbeg[1] = b.wend[0];
    b.wend[1] = wi;
    return b;
}

// Every queued set's queue index at its sorted position: key start + the
// segment's base in the key + the set's rank (256-entry chunks of each
// segment, chunk-major, grid-stride).
__global__ void __launch_bounds__(256) walk_bucket_scatter_kernel(const unsigned long long *qseg,
                                                                  const uint32_t *qaux, const uint32_t *kbase,
                                                                  uint32_t nseg, int L, uint32_t *sidx) {
    const unsigned int *hdr =
        reinterpret_cast<const unsigned int *>(qseg + (uint64_t)nseg * kSegStride);
    __shared__ unsigned int kst[kBucketMax];
    if (threadIdx.x < 64) {
        const BucketLanes b = bucket_lanes(hdr, 64u);
        kst[bucket_key(2 * threadIdx.x)] = b.st[0];
        kst[bucket_key(2 * threadIdx.x + 1)] = b.st[1];
    }
    __syncthreads();
    (void)L;
    const uint64_t items = (uint64_t)nseg * (kSegEntries / 256);
    for (uint64_t item = blockIdx.x; item < items; item += gridDim.x) {
        const uint32_t seg = (uint32_t)(item % nseg);
        const uint64_t e = (item / nseg) * 256 + threadIdx.x;
        const uint64_t qc = qseg[(uint64_t)seg * kSegStride];
        const uint64_t qn = qc < kSegEntries ? qc : kSegEntries;
        if ((item / nseg) * 256 >= qn) continue;
        if (e >= qn) continue;
        const uint32_t ax = qaux[(uint64_t)seg * kSegEntries + e];
        const uint32_t key = ax >> 24, r = ax & 0xFFFFFFu;
        const uint32_t pos = kst[key] + kbase[(uint64_t)(seg / kBucketSegs) * kBucketMax + key] + r;
        sidx[pos] = (uint32_t)((uint64_t)seg * kSegEntries + e);
    }
}

// walk_load / walk_sliced / walk_store over the sorted index: wave w of the
// table walks its sets K per lane.
template <int L, int PHASE, int K, int NVMAX>
__device__ __forceinline__ void walk_group(const uint64_t *queue, const uint32_t *sidx, uint32_t st, uint32_t cnt,
                                           uint32_t *open_lds, float *table, float *hsub, uint64_t nslots,
                                           unsigned long long *err) {
    using S = Sliced<L, K>;
    static_assert(S::NV <= NVMAX, "open bits LDS");
    constexpr int W = bits_words(L);
    const uint32_t lane = threadIdx.x;
    typename S::Vec hiV, openV;
#pragma unroll
    for (int r = 0; r < S::NV; ++r) {
        hiV[r] = 0u;
        openV[r] = 0u;
    }
    uint32_t alive = 0u;
    uint32_t ent[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t p = lane * K + k;
        ent[k] = p < cnt ? sidx[st + p] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (ent[k] == 0xFFFFFFFFu) continue;
        alive |= 1u << k;
        const uint64_t *e = queue + (uint64_t)ent[k] * (1 + 2 * W);
        uint64_t hw[W], ow[W];
#pragma unroll
        for (int wj = 0; wj < W; ++wj) {
            hw[wj] = e[1 + wj];
            ow[wj] = e[1 + W + wj];
        }
#pragma unroll
        for (int r = 0; r < S::NV0; ++r) {
            const int t0 = r * S::E;
            constexpr uint32_t EM = (uint32_t)((1ull << S::E) - 1ull);
            const uint32_t hb = (uint32_t)(hw[t0 >> 6] >> (t0 & 63)) & EM;
            const uint32_t ob = (uint32_t)(ow[t0 >> 6] >> (t0 & 63)) & EM;
            uint32_t hs = 0u, os = 0u;
            if constexpr (S::K == 8) {
                hs = (hb * 0x00204081u) & 0x01010101u;
                os = (ob * 0x00204081u) & 0x01010101u;
            } else if constexpr (S::K == 1) {
                hs = hb;
                os = ob;
            } else {
#pragma unroll
                for (int f = 0; f < S::E; ++f) {
                    hs |= ((hb >> f) & 1u) << (S::K * f);
                    os |= ((ob >> f) & 1u) << (S::K * f);
                }
            }
            hiV[r] |= hs << k;
            openV[r] |= os << k;
        }
    }
    constexpr bool v0inP = PHASE == 0;
    constexpr uint32_t Plocal = v0inP ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    uint32_t pvtop = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) pvtop |= (uint32_t)(i + (v0inP ? 0 : 1)) << (4 * i);
    uint32_t dom = 0u, pts = 0u;
    OpenLds<L, K, NVMAX * 64> ol{open_lds + lane};
#pragma unroll
    for (int r = 0; r < S::NV; ++r) {
        ol.base[r * 64] = openV[r];
        ol.base[r * 64 + NVMAX * 64] = hiV[r];
    }
    walk_sliced<L, K, L, false, OpenLds<L, K, NVMAX * 64>, PHASE>(Plocal, pvtop, alive, hiV, ol, alive, dom, pts);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (ent[k] == 0xFFFFFFFFu) continue;
        const uint64_t e0 = queue[(uint64_t)ent[k] * (1 + 2 * W)];
        const float ts = __uint_as_float((uint32_t)(e0 >> 32));
        const bool d = (dom >> k) & 1u;
        const uint32_t slot = (uint32_t)e0;
        if (slot >= nslots) {
            atomicOr(err, kErrSlot);
            continue;
        }
        table[slot] = d ? absent_f() : -ts;
        if (hsub && !d) hsub[slot] = fmaxf(hsub[slot], -ts);
    }
}

// hdr: the launch's bucket header (key totals); waves in key order, the
// all-open key's first (bucket_lanes), a grid-stride loop over them.
template <int L, int PHASE, int KL>
__global__ void __launch_bounds__(64) walk_bucket_kernel(const uint64_t *queue, const uint32_t *sidx,
                                                         const unsigned int *hdr, float *table, float *hsub,
                                                         uint64_t nslots, unsigned long long *err) {
    constexpr int NVMAX = Sliced<L, KL>::NV > Sliced<L, 1>::NV ? Sliced<L, KL>::NV : Sliced<L, 1>::NV;
    __shared__ uint32_t open_lds[2 * NVMAX * 64];  // open bits, then the hi copy
    const BucketLanes b = bucket_lanes(hdr, 64u * KL);
    const uint32_t nw = __shfl(b.wend[1], 63);
    for (uint32_t w = blockIdx.x; w < nw; w += gridDim.x) {
        // the lane holding wave w: the first whose range ends past w; then its half
        const unsigned long long past = __ballot(b.wend[1] > w);
        const int ln = __ffsll((long long)past) - 1;
        const bool h1 = __shfl(b.wend[0], ln) <= w;
        const uint32_t wbeg = h1 ? __shfl(b.wbeg[1], ln) : __shfl(b.wbeg[0], ln);
        const uint32_t st = h1 ? __shfl(b.st[1], ln) : __shfl(b.st[0], ln);
        const uint32_t tot = h1 ? __shfl(b.tot[1], ln) : __shfl(b.tot[0], ln);
        const uint32_t pk = h1 ? __shfl(b.pk[1], ln) : __shfl(b.pk[0], ln);
        const uint32_t kk = 2u * (uint32_t)ln + (h1 ? 1u : 0u);
        const uint32_t off = (w - wbeg) * pk;
        const uint32_t cw = tot - off < pk ? tot - off : pk;
        if (kk < 64)
            walk_group<L, PHASE, 1, NVMAX>(queue, sidx, st + off, cw, open_lds, table, hsub, nslots, err);
        else
            walk_group<L, PHASE, KL, NVMAX>(queue, sidx, st + off, cw, open_lds, table, hsub, nslots, err);
    }
}

// ---- wide layers (kMaxL < L <= kWideMax) ------------------------------------
// The reference's default parent limit is n - 1 (score_main.cpp:296-298), so on
// small n (data/hepatitis.clean.csv: n = 20) the layers run to 19 parents.
// Those layers use runtime-L kernels: the same Cholesky-of-the-Gram score per
// lane (the triangle in private memory), the direct-children decision in the
// scoring kernel (a present child P\{a} >= -ts is always visited at the top
// level: present keys never enter `checked`), and, for the rest, an explicit
// stack replay of find_best_subset_score (BIC_OLS.cpp:125-172)
// whose `checked` set is a 2^q-bit bitset per walking set in HBM (q local
// bits: P, plus variable 0 when P lacks it).
constexpr uint64_t kWideStepCap = 1ull << 30;  // per-set walk steps before the call fails loudly
constexpr uint64_t kWideBitsWords = 1ull << 27;  // checked bitsets, all stream groups together (1 GiB)

__device__ __forceinline__ uint64_t B64(const uint64_t *b, int a, int k) { return b[a * 64 + k]; }

__device__ __forceinline__ uint64_t unrank_colex64(uint64_t r, int l, int U, const uint64_t *b) {
    uint64_t mask = 0;
    int c = U - 1;
    for (int i = l; i >= 1; --i) {
        while (c >= 0 && B64(b, c, i) > r) --c;
        mask |= 1ull << c;
        r -= B64(b, c, i);
        --c;
    }
    return mask;
}

__device__ __forceinline__ uint64_t rank_colex64(uint64_t mask, const uint64_t *b) {
    uint64_t r = 0;
    int j = 0;
    while (mask) {
        const int x = __builtin_ctzll(mask);
        mask &= mask - 1;
        ++j;
        r += B64(b, x, j);
    }
    return r;
}

struct WideArgs {
    const double *gram;       // n x n row-major
    const uint64_t *binom;    // [64][64]
    const uint8_t *cand;      // [nv][64]
    const int *meta;          // [nv][4]
    const uint64_t *tbl_off;  // [nv*S + 1]
    const uint64_t *work;     // [nv + 1] prefix of this launch's sets
    float *table;
    uint64_t *queue;          // 3 words per undecided set: slot, compact mask, vi | ts bits << 32
    unsigned long long *qcount;
    const float *hmax;        // hi-cover tables (hikey_*_kernel) or null
    const float *pval;        // the same variables' present keys by compact mask (absent bits otherwise)
    const uint64_t *hoff;     // [nv] offset of a variable's tables in hmax / pval, ~0 = none
    int reduced;              // walk_wide_kernel: skip the reference's no-op re-tests
    double N;
    double lambda;
    int n, nv, S, L;
};

template <int LMAX, int PHASE>
__global__ void __launch_bounds__(kBlock) score_wide_kernel(WideArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *g = reinterpret_cast<double *>(smem);
    for (int i = threadIdx.x; i < a.n * a.n; i += kBlock) g[i] = a.gram[i];
    __syncthreads();
    const uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (gid >= a.work[a.nv]) return;
    int lo = 0, hi = a.nv;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a.work[mid] <= gid) lo = mid; else hi = mid;
    }
    const int vi = lo;
    const int v = a.meta[vi * 4 + 0];
    const int m = a.meta[vi * 4 + 1];
    const bool z = a.meta[vi * 4 + 2] != 0;
    const int L = a.L;
    const uint64_t r = gid - a.work[vi];
    uint64_t cm;
    if (PHASE == 0) cm = (unrank_colex64(r, L - 1, m - 1, a.binom) << 1) | 1ull;
    else if (z) cm = unrank_colex64(r, L, m - 1, a.binom) << 1;
    else cm = unrank_colex64(r, L, m, a.binom);
    const uint64_t slot = a.tbl_off[(uint64_t)vi * a.S + L] + rank_colex64(cm, a.binom);

    int gv[LMAX];
    {
        uint64_t rem = cm;
        for (int i = 0; i < L; ++i) {
            gv[i] = a.cand[vi * 64 + __builtin_ctzll(rem)];
            rem &= rem - 1;
        }
    }
    // Cholesky of G[P,P] (packed rows, row i at i(i+1)/2), y = L^-1 G[P,v]:
    // the unrolled kernels' operation order
    double Lm[LMAX * (LMAX + 1) / 2];
    double y[LMAX];
    const int n = a.n;
    for (int i = 0; i < L; ++i) {
        for (int j = 0; j <= i; ++j) Lm[i * (i + 1) / 2 + j] = g[gv[i] * n + gv[j]];
        y[i] = g[gv[i] * n + v];
    }
    const double cvv = g[v * n + v];
    for (int j = 0; j < L; ++j) {
        const int rj = j * (j + 1) / 2;
        double s = Lm[rj + j];
        for (int k = 0; k < j; ++k) s -= Lm[rj + k] * Lm[rj + k];
        const double d = sqrt(s);
        Lm[rj + j] = d;
        const double inv = 1.0 / d;
        for (int i = j + 1; i < L; ++i) {
            const int ri = i * (i + 1) / 2;
            double t = Lm[ri + j];
            for (int k = 0; k < j; ++k) t -= Lm[ri + k] * Lm[rj + k];
            Lm[ri + j] = t * inv;
        }
    }
    double yy = 0.0;
    for (int i = 0; i < L; ++i) {
        const int ri = i * (i + 1) / 2;
        double t = y[i];
        for (int k = 0; k < i; ++k) t -= Lm[ri + k] * y[k];
        t = t / Lm[ri + i];
        y[i] = t;
        yy += t * t;
    }
    const double rss = cvv - yy;
    // BIC_OLS.cpp:366
    const double the_score = a.N * log(rss / a.N) + a.lambda * log(a.N) * (double)L - 0.0;
    const float ts = (float)the_score;
    if (ts >= 0.0f) {
        const float s = -ts;  // stored by the caller iff < 0 (score_calculator.cpp:111)
        a.table[slot] = (s < 0.0f) ? s : absent_f();
        return;
    }
    const float thr = -ts;
    const uint64_t coff = a.tbl_off[(uint64_t)vi * a.S + L - 1];
    bool dom = false;
    {
        uint64_t rem = cm;
        while (rem) {
            const uint64_t bit = rem & (0 - rem);
            rem ^= bit;
            dom |= a.table[coff + rank_colex64(cm ^ bit, a.binom)] >= thr;  // absent (NaN) never >= thr
        }
    }
    if (dom) {
        a.table[slot] = absent_f();
        return;
    }
    const unsigned long long act = __ballot(1);
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)act) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(a.qcount, (unsigned long long)__popcll(act));
    base = __shfl(base, leader);
    const uint64_t pos = base + (uint64_t)__popcll(act & ((1ull << lane) - 1ull));
    uint64_t *e = a.queue + 3 * pos;
    e[0] = slot;
    e[1] = cm;
    e[2] = (uint64_t)(uint32_t)vi | ((uint64_t)fbits(ts) << 32);
}

// One lane per queued set: find_best_subset_score replayed step by step.  A
// frame at depth d holds T, the parent vector (L - d entries; entries past the
// filled ones are 0 = variable 0), the outer index idx, and while a
// child list is being built the inner position i, the fill j and u.  The walk
// stops at the first visited key >= -ts: that alone decides the store rule
// (BIC_OLS.cpp:234 with best starting at 0 < -ts).
template <int LMAX, int PHASE>
__global__ void __launch_bounds__(64) walk_wide_kernel(WideArgs a, uint64_t qbase, uint64_t qn, uint64_t *bits,
                                                       uint64_t wpl, unsigned long long *err,
                                                       unsigned long long *wstats, uint64_t budget,
                                                       uint64_t *squeue, unsigned long long *scount) {
    const uint64_t lid = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const uint64_t qi = qbase + lid;
    if (qi >= qn) return;
    const uint64_t *e = a.queue + 3 * qi;
    const uint64_t slot = e[0], cm = e[1];
    const int vi = (int)(uint32_t)e[2];
    const float ts = __uint_as_float((uint32_t)(e[2] >> 32));
    const int L = a.L;
    const bool z = a.meta[vi * 4 + 2] != 0;
    uint8_t lc[LMAX + 1];  // local bit -> compact index
    uint64_t Plocal;
    {
        uint64_t rem = cm;
        const int first = PHASE == 0 ? 0 : 1;
        lc[0] = 0;
        for (int i = first; i < L + first; ++i) {
            lc[i] = (uint8_t)__builtin_ctzll(rem);
            rem &= rem - 1;
        }
        Plocal = PHASE == 0 ? ((1ull << L) - 1ull) : (((1ull << L) - 1ull) << 1);
    }
    const uint64_t *toffv = a.tbl_off + (uint64_t)vi * a.S;
    const float thr = -ts;
    // Hi-cover prune: the walk's answer is only whether it visits a present key
    // >= -ts (a "hi" key).  From a node T it can only visit subsets of T and
    // variable 0 (U(T)), so an absent T whose U(T) holds no hi key is not
    // expanded (marked checked, as its call would have been).  Expanding it
    // could only change `checked` inside U(T), and every later difference
    // stays inside U(T) (U is monotone), so the first hi key visited -- the
    // decision -- is unchanged.  hmax[X] = max over the keys present when
    // this phase runs of the subsets of the compact mask X.
    // With the tables, a node also carries its compact mask Tc (variable 0 is
    // compact bit 0 when it is a candidate), and the presence test is one read
    // of pval[Tc] instead of a colex rank over the node's bits.
    const uint64_t ho = a.hoff ? a.hoff[vi] : ~0ull;
    const bool dense = ho != ~0ull;
    const uint64_t zb = z ? 1ull : 0ull;
    auto cbit = [&](int u) -> uint64_t { return u == 0 ? zb : (1ull << lc[u]); };
    auto hi_in_cover = [&](uint64_t Tc) -> bool { return !dense || a.hmax[ho + (Tc | zb)] >= thr; };
    if (!hi_in_cover(cm)) {  // no hi key below P at all: stored
        a.table[slot] = -ts;
        return;
    }
    uint64_t *chk = bits + lid * wpl;
    chk[0] |= 1ull;  // checked.insert(empty_set)

    // Re-test skipping (a.reduced): the inner loop calls fb(T2, npv) once per
    // appended entry, with npv = the first j appended entries + zero padding.
    // In call j >= 2 the positions below j-1 were tested by the earlier calls
    // (each is now checked, or a present key below -ts: testing it again
    // changes nothing) and the positions from j on are zeros, whose child
    // T2 ^ {0} call 1 already tested at its position 1.  So call 1 tests
    // positions 0 and 1 and call j >= 2 only position j-1: the same tests in
    // the same order, minus the no-ops (O(m) instead of O(m^2) per expanded
    // node).  ends[d] is where the current call at depth d stops.
    uint64_t Ts[LMAX + 1], Tcs[LMAX + 1];
    uint8_t idxs[LMAX + 1], is[LMAX + 1], js[LMAX + 1], us[LMAX + 1], inner[LMAX + 1], ends[LMAX + 1];
    uint8_t pvs[LMAX * (LMAX + 1) / 2 + 1];
    for (int i = 0; i < L; ++i) pvs[i] = (uint8_t)(i + (PHASE == 0 ? 0 : 1));
    int d = 0;
    Ts[0] = Plocal;
    Tcs[0] = cm;
    idxs[0] = 0;
    ends[0] = (uint8_t)L;
    inner[0] = 0;
    bool dom = false;
    uint64_t steps = 0;
    while (true) {
        if (++steps > kWideStepCap) {
            atomicOr(err, 1ull);
            break;
        }
        if (budget && steps > budget && dense) {
            // a long walk: hand it to walk_wide_lds_kernel, which replays it
            // from the start with every bitset in LDS (same walk)
            const unsigned long long pos = atomicAdd(scount, 1ull);
            squeue[3 * pos] = e[0];
            squeue[3 * pos + 1] = e[1];
            squeue[3 * pos + 2] = e[2];
            return;
        }
        const int mm = L - d;
        const int po = d * L - d * (d - 1) / 2;  // pvs offset of depth d
        if (!inner[d]) {
            if (idxs[d] == ends[d]) {  // fb returns
                if (d == 0) break;
                --d;
                const uint64_t c = Ts[d + 1];
                chk[c >> 6] |= 1ull << (c & 63);  // checked.insert(thin_parents) after the call
                continue;
            }
            const uint8_t u = pvs[po + idxs[d]];
            const uint64_t T2 = Ts[d] ^ (1ull << u);
            if ((chk[T2 >> 6] >> (T2 & 63)) & 1ull) {
                ++idxs[d];
                continue;
            }
            const uint64_t T2c = Tcs[d] ^ cbit(u);
            // is T2 in the cache as it stood when P was scored?
            bool present = false;
            const int pc = __popcll(T2);
            if (dense) {
                // pval holds exactly the keys of that cache (hikey_tile_kernel);
                // variable 0 outside the candidates is never a key's member
                if (!(PHASE == 1 && (T2 & 1ull) && !z)) {
                    const float val = a.pval[ho + T2c];
                    if (fbits(val) != kAbsentBits) {
                        present = true;
                        if (val >= thr) {
                            dom = true;
                            break;
                        }
                    }
                }
            } else if (pc < L || (PHASE == 1 && pc == L && (T2 & 1ull))) {
                if (!(PHASE == 1 && (T2 & 1ull) && !z)) {
                    uint64_t rk = 0, rem = T2;
                    int j = 0;
                    while (rem) {
                        const int lb = __builtin_ctzll(rem);
                        rem &= rem - 1;
                        ++j;
                        rk += B64(a.binom, lc[lb], j);
                    }
                    const float val = a.table[toffv[pc] + rk];
                    if (fbits(val) != kAbsentBits) {
                        present = true;
                        if (val >= thr) {
                            dom = true;
                            break;
                        }
                    }
                }
            }
            if (present) {
                ++idxs[d];
                continue;
            }
            if (!hi_in_cover(T2c)) {
                chk[T2 >> 6] |= 1ull << (T2 & 63);
                ++idxs[d];
                continue;
            }
            inner[d] = 1;
            is[d] = 0;
            js[d] = 0;
            us[d] = u;
            for (int k = 0; k < mm - 1; ++k) pvs[po + mm + k] = 0;
            continue;
        }
        if (is[d] == mm) {
            inner[d] = 0;
            ++idxs[d];
            continue;
        }
        const uint8_t pi = pvs[po + is[d]];
        ++is[d];
        if (pi == us[d]) continue;
        pvs[po + mm + js[d]] = pi;
        ++js[d];
        Ts[d + 1] = Ts[d] ^ (1ull << us[d]);
        Tcs[d + 1] = Tcs[d] ^ cbit(us[d]);
        if (a.reduced) {
            const int j = js[d];  // this is call j of fb(T2, npv)
            idxs[d + 1] = (uint8_t)(j == 1 ? 0 : j - 1);
            ends[d + 1] = (uint8_t)(j == 1 ? (mm - 1 < 2 ? mm - 1 : 2) : j);
        } else {
            idxs[d + 1] = 0;
            ends[d + 1] = (uint8_t)(mm - 1);
        }
        inner[d + 1] = 0;
        ++d;
    }
    a.table[slot] = dom ? absent_f() : -ts;
    if (wstats) {  // ULG_WALK_STATS: walks, steps, max steps, walks over 2^20 steps
        atomicAdd(&wstats[0], 1ull);
        atomicAdd(&wstats[1], (unsigned long long)steps);
        atomicMax(&wstats[2], (unsigned long long)steps);
        if (steps > (1ull << 20)) atomicAdd(&wstats[3], 1ull);
    }
}

using WideFn = void (*)(WideArgs);
using WideWalkFn = void (*)(WideArgs, uint64_t, uint64_t, uint64_t *, uint64_t, unsigned long long *,
                           unsigned long long *, uint64_t, uint64_t *, unsigned long long *);
WideFn wide_fn(int L, int phase) {
    if (L <= 16) return phase == 0 ? score_wide_kernel<16, 0> : score_wide_kernel<16, 1>;
    return phase == 0 ? score_wide_kernel<kWideMax, 0> : score_wide_kernel<kWideMax, 1>;
}
WideWalkFn wide_walk_fn(int L, int phase) {
    if (L <= 16) return phase == 0 ? walk_wide_kernel<16, 0> : walk_wide_kernel<16, 1>;
    return phase == 0 ? walk_wide_kernel<kWideMax, 0> : walk_wide_kernel<kWideMax, 1>;
}

// ---- long wide walks in LDS -----------------------------------------------
// A wide walk is one lane's sequential DFS; the few long ones set a layer's
// time (C1 at the reference's default lambda 0.5: single walks of 5-19 M
// steps at L = 18, 19), and in walk_wide_kernel every step waits on scratch
// memory and global bitsets (~1 us).  Walks over kStragBudget steps (only
// where q = |local bits| <= kStragQMax and the hi-cover tables exist) are
// re-queued and replayed here from the start, one workgroup per set.
//
// Fill: the workgroup lays out, over the 2^q local subsets, two bitsets from
// pval / hmax: `skip` (present below -ts, or absent with no key >= -ts among
// its subsets and variable 0: a test of it changes nothing but `checked`,
// which it would never consult again) and `hi` (present and >= -ts: the walk
// stops there).  A test is then: skip bit set (or checked) -> next; hi bit set
// -> dominated; otherwise expand.  `checked` merges into `skip`: checked nodes
// are expanded ones, never hi, and the empty set starts checked.
//
// Walk (lane 0): the reduced walk of walk_wide_kernel with every parent-vector
// list held as a bit mask.  A list is its real entries in increasing local-bit
// order followed by zero padding (the root list is P's bits; an expansion of
// T2 = T ^ {x} appends the caller's entries != x in order, so order is kept,
// and zeros appended from the padding read like padding), so a frame is: node
// N, removed entry x, the caller's list (remaining mask `rem`, remaining zeros
// `zr`), the appended mask B, the call count js, and whether the current call
// still owes its position-1 test (call 1 tests positions 0 and 1, call j >= 2
// position j - 1 = the entry it appended).  N is checked after each call of
// its expansion returns (BIC_OLS.cpp:234 recursion).  Wave 0 runs
// the walk with its lanes reading a node's q neighbour bits at once, so a
// test is a register bit test; frames are 32 B in LDS, pushed per expansion.
constexpr int kStragQMax = 20;                 // skip bitset 2^20 bits = 128 KiB of LDS
constexpr int kStragHiLdsQ = 19;               // hi bitset in LDS up to here, else in global scratch
constexpr uint64_t kStragBudget = 1ull << 6;  // steps in walk_wide_kernel before a walk moves here (2^13 -> 2^6: C4 0.82 -> 0.24 s, C1 10.0 -> 9.4 s)
// ULG_STRAG_BUDGET=<log2 steps> overrides it (A/B timing only: results are the same)
inline uint64_t strag_budget() {
    static const uint64_t b = std::getenv("ULG_STRAG_BUDGET") ? 1ull << std::atoi(std::getenv("ULG_STRAG_BUDGET"))
                                                              : kStragBudget;
    return b;
}
constexpr int kStragThreads = 256;             // fill threads (64 when many walks share the GPU); wave 0 walks
constexpr uint64_t kStragWide = 4096;          // replays per launch from which blocks are one wave

// The fill of one replay (entry e of the straggler queue) into skip / hib
// (word w at skip[w * stride], hib[w * stride]): lc (>= 32 bytes) and xlow
// (64 words), shared by the block, receive the local-bit -> compact index
// map and the compact masks of the 64 low-bit patterns.  Every thread of the
// block takes words w = tid, tid + nthreads, ...
template <int PHASE>
__device__ __forceinline__ void strag_fill(const WideArgs &a, const uint64_t *e, uint64_t *skip, uint64_t *hib,
                                           uint32_t stride, uint8_t *lc, uint64_t *xlow, uint32_t tid,
                                           uint32_t nthreads) {
    const int L = a.L;
    const int q = PHASE == 0 ? L : L + 1;
    const uint32_t nw = (1u << q) >> 6;
    const uint64_t cm = e[1];
    const int vi = (int)(uint32_t)e[2];
    const float thr = -__uint_as_float((uint32_t)(e[2] >> 32));
    const bool z = a.meta[vi * 4 + 2] != 0;
    const uint64_t zb = z ? 1ull : 0ull;
    const uint64_t ho = a.hoff[vi];
    if (tid == 0) {
        uint64_t rem = cm;
        const int first = PHASE == 0 ? 0 : 1;
        lc[0] = 0;
        for (int i = first; i < L + first; ++i) {
            lc[i] = (uint8_t)__builtin_ctzll(rem);
            rem &= rem - 1;
        }
    }
    __syncthreads();
    if (tid < 64) {  // compact mask of local bits 1..5 of pattern tid (bit 0 = variable 0: zb)
        uint64_t X = 0;
        for (uint32_t y = tid & ~1u; y; y &= y - 1) X |= 1ull << lc[__builtin_ctz(y)];
        xlow[tid] = X | ((tid & 1u) ? zb : 0ull);
    }
    __syncthreads();
    for (uint32_t w = tid; w < nw; w += nthreads) {
        uint64_t sw = 0, hw = 0;
        uint64_t Xw = 0;  // compact mask of the word's high local bits
        for (uint32_t y = (w << 6); y; y &= y - 1) Xw |= 1ull << lc[__builtin_ctz(y)];
#pragma unroll 8
        for (int b = 0; b < 64; ++b) {
            const uint32_t t = (w << 6) | (uint32_t)b;
            const uint64_t X = Xw | xlow[b];
            bool pres = false, hi = false;
            if (!(PHASE == 1 && (t & 1u) && !z)) {
                const float val = a.pval[ho + X];
                if (fbits(val) != kAbsentBits) {
                    pres = true;
                    hi = val >= thr;
                }
            }
            const bool sk = t == 0 || (pres ? !hi : !(a.hmax[ho + (X | zb)] >= thr));
            if (sk) sw |= 1ull << b;
            if (hi && t != 0) hw |= 1ull << b;
        }
        skip[(uint64_t)w * stride] = sw;
        hib[(uint64_t)w * stride] = hw;
    }
    __syncthreads();
}

// The fills of the replays handed to the host (one block each, entries
// sq[3 * idx[b]]), written to out: [b][skip nw words][hi nw words].
template <int PHASE>
__global__ void __launch_bounds__(256) strag_fill_global_kernel(WideArgs a, const uint64_t *sq, const uint32_t *idx,
                                                                uint64_t *out) {
    __shared__ uint8_t lc[64];
    __shared__ uint64_t xlow[64];
    const int q = PHASE == 0 ? a.L : a.L + 1;
    const uint64_t nw = ((uint64_t)1 << q) >> 6;
    uint64_t *o = out + (uint64_t)blockIdx.x * 2 * nw;
    strag_fill<PHASE>(a, sq + 3 * (uint64_t)idx[blockIdx.x], o, o + nw, 1, lc, xlow, threadIdx.x, blockDim.x);
}

// host_budget > 0: a walk still running after that many iterations stops,
// and its queue index goes to hq (count *hqc) for the host (host_walk):
// one wave issues at most one instruction every 4 cycles, so a long
// sequential walk runs far faster on a host core.
template <int PHASE, bool HI_LDS>
__global__ void __launch_bounds__(kStragThreads) walk_wide_lds_kernel(WideArgs a, const uint64_t *sq,
                                                                      uint64_t *hig, unsigned long long *err,
                                                                      unsigned long long *wstats, uint64_t host_budget,
                                                                      uint32_t *hq, unsigned int *hqc, uint32_t qbase) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int L = a.L;
    const int q = PHASE == 0 ? L : L + 1;
    const uint32_t nw = (1u << q) >> 6;
    // HI_LDS: skip and hi words interleaved (one 16-B read per neighbour);
    // else skip in LDS and hi in this block's global scratch
    constexpr uint32_t kS = HI_LDS ? 2u : 1u;
    uint64_t *skip = reinterpret_cast<uint64_t *>(smem);
    uint64_t *hib = HI_LDS ? skip + 1 : hig + (uint64_t)blockIdx.x * nw;
    uint64_t *xlow = skip + (HI_LDS ? 2 * nw : nw);
    uint8_t *lc = reinterpret_cast<uint8_t *>(xlow + 64);
    const uint64_t *e = sq + 3 * (uint64_t)blockIdx.x;
    const uint64_t slot = e[0];
    const float ts = __uint_as_float((uint32_t)(e[2] >> 32));
    const uint64_t tk0 = wstats ? wall_clock64() : 0;
    strag_fill<PHASE>(a, e, skip, hib, kS, lc, xlow, threadIdx.x, blockDim.x);
    if (threadIdx.x >= 64) return;
    // wave 0 walks, every lane in step (the walk state is wave-uniform); the
    // lanes only split up to read a node's neighbour bits: bit l of sm / hm is
    // the skip / hi bit of N ^ {l}.  Within one expansion only its children's
    // subtrees change `skip` (N's own mark is not a neighbour of N), so sm is
    // re-read after each child returns and every test is a register bit test.
    const int lane = threadIdx.x;
    const uint64_t tk1 = wstats ? wall_clock64() : 0;
    // lanes >= q read a valid word too, so both loads issue back to back
    const uint32_t lbit = 1u << (lane < q ? lane : 0);
    auto nbr = [&](uint32_t Nn, uint32_t &sm_, uint32_t &hm_) {
        const uint32_t t = Nn ^ lbit;
        uint64_t sw, hw;
        if constexpr (HI_LDS) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(skip + 2 * (t >> 6));
            sw = v.x;
            hw = v.y;
        } else {
            sw = skip[t >> 6];
            hw = hib[t >> 6];
        }
        sm_ = (uint32_t)__ballot((int)(((sw >> (t & 63)) & 1ull) | (lane >= q)));
        hm_ = (uint32_t)__ballot((int)(((hw >> (t & 63)) & 1ull) & (lane < q)));
    };
    // frames in VGPR lanes: lane d of fN .. fSm holds frame d (kStragDepth <= 64)
    uint32_t fN = 0, fRem = 0, fB = 0, fW = 0, fHm = 0, fSm = 0;
    auto wl = [&](uint32_t v, int l, uint32_t old) -> uint32_t { return lane == l ? v : old; };
    auto rl = [](uint32_t v, int l) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); };
    const uint32_t P = PHASE == 0 ? ((1u << L) - 1u) : (((1u << L) - 1u) << 1);
    uint32_t N = P, rem = P, B = 0, sm, hm;
    nbr(N, sm, hm);
    int x = 31, zr = 0, js = 0, d = 0, mS = L;
    bool pend = false, incall = false, dom = false;
    uint64_t it = 0;
    while (true) {
        if (++it > kStragIterCap) {
            if (lane == 0) atomicOr(err, 1ull);
            break;
        }
        if (host_budget && it > host_budget) {  // to the host, from the start
            if (lane == 0) hq[atomicAdd(hqc, 1u)] = qbase + blockIdx.x;
            return;
        }
        int y;
        if (pend) {  // call 1's position-1 test: the zero padding, variable 0
            pend = false;
            y = 0;
        } else {
            if (incall) {  // the call returned: checked.insert(N)
                if (lane == 0) atomicOr(&skip[(N >> 6) * kS], 1ull << (N & 63));
                incall = false;
            }
            // Next test that is not a no-op.  A test whose node has its skip
            // bit set changes nothing, so after call 1 (N is checked from then
            // on) a run of such calls only appends its entries to B.
            const uint32_t xb = x < 32 ? 1u << x : 0u;
            const uint32_t cand = rem & ~xb;  // real entries that make calls
            bool found = false;
            if (d == 0) {  // the root call: P's entries, no appends
                const uint32_t ev = rem & ~sm;
                if (ev) {
                    y = __builtin_ctz(ev);
                    rem &= ~((2u << y) - 1u);
                    found = true;
                }
            } else if (js == 0) {  // call 1, with its position-1 test
                if (cand) {
                    y = __builtin_ctz(cand);
                    rem &= ~((2u << y) - 1u);
                    B |= 1u << y;
                    found = true;
                } else if (zr && x != 0) {  // the first entry is padding
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
                    const uint32_t run = cand & ((2u << y) - 1u);  // skipped calls + this one
                    B |= run;
                    js += __popc(run);
                    rem &= ~((2u << y) - 1u);
                    incall = true;
                    found = true;
                } else {
                    B |= cand;  // the rest of the real entries: no-op calls
                    js += __popc(cand);
                    rem = 0;
                    if (zr && x != 0) {  // padding entries: each a call testing N ^ {0}
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
            if (!found) {  // the expansion (or the root call) is done
                if (d == 0) break;
                // Back in the caller's frame, whose neighbour bits the subtree of
                // N = caller ^ {x} changed only at N itself (marked iff it made
                // a call) when x != 0: x never re-enters a list below it, so
                // every node of the subtree differs from the caller in bit x.
                // Variable 0 re-enters as padding: then read them again.
                const int cx = x;
                const bool cmarked = js > 0;
                --d;
                N = rl(fN, d);
                rem = rl(fRem, d);
                B = rl(fB, d);
                const uint32_t w = rl(fW, d);
                hm = rl(fHm, d);
                sm = rl(fSm, d);
                x = (int)(w & 31u);
                zr = (int)((w >> 5) & 31u);
                js = (int)((w >> 10) & 31u);
                pend = (w >> 15) & 1u;
                incall = (w >> 16) & 1u;
                mS = d == 0 ? L : L - d + 1;
                if (cx != 0) {
                    if (cmarked) sm |= 1u << cx;
                } else {
                    uint32_t h2;
                    nbr(N, sm, h2);
                }
                continue;
            }
        }
        if ((sm >> y) & 1u) continue;
        if ((hm >> y) & 1u) {
            dom = true;
            break;
        }
        // expand N ^ {y} with the current call's list (root: P's bits; else B_j)
        const uint32_t Sc = d == 0 ? P : B;
        const int mc = d == 0 ? L : mS - 1;
        if (d + 1 >= kStragDepth || mc < __popc(Sc)) {  // cannot happen: the list holds its entries
            if (lane == 0) atomicOr(err, 1ull);
            break;
        }
        fN = wl(N, d, fN);
        fRem = wl(rem, d, fRem);
        fB = wl(B, d, fB);
        fW = wl((uint32_t)x | ((uint32_t)zr << 5) | ((uint32_t)js << 10) | ((uint32_t)pend << 15) |
                    ((uint32_t)incall << 16),
                d, fW);
        fHm = wl(hm, d, fHm);
        fSm = wl(sm, d, fSm);
        ++d;
        N ^= 1u << y;
        x = y;
        rem = Sc;
        zr = mc - __popc(Sc);
        B = 0;
        js = 0;
        pend = false;
        incall = false;
        mS = mc;
        nbr(N, sm, hm);
    }
    if (lane != 0) return;
    a.table[slot] = dom ? absent_f() : -ts;
    if (wstats) {  // ULG_WALK_STATS: replays, iterations, max iterations, max fill / walk ticks
        const uint64_t tk2 = wall_clock64();
        atomicAdd(&wstats[4], 1ull);
        atomicAdd(&wstats[5], (unsigned long long)it);
        atomicMax(&wstats[6], (unsigned long long)it);
        atomicMax(&wstats[7], (unsigned long long)(tk1 - tk0));
        atomicMax(&wstats[8], (unsigned long long)(tk2 - tk1));
    }
}

// ---- hi-cover tables for the wide walks ---------------------------------
// Per walking variable (m <= kHiMaxBits candidates), before each wide walk
// launch: hmax[X] = max over the keys present in the cache when this phase
// runs (layers < L, and in phase 1 the layer-L sets holding variable 0,
// SURVEY N4) of their stored value, over every subset of the compact mask X;
// absent keys count as -inf.  A subset-max (zeta) transform: the low
// kHiTileBits bits per LDS tile, the rest kHiGroup bits per strided pass.
constexpr int kHiTileBits = 12;
constexpr int kHiMaxBits = 24;  // 64 MB of floats per variable at most
constexpr int kHiGroup = 4;

struct HiArgs {
    const int *lvars;     // walking variables of this launch (batch index)
    const int *prefix;    // [nl + 1]: tiles (tile pass) or blocks (strided pass) per variable
    int nl;
    const int *meta;
    const uint64_t *tbl_off;
    const float *table;
    const uint64_t *binom;  // [64][64]
    float *hmax;
    float *pval;
    const uint64_t *hoff;
    int S, L, kmax, bit_lo;
};

__device__ __forceinline__ int hi_find(const int *prefix, int nl, int x) {
    int lo = 0, hi = nl;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (prefix[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

template <int PHASE>
__global__ void __launch_bounds__(1024) hikey_tile_kernel(HiArgs a) {
    __shared__ float t[1 << kHiTileBits];
    const int li = hi_find(a.prefix, a.nl, blockIdx.x);
    const int vi = a.lvars[li];
    const int m = a.meta[vi * 4 + 1];
    const bool z = a.meta[vi * 4 + 2] != 0;
    const int tb = m < kHiTileBits ? m : kHiTileBits;
    const int cnt = 1 << tb;
    const uint64_t base = (uint64_t)(blockIdx.x - a.prefix[li]) << kHiTileBits;
    const uint64_t *toff = a.tbl_off + (uint64_t)vi * a.S;
    for (int i = threadIdx.x; i < cnt; i += 1024) {
        const uint64_t X = base + (uint64_t)i;
        const int l = __popcll(X);
        float val = -INFINITY, pv = absent_f();
        if (l <= a.kmax && (l < a.L || (PHASE == 1 && l == a.L && (X & 1ull) && z))) {
            const float f = a.table[toff[l] + rank_colex64(X, a.binom)];
            pv = f;
            if (fbits(f) != kAbsentBits && f == f) val = f;  // absent or NaN: never >= -ts
        }
        a.pval[a.hoff[vi] + X] = pv;
        t[i] = val;
    }
    __syncthreads();
    for (int b = 0; b < tb; ++b) {
        for (int i = threadIdx.x; i < cnt; i += 1024)
            if (!((i >> b) & 1)) t[i | (1 << b)] = fmaxf(t[i | (1 << b)], t[i]);
        __syncthreads();
    }
    float *h = a.hmax + a.hoff[vi] + base;
    for (int i = threadIdx.x; i < cnt; i += 1024) h[i] = t[i];
}

__global__ void __launch_bounds__(256) hikey_strided_kernel(HiArgs a) {
    const int li = hi_find(a.prefix, a.nl, blockIdx.x);
    const int vi = a.lvars[li];
    const int m = a.meta[vi * 4 + 1];
    const int G = m - a.bit_lo < kHiGroup ? m - a.bit_lo : kHiGroup;
    const uint64_t tid = (uint64_t)(blockIdx.x - a.prefix[li]) * 256 + threadIdx.x;
    if (G <= 0 || tid >= (1ull << (m - G))) return;
    const uint64_t lowm = (1ull << a.bit_lo) - 1ull;
    const uint64_t base = ((tid & ~lowm) << G) | (tid & lowm);
    float *h = a.hmax + a.hoff[vi];
    float r[1 << kHiGroup];
    for (int k = 0; k < (1 << G); ++k) r[k] = h[base + ((uint64_t)k << a.bit_lo)];
    for (int b = 0; b < G; ++b)
        for (int k = 0; k < (1 << G); ++k)
            if (!((k >> b) & 1)) r[k | (1 << b)] = fmaxf(r[k | (1 << b)], r[k]);
    for (int k = 0; k < (1 << G); ++k) h[base + ((uint64_t)k << a.bit_lo)] = r[k];
}

// The call's first launch: cache[empty] = -0.0f per variable (BIC_OLS.cpp:249)
// and the walk-queue counters zeroed.  It sits inside the call's hipGraph;
// as three eager launches before the replay (a kernel and two memsets) they
// left ~40 us of submission gaps ahead of the first layer.
__global__ void call_prologue_kernel(const uint64_t *tbl_off, int nv, int S, float *table,
                                     unsigned long long *qcount, uint64_t nqc, unsigned long long *qseg,
                                     uint64_t nseg) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (uint64_t)nv) table[tbl_off[i * (uint64_t)S]] = -0.0f;
    if (qcount && i < nqc) qcount[i] = 0ull;
    if (qseg && i < nseg) qseg[i] = 0ull;
}

// ---- compaction of the slabs into (set, score) lists ------------------------
constexpr int kSlotsPerThread = 16;  // contiguous slots per thread (four 16-B loads)
constexpr int kSlotsPerBlock = kBlock * kSlotsPerThread;

// the thread's kSlotsPerThread slots from `base` (absent past the end)
__device__ __forceinline__ void load_slots(const float *table, uint64_t total, uint64_t base,
                                           float (&v)[kSlotsPerThread]) {
    if (base + kSlotsPerThread <= total) {
        const float4 *p = reinterpret_cast<const float4 *>(table + base);
#pragma unroll
        for (int q = 0; q < kSlotsPerThread / 4; ++q) {
            const float4 f = p[q];
            v[4 * q] = f.x;
            v[4 * q + 1] = f.y;
            v[4 * q + 2] = f.z;
            v[4 * q + 3] = f.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kSlotsPerThread; ++j) v[j] = base + j < total ? table[base + j] : absent_f();
    }
}

__global__ void __launch_bounds__(kBlock) count_kernel(const float *table, uint64_t total, uint64_t *blk) {
    __shared__ uint32_t red[kBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kSlotsPerBlock + threadIdx.x * kSlotsPerThread;
    float v[kSlotsPerThread];
    load_slots(table, total, base, v);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kSlotsPerThread; ++j) c += fbits(v[j]) != kAbsentBits;
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w];
        blk[blockIdx.x] = t;
    }
}

// exclusive scan of nb block counts in place, total in blk[nb] and in
// *total (the lists' end offset, offsets[nv]); one block: each thread sums
// its run of counts, a shuffle scan per wave and one over the 16 wave
// totals (two barriers; the Hillis-Steele form took 20, 10.6 us at C3)
// blk[nb + 1]: a copy of the call's error word (0 without one), so one copy
// brings the stored count and the error bits to the host
__global__ void __launch_bounds__(1024) scan_kernel(uint64_t *blk, int64_t nb, int64_t *total,
                                                    const unsigned long long *err) {
    __shared__ unsigned long long wsum[16];
    const int64_t per = (nb + 1023) / 1024;
    const int64_t b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
    unsigned long long s = 0;
    for (int64_t i = b0; i < b1; ++i) s += blk[i];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (wv == 0) {
        const unsigned long long w = lane < 16 ? wsum[lane] : 0ull;
        unsigned long long wi = w;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const unsigned long long t = __shfl_up(wi, o);
            if (lane >= o) wi += t;
        }
        if (lane < 16) wsum[lane] = wi - w;
        if (lane == 15) {
            blk[nb] = wi;
            blk[nb + 1] = err ? *err : 0ull;
            *total = (int64_t)wi;
        }
    }
    __syncthreads();
    uint64_t acc = wsum[wv] + incl - s;
    for (int64_t i = b0; i < b1; ++i) {
        const uint64_t t = blk[i];
        blk[i] = acc;
        acc += t;
    }
}

struct WriteArgs {
    const float *table;
    const uint64_t *blk;
    const uint64_t *tbl_off;
    const int *meta;
    const uint8_t *cand;
    const uint32_t *binom;
    const uint64_t *binom64;  // wide layers (L > kMaxL)
    uint64_t total;
    int nv, S;
    uint64_t *sets;
    float *scores;
    int64_t *offsets;
};

constexpr int kWriteLdsSegs = 2048;  // slab offsets staged in LDS up to this many (vi, L) segments

// Stored slots -> (set, score) lists.  A thread's slots are contiguous, so it
// locates its first slot's (variable, layer) segment and unranks it once;
// every later slot is the colex successor (Gosper's hack, typedefs.h:692-697)
// inside the segment, or the first set (1 << L) - 1 of the next one.
// 8 waves per SIMD (<= 64 VGPRs) and the slab offsets in dynamic LDS sized
// to the call ((nv * S + 1) * 8 bytes, 1.6 KB at C3, instead of a fixed 16 KB):
// the kernel waits on its loads, so resident waves are what it needs.
__global__ void __launch_bounds__(kBlock, 8) write_kernel(WriteArgs a) {
    __shared__ uint32_t pre[kBlock / 64];
    __shared__ uint32_t binom[64 * kBinomK];
    extern __shared__ uint64_t toff_s[];  // (nv * S + 1) entries when nv * S <= kWriteLdsSegs
    __shared__ uint32_t cand_s[64 * 16];  // the candidate lists (64 bytes per variable, nv <= 64)
    const int nseg = a.nv * a.S;
    const bool lds_off = nseg <= kWriteLdsSegs;
    for (int i = threadIdx.x; i < 64 * kBinomK; i += kBlock) binom[i] = a.binom[i];
    for (int i = threadIdx.x; i < a.nv * 16; i += kBlock) cand_s[i] = reinterpret_cast<const uint32_t *>(a.cand)[i];
    const uint8_t *cand = reinterpret_cast<const uint8_t *>(cand_s);
    if (lds_off)
        for (int i = threadIdx.x; i <= nseg; i += kBlock) toff_s[i] = a.tbl_off[i];
    const uint64_t *toff = lds_off ? toff_s : a.tbl_off;
    const uint64_t base = (uint64_t)blockIdx.x * kSlotsPerBlock + threadIdx.x * kSlotsPerThread;
    float vals[kSlotsPerThread];
    load_slots(a.table, a.total, base, vals);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kSlotsPerThread; ++j) c += fbits(vals[j]) != kAbsentBits;
    // block-wide exclusive prefix of the per-thread counts: wave scan + wave totals
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t incl = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) pre[wv] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wv; ++w) wbase += pre[w];
    if (c == 0) return;
    uint64_t pos = a.blk[blockIdx.x] + wbase + incl - c;
    int first = 0;
    while (fbits(vals[first]) == kAbsentBits) ++first;
    uint64_t s0 = base + first;
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (toff[mid] <= s0) lo = mid; else hi = mid;
    }
    int seg = lo;
    int vi = seg / a.S, L = seg % a.S;
    int m = a.meta[vi * 4 + 1];
    uint64_t cm = L <= kMaxL ? unrank_colex(s0 - toff[seg], L, m, binom)
                             : unrank_colex64(s0 - toff[seg], L, m, a.binom64);
    for (int j = first; j < kSlotsPerThread; ++j) {
        const uint64_t s = base + j;
        // the last block's slots past the table hold nothing, and the
        // segment search below must not run past the last offset
        // (toff[nseg] = total): it read toff[nseg + 1]
        if (s >= a.total) break;
        if (j > first) {
            if (s >= toff[seg + 1]) {
                while (s >= toff[seg + 1]) ++seg;
                vi = seg / a.S;
                L = seg % a.S;
                m = a.meta[vi * 4 + 1];
                cm = L ? (~0ull >> (64 - L)) : 0ull;
            } else {
                const uint64_t r = cm + (cm & (0 - cm));
                cm = r | (((r ^ cm) >> 2) >> __builtin_ctzll(cm));
            }
        }
        if (fbits(vals[j]) == kAbsentBits) continue;
        uint64_t gs = 0;
        uint64_t rem = cm;
        while (rem) {
            const int b = __builtin_ctzll(rem);
            rem &= rem - 1;
            gs |= 1ull << cand[vi * 64 + b];
        }
        a.sets[pos] = gs;
        a.scores[pos] = vals[j];
        if (L == 0) a.offsets[vi] = (int64_t)pos;
        ++pos;
    }
}


__global__ void quantize_kernel(const float *in, float *out, int64_t count) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < count) out[i] = quantize_score(in[i]);
}

// ScoringFunction::calculateScore's return value for arbitrary (variable,
// parent set) pairs (BIC_OLS.cpp:174-276 via calculateScoreAndBeta, :277-388):
// -float(N ln(RSS/N) + lambda ln(N) |P|), 0 parents -> -0.0f (BIC_OLS.cpp:
// 300-303).  One lane per pair, parents in ascending order (parent_vec), the
// Cholesky in the layer kernels' operation order, so a stored set's value is
// the one ulg_cbic_score stored for it.
__global__ void __launch_bounds__(kBlock) score_sets_kernel(const double *gram, const uint64_t *pairs, int64_t count,
                                                            int n, double N, double lambda, float *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *g = reinterpret_cast<double *>(smem);
    for (int i = threadIdx.x; i < n * n; i += kBlock) g[i] = gram[i];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const int v = (int)pairs[2 * i];
    const uint64_t P = pairs[2 * i + 1] & ~(1ull << v);
    const int L = __builtin_popcountll(P);
    if (L == 0) {
        out[i] = -0.0f;
        return;
    }
    int gv[kWideMax];
    {
        uint64_t rem = P;
        for (int j = 0; j < L; ++j) {
            gv[j] = __builtin_ctzll(rem);
            rem &= rem - 1;
        }
    }
    double Lm[kWideMax * (kWideMax + 1) / 2];
    double y[kWideMax];
    for (int r = 0; r < L; ++r) {
        for (int j = 0; j <= r; ++j) Lm[r * (r + 1) / 2 + j] = g[gv[r] * n + gv[j]];
        y[r] = g[gv[r] * n + v];
    }
    const double cvv = g[v * n + v];
    for (int j = 0; j < L; ++j) {
        const int rj = j * (j + 1) / 2;
        double s = Lm[rj + j];
        for (int k = 0; k < j; ++k) s -= Lm[rj + k] * Lm[rj + k];
        const double d = sqrt(s);
        Lm[rj + j] = d;
        const double inv = 1.0 / d;
        for (int r = j + 1; r < L; ++r) {
            const int rr = r * (r + 1) / 2;
            double t = Lm[rr + j];
            for (int k = 0; k < j; ++k) t -= Lm[rr + k] * Lm[rj + k];
            Lm[rr + j] = t * inv;
        }
    }
    double yy = 0.0;
    for (int r = 0; r < L; ++r) {
        const int rr = r * (r + 1) / 2;
        double t = y[r];
        for (int k = 0; k < r; ++k) t -= Lm[rr + k] * y[k];
        t = t / Lm[rr + r];
        y[r] = t;
        yy += t * t;
    }
    const double rss = cvv - yy;
    const double the_score = N * log(rss / N) + lambda * log(N) * (double)L - 0.0;  // BIC_OLS.cpp:366
    out[i] = -(float)the_score;
}

using KernelFn = void (*)(ScoreArgs);
template <int L, int V>
KernelFn pick_phase(int phase) {
    return phase == 0 ? score_layer_kernel<L, 0, V> : score_layer_kernel<L, 1, V>;
}
// variants (ulg_set_option "score_variant"): bit 0 unrolled presence gathers
// (layers <= 6), bit 4 two-pass (settle, queue the rest for a walk launch),
// bit 5 bit-sliced walk, bit 6 subset maxima.  1: one-pass (also the form for
// tables of 2^30 slots or more); 65: one-pass with the subset maxima (the
// small layers of 113); 49: two-pass with the bit-sliced walk (the tests'
// every-set-gathered reference); 113: the same with the subset maxima (the
// default).  Gone after measurement: round 4's per-lane walk forms 17 / 81
// and a variant that walked the open sets inside the scoring kernel (C5 5.05
// against 3.59 ms: a 64-set union tree repeats work a 256-set one shares);
// round 1's loop gathers at every layer, stack-machine recursion,
// decision-only per-lane walk and statistics build.
template <int L>
KernelFn pick(int phase, int variant) {
    switch (variant) {
        case 1: return pick_phase<L, 1>(phase);
        case 49: return pick_phase<L, 17>(phase);
        case 65: return pick_phase<L, 65>(phase);
        case 113: return pick_phase<L, 81>(phase);
        case 241: return pick_phase<L, 209>(phase);
        default: return nullptr;
    }
}
using SlicedFn = void (*)(const uint64_t *, const unsigned long long *, float *, float *, uint64_t *, uint64_t,
                         unsigned long long *);
template <int L, int K>
SlicedFn sliced_pick(int phase) {
    return phase == 0 ? walk_sliced_kernel<L, 0, K> : walk_sliced_kernel<L, 1, K>;
}
template <int K>
SlicedFn sliced_fn_k(int L, int phase) {
    switch (L) {
        case 1: return sliced_pick<1, K>(phase);
        case 2: return sliced_pick<2, K>(phase);
        case 3: return sliced_pick<3, K>(phase);
        case 4: return sliced_pick<4, K>(phase);
        case 5: return sliced_pick<5, K>(phase);
        case 6: return sliced_pick<6, K>(phase);
        default: return nullptr;
    }
}
// L = 7, 8 (256 / 512 local subsets): 2 and 1 sets per lane keep each of the
// two vectors at 16 registers (C4: 3.95 -> 2.75 ms per step against the
// per-lane walk_kernel)
SlicedFn sliced_fn_wide(int L, int phase) {
    switch (L) {
        case 7: return sliced_pick<7, 2>(phase);
        case 8: return sliced_pick<8, 1>(phase);
        default: return nullptr;
    }
}
// sets per lane: more sets share one walk of the union tree, fewer give more
// waves to hide the walk's latency
// sets per lane of the bit-sliced walk: 2 up to layer 5, 4 at layer 6
// (rounds 2-4: with the open bits in LDS, 4 / 8 measured 0.558 against 0.547
// ms per C3 bench step over three alternating runs, 4 / 4 0.556, though C5
// calls prefer 4 / 8: 3.15 against 3.36 ms); ULG_SLICED_K=1|2|4|8 (every
// layer) or a,b (layers <= 5, layer 6) overrides for A/B
constexpr int kSlicedKSmall = 2;  // default sets per lane up to layer 5
constexpr int kSlicedK6 = 4;      // ... at layer 6
// A layer-6 launch of fewer than `small` sets (the shares of 4 and 8 ranks,
// where a stream group holds one or two variables) walks one set per lane:
// its few waves then each walk a quarter of the union tree, and the launch
// ends with its longest wave (C3 8-rank share 0.80 -> 0.73 ms; the one-GPU
// launches keep the wide union, best there, `profiles/r4/`).
int sliced_k(int L, uint64_t cnt = ~0ull, uint64_t small = 0, int k6 = kSlicedK6) {
    if (L >= 7) return L == 7 ? 2 : 1;
    // ULG_SLICED_K=a (every layer) or a,b (layers <= 5, layer 6): A/B only
    const char *e = std::getenv("ULG_SLICED_K");
    int k = L <= 5 ? kSlicedKSmall : (cnt < small ? 1 : k6);
    if (e) {
        const char *comma = std::strchr(e, ',');
        k = (L <= 5 || !comma) ? std::atoi(e) : std::atoi(comma + 1);
    }
    return (k == 1 || k == 2 || k == 8) ? k : 4;
}
// queued sets per walk wave
SlicedFn sliced_fn(int L, int phase, int k) {
    if (L >= 7) return sliced_fn_wide(L, phase);
    switch (k) {
        case 1: return sliced_fn_k<1>(L, phase);
        case 2: return sliced_fn_k<2>(L, phase);
        case 4: return sliced_fn_k<4>(L, phase);
        default: return sliced_fn_k<8>(L, phase);
    }
}

using BucketFn = void (*)(const uint64_t *, const uint32_t *, const unsigned int *, float *, float *, uint64_t,
                         unsigned long long *);
template <int L, int KL>
BucketFn bucket_pick(int phase) {
    return phase == 0 ? walk_bucket_kernel<L, 0, KL> : walk_bucket_kernel<L, 1, KL>;
}
// layers 5 and 6; KL = sets per lane of the light keys (2 or 4 at layer 5, 4 or 8 at 6)
BucketFn bucket_fn(int L, int phase, int kl) {
    if (L == 5) return kl >= 4 ? bucket_pick<5, 4>(phase) : bucket_pick<5, 2>(phase);
    if (L == 6) return kl >= 8 ? bucket_pick<6, 8>(phase) : bucket_pick<6, 4>(phase);
    return nullptr;
}

const char *kWalkNames[2][kMaxL + 1] = {
    {"", "walk_1_var0", "walk_2_var0", "walk_3_var0", "walk_4_var0", "walk_5_var0", "walk_6_var0", "walk_7_var0",
     "walk_8_var0"},
    {"", "walk_1_rest", "walk_2_rest", "walk_3_rest", "walk_4_rest", "walk_5_rest", "walk_6_rest", "walk_7_rest",
     "walk_8_rest"}};

using SmallFn = void (*)(ScoreArgs, const uint64_t *);
SmallFn small_kernel(int Lf) {
    switch (Lf) {
        case 1: return score_small_kernel<1, 65>;
        case 2: return score_small_kernel<2, 65>;
        case 3: return score_small_kernel<3, 65>;
        default: return score_small_kernel<4, 65>;
    }
}

KernelFn layer_kernel(int L, int phase, int variant) {
    switch (L) {
        case 1: return pick<1>(phase, variant);
        case 2: return pick<2>(phase, variant);
        case 3: return pick<3>(phase, variant);
        case 4: return pick<4>(phase, variant);
        case 5: return pick<5>(phase, variant);
        case 6: return pick<6>(phase, variant);
        case 7: return pick<7>(phase, variant);
        case 8: return pick<8>(phase, variant);
        default: return nullptr;
    }
}
static_assert(kMaxL == 8, "layer_kernel dispatch covers layers 1..8");

const char *kLayerNames[2][kMaxL + 1] = {
    {"", "score_layer_1_var0", "score_layer_2_var0", "score_layer_3_var0", "score_layer_4_var0",
     "score_layer_5_var0", "score_layer_6_var0", "score_layer_7_var0", "score_layer_8_var0"},
    {"", "score_layer_1_rest", "score_layer_2_rest", "score_layer_3_rest", "score_layer_4_rest",
     "score_layer_5_rest", "score_layer_6_rest", "score_layer_7_rest", "score_layer_8_rest"}};

// One wide layer phase on stream st: the scoring launch, then (one sync for
// the queue length) the walks, in chunks whose checked bitsets fit the budget.
// `bits` is this stream group's own slice of c->d_wbits (`slice` words): the
// groups' walks run concurrently on their own streams.
// One wide layer phase for every stream group, in stages so the groups stay
// concurrent: every group's scoring launch; the queue lengths (one D2H each
// into pinned memory, then the syncs -- the launches already overlap); every
// group's hi-cover tables and walks; the long-walk counts; the LDS replays.
// `bits` is each group's own slice of c->d_wbits (`slice` words).
struct WideGroup {
    hipStream_t st;
    const uint64_t *d_work, *h_work;
    uint64_t cnt;
    uint64_t *queue;
    unsigned long long *qc, *scnt;
    uint64_t *bits;
    int *d_hmeta;
    WideArgs wa;
    std::vector<int> hm;  // hi-cover launch metadata (kept until its copy ran)
    uint64_t qn = 0;
    uint32_t *hq = nullptr;      // replays handed to the host (indices into the straggler queue)
    unsigned int *hqc = nullptr;
};

// table[pairs[2j]] = pairs[2j + 1] (the bits of a float): the host walks' decisions
__global__ void scatter_decisions_kernel(const uint64_t *pairs, uint32_t cnt, float *table) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j < cnt) table[pairs[2 * (uint64_t)j]] = __uint_as_float((uint32_t)pairs[2 * (uint64_t)j + 1]);
}

constexpr uint64_t kHostFewReplays = 64;  // launches of at most this many replays ...
constexpr uint64_t kHostFewBudget = 512;   // ... hand walks to the host after this many iterations

// The replays walk_wide_lds_kernel handed over (more than c->wide_host
// iterations): their fills again into the group's bitset slice, one copy
// back, the walks on host threads, the decisions written into the table.
int host_walks(ulg_ctx *c, WideGroup &G, int L, int ph, int q, uint64_t sn, uint64_t slice,
               unsigned long long *errf) {
    const auto th0 = std::chrono::steady_clock::now();
    unsigned int cnt = 0;
    ULG_HIP(c, hipMemcpyAsync(&cnt, G.hqc, 4, hipMemcpyDeviceToHost, G.st));
    ULG_HIP(c, hipStreamSynchronize(G.st));
    const auto th1 = std::chrono::steady_clock::now();  // the LDS replays are done
    if (cnt == 0) return ULG_OK;
    if (cnt > sn) return set_err(c, ULG_ERR_STATE, "ulg_cbic_score: host walk queue overflow");
    std::vector<uint32_t> idx(cnt);
    std::vector<uint64_t> ent((size_t)3 * sn);
    const uint64_t *sq = G.queue + 3 * G.qn;
    ULG_HIP(c, hipMemcpyAsync(idx.data(), G.hq, (size_t)cnt * 4, hipMemcpyDeviceToHost, G.st));
    ULG_HIP(c, hipMemcpyAsync(ent.data(), sq, ent.size() * 8, hipMemcpyDeviceToHost, G.st));
    ULG_HIP(c, hipStreamSynchronize(G.st));
    const uint64_t nw = ((uint64_t)1 << q) >> 6;
    const uint64_t per = std::max<uint64_t>(1, slice / (2 * nw));
    std::vector<uint64_t> bits;
    std::vector<uint32_t> vals(cnt);
    std::vector<uint64_t> slots(cnt);
    double walk_ms = 0.0, copy_ms = 0.0;
    const auto th2 = std::chrono::steady_clock::now();
    for (uint64_t b0 = 0; b0 < cnt; b0 += per) {
        const uint64_t k = std::min<uint64_t>(per, cnt - b0);
        // this chunk's queue indices (the kernel's list is on the host now)
        ULG_HIP(c, hipMemcpyAsync(G.hq, idx.data() + b0, k * 4, hipMemcpyHostToDevice, G.st));
        prof_begin_s(c, "walk_wide_host_fill", G.st);
        if (ph == 0) strag_fill_global_kernel<0><<<(unsigned)k, 256, 0, G.st>>>(G.wa, sq, G.hq, G.bits);
        else strag_fill_global_kernel<1><<<(unsigned)k, 256, 0, G.st>>>(G.wa, sq, G.hq, G.bits);
        prof_end_s(c, G.st);
        ULG_HIP(c, hipGetLastError());
        bits.resize((size_t)(k * 2 * nw));
        ULG_HIP(c, hipStreamSynchronize(G.st));
        const auto tf0 = std::chrono::steady_clock::now();
        ULG_HIP(c, hipMemcpyAsync(bits.data(), G.bits, bits.size() * 8, hipMemcpyDeviceToHost, G.st));
        ULG_HIP(c, hipStreamSynchronize(G.st));
        copy_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
        if (const char *dd = std::getenv("ULG_DUMP_HOSTWALK")) {  // diagnostics: the bitsets of the largest ones
            static std::atomic<int> nd{0};
            static const int qmin = std::getenv("ULG_DUMP_HOSTWALK_Q") ? std::atoi(std::getenv("ULG_DUMP_HOSTWALK_Q")) : 15;
            if (q >= qmin && nd < 64) {
                char fn[512];
                std::snprintf(fn, sizeof fn, "%s/hostwalk_%d_L%d_p%d_q%d.bin", dd, nd++, L, ph, q);
                if (FILE *f = std::fopen(fn, "wb")) {
                    std::fwrite(bits.data(), 8, 2 * nw, f);
                    std::fclose(f);
                }
            }
        }
        std::atomic<uint64_t> next{0};
        std::atomic<bool> bad{false};
        auto work = [&]() {
            for (uint64_t j = next++; j < k; j = next++) {
                bool e = false;
                const bool dom = host_walk(L, ph, bits.data() + j * 2 * nw, bits.data() + j * 2 * nw + nw, &e);
                if (e) bad = true;
                const uint64_t *en = ent.data() + 3 * (uint64_t)idx[b0 + j];
                // the stored value is -ts: flip the float's sign bit
                vals[b0 + j] = dom ? kAbsentBits : ((uint32_t)(en[2] >> 32) ^ 0x80000000u);
                slots[b0 + j] = en[0];
            }
        };
        const unsigned nth = (unsigned)std::min<uint64_t>(
            k, std::min((unsigned)c->wide_host_threads, std::max(1u, std::thread::hardware_concurrency())));
        const auto twa = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nth; ++t) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
        walk_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - twa).count();
        if (bad) {
            const unsigned long long one = 1;
            ULG_HIP(c, hipMemcpyAsync(errf, &one, 8, hipMemcpyHostToDevice, G.st));
        }
    }
    // the decisions: one copy of (slot, value) pairs into the group's bitset
    // slice (free again), then one scatter launch
    const auto tw1 = std::chrono::steady_clock::now();
    std::vector<uint64_t> pairs((size_t)2 * cnt);
    for (unsigned j = 0; j < cnt; ++j) {
        pairs[2 * (size_t)j] = slots[j];
        pairs[2 * (size_t)j + 1] = vals[j];
    }
    ULG_HIP(c, hipMemcpyAsync(G.bits, pairs.data(), pairs.size() * 8, hipMemcpyHostToDevice, G.st));
    scatter_decisions_kernel<<<(cnt + 255) / 256, 256, 0, G.st>>>(G.bits, cnt, G.wa.table);
    ULG_HIP(c, hipGetLastError());
    ULG_HIP(c, hipStreamSynchronize(G.st));  // pairs is about to go
    static const bool wstat = std::getenv("ULG_WALK_STATS") != nullptr;
    if (wstat) {
        const auto tw2 = std::chrono::steady_clock::now();
        auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        std::fprintf(stderr,
                     "walk_host_stats L=%d phase=%d q=%d handed=%u of %llu ms=%.2f (gpu replays %.2f, lists %.2f, "
                     "bits copy %.2f, walks %.2f, write %.2f)\n",
                     L, ph, q, cnt, (unsigned long long)sn, ms(th0, tw2), ms(th0, th1), ms(th1, th2), copy_ms, walk_ms,
                     ms(tw1, tw2));
    }
    return ULG_OK;
}

// pin: 2 * gs.size() pinned words of the caller's (queue lengths, long-walk counts)
int score_wide_groups(ulg_ctx *c, int L, int ph, std::vector<WideGroup> &gs, int nv, int S, int kmax,
                      unsigned long long *errf, uint64_t slice, const std::vector<uint64_t> &hoff,
                      const std::vector<int> &meta, unsigned long long *pin) {
    const int ng = (int)gs.size();
    const int q = ph == 0 ? L : L + 1;
    // 1. scoring launches
    for (int gi = 0; gi < ng; ++gi) {
        WideGroup &G = gs[gi];
        WideArgs &wa = G.wa;
        wa.gram = c->gram.p;
        wa.binom = c->d_binom64.p;
        wa.cand = c->d_cand.p;
        wa.meta = c->d_meta.p;
        wa.tbl_off = c->d_tbl_off.p;
        wa.work = G.d_work;
        wa.table = c->table.p;
        wa.queue = G.queue;
        wa.qcount = G.qc;
        wa.hmax = nullptr;
        wa.pval = nullptr;
        wa.hoff = nullptr;
        wa.reduced = c->wide_reduced;
        wa.N = (double)c->N;
        wa.lambda = c->lambda;
        wa.n = c->n;
        wa.nv = nv;
        wa.S = S;
        wa.L = L;
        const uint64_t blocks = (G.cnt + kBlock - 1) / kBlock;
        const WideFn sf = wide_fn(L, ph);
        const int lds = c->n * c->n * 8;
        if (lds > 64 * 1024)
            ULG_HIP(c, hipFuncSetAttribute((const void *)sf, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        prof_begin_s(c, ph == 0 ? "score_wide_var0" : "score_wide_rest", G.st);
        hipLaunchKernelGGL(sf, dim3((unsigned)blocks), dim3(kBlock), (size_t)lds, G.st, wa);
        prof_end_s(c, G.st);
        ULG_HIP(c, hipGetLastError());
        ULG_HIP(c, hipMemcpyAsync(pin + gi, G.qc, 8, hipMemcpyDeviceToHost, G.st));
    }
    for (int gi = 0; gi < ng; ++gi) {
        ULG_HIP(c, hipStreamSynchronize(gs[gi].st));
        gs[gi].qn = pin[gi];
    }
    // 2. hi-cover tables and walks
    static const bool wstat = std::getenv("ULG_WALK_STATS") != nullptr;  // diagnostics: synchronises
    const WideWalkFn wf = wide_walk_fn(L, ph);
    const uint64_t wpl = q <= 6 ? 1ull : (1ull << (q - 6));
    std::vector<uint64_t> budget(ng, 0);
    for (int gi = 0; gi < ng; ++gi) {
        WideGroup &G = gs[gi];
        if (G.qn == 0) continue;
        hipStream_t st = G.st;
        WideArgs &wa = G.wa;
        if (G.d_hmeta) {
            // hi-cover tables of this launch's variables: [lvars][tile prefix][one
            // block prefix per strided pass], one upload
            std::vector<int> lv;
            for (int i = 0; i < nv; ++i)
                if (G.h_work[i + 1] > G.h_work[i] && hoff[i] != ~0ull) lv.push_back(i);
            const int nl = (int)lv.size();
            if (nl > 0) {
                int maxm = 0;
                for (int vi : lv) maxm = std::max(maxm, meta[vi * 4 + 1]);
                const int passes = maxm > kHiTileBits ? (maxm - kHiTileBits + kHiGroup - 1) / kHiGroup : 0;
                std::vector<int> &hm = G.hm;
                hm.assign((size_t)nl + (size_t)(nl + 1) * (1 + passes), 0);
                for (int i = 0; i < nl; ++i) hm[i] = lv[i];
                int *tp = hm.data() + nl;
                for (int i = 0; i < nl; ++i) {
                    const int m = meta[lv[i] * 4 + 1];
                    tp[i + 1] = tp[i] + (m <= kHiTileBits ? 1 : 1 << (m - kHiTileBits));
                }
                for (int pp = 0; pp < passes; ++pp) {
                    int *bp = tp + (size_t)(nl + 1) * (1 + pp);
                    const int bit_lo = kHiTileBits + pp * kHiGroup;
                    for (int i = 0; i < nl; ++i) {
                        const int m = meta[lv[i] * 4 + 1];
                        const int Gb = std::min(kHiGroup, m - bit_lo);
                        bp[i + 1] = bp[i] + (Gb > 0 ? (int)(((1ull << (m - Gb)) + 255) / 256) : 0);
                    }
                }
                ULG_HIP(c, hipMemcpyAsync(G.d_hmeta, hm.data(), hm.size() * 4, hipMemcpyHostToDevice, st));
                HiArgs ha{G.d_hmeta, G.d_hmeta + nl, nl, c->d_meta.p, c->d_tbl_off.p, c->table.p, c->d_binom64.p,
                          c->d_hmax.p, c->d_hmax.p + c->hmax_half, c->d_hoff.p, S, L, kmax, 0};
                prof_begin_s(c, "wide_hicover", st);
                if (ph == 0) hikey_tile_kernel<0><<<tp[nl], 1024, 0, st>>>(ha);
                else hikey_tile_kernel<1><<<tp[nl], 1024, 0, st>>>(ha);
                for (int pp = 0; pp < passes; ++pp) {
                    ha.prefix = G.d_hmeta + nl + (size_t)(nl + 1) * (1 + pp);
                    ha.bit_lo = kHiTileBits + pp * kHiGroup;
                    const int nb = tp[(size_t)(nl + 1) * (1 + pp) + nl];
                    if (nb > 0) hikey_strided_kernel<<<nb, 256, 0, st>>>(ha);
                }
                prof_end_s(c, st);
                ULG_HIP(c, hipGetLastError());
                wa.hmax = c->d_hmax.p;
                wa.pval = c->d_hmax.p + c->hmax_half;
                wa.hoff = c->d_hoff.p;
            }
        }
        // checked bitset: 2^q bits per walking set, q = L (P holds variable 0) or L + 1
        const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(G.qn, slice / wpl));  // slice >= wpl
        unsigned long long *ws = nullptr;
        if (wstat) {
            int rc2;
            if ((rc2 = ensure(c, c->d_stats, 16))) return rc2;
            ws = c->d_stats.p;
            ULG_HIP(c, hipStreamSynchronize(st));
            ULG_HIP(c, hipMemsetAsync(ws, 0, 64, st));
        }
        // long walks move to the LDS kernel (reduced walks with hi-cover tables only)
        budget[gi] = (wa.hoff && wa.reduced && q <= kStragQMax && c->wide_lds)
                         ? (c->wide_lds == 2 ? 1 : strag_budget())
                         : 0;
        uint64_t *sq = G.queue + 3 * G.qn;  // straggler queue after this launch's entries (the queue has room)
        if (budget[gi]) ULG_HIP(c, hipMemsetAsync(G.scnt, 0, 8, st));
        const auto tw0 = std::chrono::steady_clock::now();
        for (uint64_t base = 0; base < G.qn; base += per) {
            const uint64_t k = std::min<uint64_t>(per, G.qn - base);
            ULG_HIP(c, hipMemsetAsync(G.bits, 0, (size_t)(k * wpl * 8), st));
            prof_begin_s(c, ph == 0 ? "walk_wide_var0" : "walk_wide_rest", st);
            hipLaunchKernelGGL(wf, dim3((unsigned)((k + 63) / 64)), dim3(64), 0, st, wa, base, base + k, G.bits, wpl,
                               errf, ws, budget[gi], sq, G.scnt);
            prof_end_s(c, st);
            ULG_HIP(c, hipGetLastError());
        }
        if (budget[gi]) ULG_HIP(c, hipMemcpyAsync(pin + ng + gi, G.scnt, 8, hipMemcpyDeviceToHost, st));
        if (wstat) {
            unsigned long long h[4];
            ULG_HIP(c, hipMemcpyAsync(h, ws, 32, hipMemcpyDeviceToHost, st));
            ULG_HIP(c, hipStreamSynchronize(st));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count();
            std::fprintf(stderr,
                         "walk_stats L=%d phase=%d queued=%llu walks=%llu steps=%llu max=%llu over2^20=%llu "
                         "launch_ms=%.1f\n",
                         L, ph, (unsigned long long)G.qn, h[0], h[1], h[2], h[3], ms);
        }
    }
    // 3. the long walks, replayed in LDS
    for (int gi = 0; gi < ng; ++gi) {
        WideGroup &G = gs[gi];
        if (G.qn == 0 || !budget[gi]) continue;
        ULG_HIP(c, hipStreamSynchronize(G.st));
        const unsigned long long sn = pin[ng + gi];
        if (sn == 0) continue;
        // skip bitset in LDS; the hi bitset too up to q = kStragHiLdsQ, else in
        // this group's checked-bitset slice (free once its walks are done)
        const bool hl = q <= kStragHiLdsQ;
        const uint64_t nw = ((uint64_t)1 << q) >> 6;
        const size_t lds = (size_t)(hl ? 2 : 1) * nw * 8 + 64 * 8 + 64;  // bitsets, xlow, lc
        using LdsFn = void (*)(WideArgs, const uint64_t *, uint64_t *, unsigned long long *, unsigned long long *,
                               uint64_t, uint32_t *, unsigned int *, uint32_t);
        const LdsFn kf = ph == 0 ? (hl ? walk_wide_lds_kernel<0, true> : walk_wide_lds_kernel<0, false>)
                                 : (hl ? walk_wide_lds_kernel<1, true> : walk_wide_lds_kernel<1, false>);
        ULG_HIP(c, hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        const uint64_t per = hl ? sn : std::max<uint64_t>(1, slice / nw);
        unsigned long long *ws = wstat ? c->d_stats.p : nullptr;
        if (wstat) ULG_HIP(c, hipMemsetAsync(ws, 0, 128, G.st));
        const auto tl0 = std::chrono::steady_clock::now();
        // walks past this many iterations finish on the host; with few
        // replays in the launch the host takes them sooner (it runs them in
        // parallel threads, while the GPU's launch time is its longest walk)
        // Host threads take the long walks only of launches with few replays
        // (wide_host_max): with thousands of long walks (C1 at lambda 0.5) a
        // few host threads would queue them behind each other while the GPU
        // runs them all at once (C1 10.7 s GPU-only against 32 s with every
        // launch handing over).
        const uint64_t hbud = sn > c->wide_host_max ? 0
                              : sn <= kHostFewReplays ? std::min<uint64_t>(c->wide_host_iters, kHostFewBudget)
                                                      : c->wide_host_iters;
        // ... and so do launches of few replays over 2^q >= 2^wide_host_q
        // local subsets: at the top layers of the largest candidate sets
        // nearly every replay outlives the LDS budget anyway (C4 v = 23:
        // L >= 15 hands over 13 of 14, 13 of 15, 1 of 1), so its LDS phase is
        // pure latency
        if (hbud && (sn <= c->wide_host_first || (c->wide_host_q > 0 && q >= c->wide_host_q && sn <= 128))) {
            // so few replays that the host takes them all at once: no GPU
            // replay phase (its length is its longest walk's), straight to
            // the fills, the copy and the host threads
            std::vector<uint32_t> all((size_t)sn);
            for (uint32_t j = 0; j < (uint32_t)sn; ++j) all[j] = j;
            const unsigned int n32 = (unsigned int)sn;
            ULG_HIP(c, hipMemcpyAsync(G.hq, all.data(), all.size() * 4, hipMemcpyHostToDevice, G.st));
            ULG_HIP(c, hipMemcpyAsync(G.hqc, &n32, 4, hipMemcpyHostToDevice, G.st));
            int rc2;
            if ((rc2 = host_walks(c, G, L, ph, q, sn, slice, errf))) return rc2;
            continue;
        }
        if (hbud) ULG_HIP(c, hipMemsetAsync(G.hqc, 0, 4, G.st));
        for (uint64_t base = 0; base < sn; base += per) {
            const uint64_t k = std::min<uint64_t>(per, sn - base);
            prof_begin_s(c, "walk_wide_lds", G.st);
            // many short replays: one wave per block, so more walks run at once
            // (the walk is one wave's; waves 1-3 only speed up the fill)
            const unsigned th = sn >= kStragWide ? 64u : (unsigned)kStragThreads;
            hipLaunchKernelGGL(kf, dim3((unsigned)k), dim3(th), lds, G.st, G.wa,
                               G.queue + 3 * (G.qn + base), G.bits, errf, ws, hbud, G.hq, G.hqc, (uint32_t)base);
            prof_end_s(c, G.st);
            ULG_HIP(c, hipGetLastError());
        }
        if (hbud) {
            int rc2;
            if ((rc2 = host_walks(c, G, L, ph, q, sn, slice, errf))) return rc2;
        }
        if (wstat) {
            unsigned long long h[16];
            ULG_HIP(c, hipMemcpyAsync(h, ws, 128, hipMemcpyDeviceToHost, G.st));
            ULG_HIP(c, hipStreamSynchronize(G.st));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl0).count();
            std::fprintf(stderr,
                         "walk_lds_stats L=%d phase=%d q=%d replays=%llu iters=%llu max=%llu fill_max_us=%.1f "
                         "walk_max_us=%.1f launch_ms=%.1f\n",
                         L, ph, q, h[4], h[5], h[6], h[7] / 100.0, h[8] / 100.0, ms);
        }
    }
    // the hi-cover metadata vectors must outlive their copies
    for (int gi = 0; gi < ng; ++gi)
        if (!gs[gi].hm.empty()) ULG_HIP(c, hipStreamSynchronize(gs[gi].st));
    return ULG_OK;
}


// The wide layers L0..kmax of every variable that reaches them, one variable
// per task on G host threads; thread t drives stream gst[t] with stream group
// t's queue, counter, bitset and hi-cover-metadata slices.  Results are the
// grouped form's (a variable's decisions read only its own slabs).
int wide_pool(ulg_ctx *c, int L0, int G, const std::vector<hipStream_t> &gst, int nv, int S, int kmax,
              int max_parents, const std::vector<int> &mv, const std::vector<int> &meta,
              const std::vector<uint64_t> &work, uint64_t wqwords, uint64_t wslice, const std::vector<uint64_t> &hoff,
              size_t nqc) {
    // every stream's earlier layers first (the slabs the wide layers read)
    for (int g = 0; g < G; ++g) ULG_HIP(c, hipStreamSynchronize(gst[g]));
    std::vector<int> order;
    for (int i = 0; i < nv; ++i)
        if (std::min(mv[i], max_parents) >= L0) order.push_back(i);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return mv[a] > mv[b]; });
    // per-variable launch prefixes: [task][L][phase][nv + 1], only variable i counts
    const size_t stride = (size_t)(kmax + 1) * 2 * (nv + 1);
    std::vector<uint64_t> vw(order.size() * stride, 0);
    for (size_t k = 0; k < order.size(); ++k) {
        const int i = order[k];
        for (int L = L0; L <= kmax; ++L)
            for (int ph = 0; ph < 2; ++ph) {
                const uint64_t *w = &work[((size_t)L * 2 + ph) * (nv + 1)];
                uint64_t *o = &vw[k * stride + ((size_t)L * 2 + ph) * (nv + 1)];
                const uint64_t cnt = w[i + 1] - w[i];
                for (int j = 0; j <= nv; ++j) o[j] = j > i ? cnt : 0;
            }
    }
    int rc;
    if ((rc = upload(c, c->d_vwork, c->mir_vwork, vw))) return rc;
    ULG_HIP(c, hipStreamSynchronize(c->stream));  // the other threads' streams read it next
    std::atomic<size_t> next{0};
    std::vector<int> rcs(G, ULG_OK);
    auto run = [&](int t) {
        if (hipSetDevice(c->device) != hipSuccess) {
            rcs[t] = set_err(c, ULG_ERR_HIP, "hipSetDevice failed in a wide-layer thread");
            return;
        }
        for (size_t k = next++; k < order.size(); k = next++) {
            const int i = order[k];
            const int top = std::min(mv[i], max_parents);
            for (int L = L0; L <= top; ++L)
                for (int ph = 0; ph < 2; ++ph) {
                    const size_t wo = ((size_t)L * 2 + ph) * (nv + 1);
                    const uint64_t cnt = vw[k * stride + wo + nv];
                    if (cnt == 0) continue;
                    WideGroup wg;
                    wg.st = gst[t];
                    wg.d_work = c->d_vwork.p + k * stride + wo;
                    wg.h_work = vw.data() + k * stride + wo;
                    wg.cnt = cnt;
                    wg.queue = c->d_wqueue.p + t * wqwords;
                    wg.qc = c->d_qcount.p + (size_t)t * 2 * (kmax + 1) + (L * 2 + ph);
                    wg.scnt = c->d_scount.p + t;
                    wg.bits = c->d_wbits.p + (size_t)t * wslice;
                    wg.d_hmeta = hoff.empty() ? nullptr : c->d_hmeta.p + (size_t)t * (nv + (size_t)(nv + 1) * 8);
                    wg.hq = c->d_hq.p + (size_t)t * std::max<uint64_t>(wqwords / 6, 1);
                    wg.hqc = c->d_hqc.p + t;
                    // this slot's counter served the previous variable's launch
                    if (hipMemsetAsync(wg.qc, 0, 8, wg.st) != hipSuccess) {
                        rcs[t] = set_err(c, ULG_ERR_HIP, "hipMemsetAsync failed in a wide-layer thread");
                        return;
                    }
                    std::vector<WideGroup> one{std::move(wg)};
                    const int r = score_wide_groups(c, L, ph, one, nv, S, kmax, c->d_qcount.p + nqc - 1, wslice, hoff,
                                                    meta, c->wide_pinned + 2 * t);
                    if (r) {
                        rcs[t] = r;
                        next = order.size();  // the other threads stop at their next task
                        return;
                    }
                }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < G; ++t) th.emplace_back(run, t);
    run(0);
    for (auto &x : th) x.join();
    for (int r : rcs)
        if (r) return r;
    return ULG_OK;
}

}  // namespace

namespace {
uint64_t dbits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
}  // namespace

extern "C" {

int ulg_cbic_load(ulg_ctx *c, const double *data, int64_t N, int n, double lambda) {
    if (!c || !data || N < 2 || n < 1 || n > kMaxVars) return set_err(c, ULG_ERR_ARG, "ulg_cbic_load: bad arguments");
    ULG_HIP(c, hipSetDevice(c->device));
    c->loaded = false;
    c->scored = false;
    c->n = n;
    c->N = N;
    c->lambda = lambda;
    c->npad = (n + 15) / 16 * 16;
    const int tiles = c->npad / 16;
    const int chunks = (int)((N + kGramRows - 1) / kGramRows);
    int rc;
    if ((rc = ensure(c, c->raw, (size_t)(N * n))) || (rc = ensure(c, c->z, (size_t)(N * c->npad))) ||
        (rc = ensure(c, c->gram, (size_t)(n * n))) || (rc = ensure(c, c->colstat, (size_t)(2 * n))) ||
        (rc = ensure(c, c->partials, (size_t)chunks * tiles * tiles * 256)))
        return rc;
    ULG_HIP(c, hipMemcpyAsync(c->raw.p, data, sizeof(double) * (size_t)(N * n), hipMemcpyHostToDevice, c->stream));
    prof_begin(c, "colstats");
    colstats_kernel<<<n, kBlock, 0, c->stream>>>(c->raw.p, N, c->colstat.p);
    prof_end(c);
    const int64_t tot = N * c->npad;
    prof_begin(c, "normalise");
    normalise_kernel<<<(unsigned)((tot + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(c->raw.p, N, n, c->npad,
                                                                                         c->colstat.p, c->z.p);
    prof_end(c);
    prof_begin(c, "gram_mfma_f64");
    gram_mfma_kernel<<<dim3(chunks, tiles * tiles), 64, 0, c->stream>>>(c->z.p, N, c->npad, tiles, c->partials.p);
    prof_end(c);
    prof_begin(c, "gram_reduce");
    gram_reduce_kernel<<<(n * n + kBlock - 1) / kBlock, kBlock, 0, c->stream>>>(c->partials.p, chunks, tiles, n,
                                                                               c->gram.p);
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    c->loaded = true;
    return ULG_OK;
}

int ulg_cbic_gram(ulg_ctx *c, double *out) {
    if (!c || !out) return ULG_ERR_ARG;
    if (!c->loaded) return set_err(c, ULG_ERR_STATE, "ulg_cbic_gram: no data loaded");
    ULG_HIP(c, hipSetDevice(c->device));
    ULG_HIP(c, hipMemcpy(out, c->gram.p, sizeof(double) * (size_t)(c->n * c->n), hipMemcpyDeviceToHost));
    return ULG_OK;
}

static int cbic_score(ulg_ctx *c, const int *vars, int nv, const uint64_t *candidates, int max_parents,
                      int64_t *total_stored, int64_t *total_scored, bool async);

// ULG_WALK_CLOCK diagnostics: every walk wave's start / end clock and its
// union points (steps) into <dir>/sliced_L<L>_p<phase>.bin (synchronising)
static int dump_walk_clock(ulg_ctx *c, hipStream_t st, uint64_t sb, const char *dir, int L, int ph) {
    std::vector<uint64_t> hw((size_t)3 * sb);
    ULG_HIP(c, hipMemcpyAsync(hw.data(), c->d_dump.p, hw.size() * 8, hipMemcpyDeviceToHost, st));
    ULG_HIP(c, hipStreamSynchronize(st));
    char fn[512];
    std::snprintf(fn, sizeof fn, "%s/sliced_L%d_p%d.bin", dir, L, ph);
    if (FILE *f = std::fopen(fn, "wb")) {
        std::fwrite(hw.data(), 8, hw.size(), f);
        std::fclose(f);
    }
    return ULG_OK;
}

// Diagnostics (ULG_WALK_CLOCK with ULG_WALK_QUEUE_DUMP, after a layer's walk
// launch): the walk queue of that launch, compacted, with each entry's
// decision as the walk left it in the table -- scripts/walk_sched_study.cpp
// replays the walks offline.  File: nseg, W, then per segment its count,
// count x (1 + 2W) entry words and count decision words (the table's bits at
// the entry's slot).
static int dump_walk_queue(ulg_ctx *c, hipStream_t st, const uint64_t *queue, const unsigned long long *qc,
                           uint64_t nseg, int W, uint64_t nslots, const char *dir, int L, int ph) {
    std::vector<unsigned long long> cnt(nseg * kSegStride);
    ULG_HIP(c, hipMemcpyAsync(cnt.data(), qc, cnt.size() * 8, hipMemcpyDeviceToHost, st));
    ULG_HIP(c, hipStreamSynchronize(st));
    char fn[512];
    std::snprintf(fn, sizeof fn, "%s/queue_L%d_p%d.bin", dir, L, ph);
    FILE *f = std::fopen(fn, "wb");
    if (!f) return ULG_OK;
    const uint64_t hdr[2] = {nseg, (uint64_t)W};
    std::fwrite(hdr, 8, 2, f);
    const uint64_t ew = 1 + 2 * (uint64_t)W;
    std::vector<uint32_t> tab((size_t)nslots);
    ULG_HIP(c, hipMemcpyAsync(tab.data(), reinterpret_cast<const uint32_t *>(c->table.p), tab.size() * 4,
                              hipMemcpyDeviceToHost, st));
    ULG_HIP(c, hipStreamSynchronize(st));
    for (uint64_t s = 0; s < nseg; ++s) {
        const uint64_t n = std::min<uint64_t>(cnt[s * kSegStride], kSegEntries);
        std::vector<uint64_t> e(n * ew);
        std::vector<uint32_t> d(n);
        if (n) {
            ULG_HIP(c, hipMemcpyAsync(e.data(), queue + s * kSegEntries * ew, e.size() * 8, hipMemcpyDeviceToHost, st));
            ULG_HIP(c, hipStreamSynchronize(st));
            for (uint64_t i = 0; i < n; ++i) {
                const uint32_t slot = (uint32_t)e[i * ew];
                d[i] = slot < tab.size() ? tab[slot] : 0u;
            }
        }
        std::fwrite(&n, 8, 1, f);
        std::fwrite(e.data(), 8, e.size(), f);
        std::fwrite(d.data(), 4, d.size(), f);
    }
    std::fclose(f);
    return ULG_OK;
}

// The call's error word (kErr* bits) as a status.
static int call_error(ulg_ctx *c, unsigned long long w) {
    c->last_err_word = w;
    if (w & kErrWide)
        return set_err(c, ULG_ERR_UNSUPPORTED,
                       "ulg_cbic_score: a find_best_subset_score walk in a wide layer exceeded its cap (2^30 steps "
                       "in walk_wide_kernel, 2^32 iterations or 24 frames in the LDS / host replay)");
    if (w & (kErrQueue | kErrSlot))
        return set_err(c, ULG_ERR_STATE,
                       (w & kErrQueue) ? "ulg_cbic_score: a walk-queue segment overflowed (internal sizing error)"
                                       : "ulg_cbic_score: a walk entry named a slot past the call's table");
    return ULG_OK;
}

int ulg_cbic_score_finish(ulg_ctx *c, int64_t *total_stored, int64_t *total_scored) {
    if (!c) return ULG_ERR_ARG;
    if (c->async_pending) {
        c->async_pending = false;
        ULG_HIP(c, hipSetDevice(c->device));
        ULG_HIP(c, hipStreamSynchronize(c->stream));
        prof_collect(c);
        c->total_stored = (int64_t)c->async_pinned[0];
        c->last_err_word = c->async_pinned[1];
        if (int rc = call_error(c, c->async_pinned[1])) {
            c->scored = false;
            return rc;
        }
    }
    if (!c->scored) return set_err(c, ULG_ERR_STATE, "ulg_cbic_score_finish: nothing scored");
    if (total_stored) *total_stored = c->total_stored;
    if (total_scored) *total_scored = c->total_scored;
    return ULG_OK;
}

int ulg_cbic_score(ulg_ctx *c, const int *vars, int nv, const uint64_t *candidates, int max_parents,
                   int64_t *total_stored, int64_t *total_scored) {
    return cbic_score(c, vars, nv, candidates, max_parents, total_stored, total_scored, false);
}

int ulg_cbic_score_async(ulg_ctx *c, const int *vars, int nv, const uint64_t *candidates, int max_parents) {
    return cbic_score(c, vars, nv, candidates, max_parents, nullptr, nullptr, true);
}

static int cbic_score(ulg_ctx *c, const int *vars, int nv, const uint64_t *candidates, int max_parents,
                      int64_t *total_stored, int64_t *total_scored, bool async) {
    if (!c) return ULG_ERR_ARG;
    if (c->async_pending) {  // the previous async call's launches still own the buffers
        int rc0 = ulg_cbic_score_finish(c, nullptr, nullptr);
        if (rc0) return rc0;
    }
    if (!c->loaded) return set_err(c, ULG_ERR_STATE, "ulg_cbic_score: call ulg_cbic_load first");
    if (!vars || !candidates || nv < 1 || nv > c->n) return set_err(c, ULG_ERR_ARG, "ulg_cbic_score: bad variable list");
    ULG_HIP(c, hipSetDevice(c->device));
    const int n = c->n;
    uint64_t seen = 0;
    for (int i = 0; i < nv; ++i) {
        if (vars[i] < 0 || vars[i] >= n || ((seen >> vars[i]) & 1ull))
            return set_err(c, ULG_ERR_ARG, "ulg_cbic_score: variables must be distinct and < n");
        seen |= 1ull << vars[i];
    }
    const uint64_t allmask = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    if (max_parents < 1 || max_parents > n - 1) max_parents = n - 1;
    // per-variable candidate lists (the variable itself never enters a set,
    // score_calculator.cpp:100)
    std::vector<uint8_t> cand((size_t)nv * 64, 0);
    std::vector<int> meta((size_t)nv * 4, 0);
    std::vector<int> mv(nv);
    int kmax = 0;
    for (int i = 0; i < nv; ++i) {
        const uint64_t C = candidates[i] & allmask & ~(1ull << vars[i]);
        int m = 0;
        for (int b = 0; b < n; ++b)
            if ((C >> b) & 1ull) cand[(size_t)i * 64 + m++] = (uint8_t)b;
        mv[i] = m;
        meta[i * 4 + 0] = vars[i];
        meta[i * 4 + 1] = m;
        meta[i * 4 + 2] = (C & 1ull) ? 1 : 0;  // variable 0 is a candidate (compact index 0)
        kmax = std::max(kmax, std::min(m, max_parents));
    }
    if (kmax > kWideMax)
        return set_err(c, ULG_ERR_UNSUPPORTED,
                       "ulg_cbic_score: parent sets larger than ULG_MAX_PARENTS_GPU (31) are not supported");
    const int S = kmax + 1;
    // slab offsets: (vi, L) -> start, final sentinel = total slots
    std::vector<uint64_t> toff((size_t)nv * S + 1);
    uint64_t acc = 0;
    int64_t scored = 0;
    for (int i = 0; i < nv; ++i)
        for (int L = 0; L < S; ++L) {
            toff[(size_t)i * S + L] = acc;
            const uint64_t cnt = (L <= max_parents) ? binom64(mv[i], L) : 0;
            acc += cnt;
            scored += (int64_t)cnt;
        }
    toff[(size_t)nv * S] = acc;
    const uint64_t total_slots = acc;
    // per launch work prefixes: [L][phase][nv+1]
    std::vector<uint64_t> work((size_t)(kmax + 1) * 2 * (nv + 1), 0);
    for (int L = 1; L <= kmax; ++L)
        for (int ph = 0; ph < 2; ++ph) {
            uint64_t *w = &work[((size_t)L * 2 + ph) * (nv + 1)];
            uint64_t s = 0;
            for (int i = 0; i < nv; ++i) {
                w[i] = s;
                const bool z = meta[i * 4 + 2] != 0;
                uint64_t cnt;
                if (L > max_parents) cnt = 0;
                else if (ph == 0) cnt = z ? binom64(mv[i] - 1, L - 1) : 0;
                else cnt = z ? binom64(mv[i] - 1, L) : binom64(mv[i], L);
                s += cnt;
            }
            w[nv] = s;
        }
    int rc;
    // the output lists are sized for every slot, so the compaction needs no
    // mid-call sync for the stored count
    if ((rc = ensure(c, c->table, total_slots)) || (rc = upload(c, c->d_tbl_off, c->mir_tbl_off, toff)) ||
        (rc = upload(c, c->d_work, c->mir_work, work)) || (rc = upload(c, c->d_cand, c->mir_cand, cand)) ||
        (rc = upload(c, c->d_meta, c->mir_meta, meta)) || (rc = ensure(c, c->out_sets, total_slots)) ||
        (rc = ensure(c, c->out_scores, total_slots)) || (rc = ensure(c, c->out_offsets, (size_t)nv + 1)))
        return rc;

    ScoreArgs sa;
    sa.hsub_out = 1;
    sa.gram = c->gram.p;
    sa.binom = c->d_binom.p;
    sa.cand = c->d_cand.p;
    sa.meta = c->d_meta.p;
    sa.tbl_off = c->d_tbl_off.p;
    sa.table = c->table.p;
    sa.hsub = nullptr;
    sa.queue = nullptr;
    sa.qcount = nullptr;
    sa.err = nullptr;
    sa.qkey = nullptr;
    sa.N = (double)c->N;
    sa.lambda = c->lambda;
    sa.n = n;
    sa.nv = nv;
    sa.S = S;
    sa.xcd = c->score_xcd;
    // tables of 2^30 slots or more: the one-pass form with 64-bit slots (the
    // others keep 32-bit byte offsets in their gathers and slots in entries)
    const int variant = (total_slots >> 30) ? 1 : c->score_variant;
    if (variant & 64) {
        if ((rc = ensure(c, c->d_hsub, total_slots))) return rc;
        sa.hsub = c->d_hsub.p;
    }
    const char *wck = std::getenv("ULG_WALK_CLOCK");  // walk diagnostics (synchronising)
    // Variables never read each other's slabs, so they are striped over G
    // groups on concurrent streams: a group's latency-bound walk kernels
    // overlap the other groups' scoring kernels.  Diagnostics run on one.
    const int G = ((variant & 16) && !wck) ? std::max(1, std::min(c->score_streams, nv)) : 1;
    while ((int)c->aux_streams.size() < G - 1) {
        hipStream_t st;
        ULG_HIP(c, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        c->aux_streams.push_back(st);
    }
    while ((int)c->sync_events.size() < 2 * G) {
        hipEvent_t ev;
        ULG_HIP(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->sync_events.push_back(ev);
    }
    std::vector<hipStream_t> gst(G);
    gst[0] = c->stream;
    for (int g = 1; g < G; ++g) gst[g] = c->aux_streams[g - 1];
    // per group work prefixes (variables outside the group count 0 sets)
    const size_t wstride = (size_t)(kmax + 1) * 2 * (nv + 1);
    std::vector<uint64_t> workg(G == 1 ? 0 : (size_t)G * wstride, 0);
    if (G > 1) {
        for (int g = 0; g < G; ++g)
            for (int L = 1; L <= kmax; ++L)
                for (int ph = 0; ph < 2; ++ph) {
                    const uint64_t *w = &work[((size_t)L * 2 + ph) * (nv + 1)];
                    uint64_t *wg = &workg[(size_t)g * wstride + ((size_t)L * 2 + ph) * (nv + 1)];
                    uint64_t acc2 = 0;
                    for (int i = 0; i < nv; ++i) {
                        wg[i] = acc2;
                        if (i % G == g) acc2 += w[i + 1] - w[i];
                    }
                    wg[nv] = acc2;
                }
        if ((rc = upload(c, c->d_workg, c->mir_workg, workg))) return rc;
    }
    const uint64_t *d_wk = G > 1 ? c->d_workg.p : c->d_work.p;
    const std::vector<uint64_t> &h_wk = G > 1 ? workg : work;
    uint64_t qwords = 0;   // per group: every lane of its largest launch may be queued
    uint64_t wqwords = 0;  // the same for the wide layers' queue (3 words per set)
    for (int g = 0; g < G; ++g)
        for (int L = 1; L <= kmax; ++L)
            for (int ph = 0; ph < 2; ++ph) {
                const uint64_t cnt = h_wk[(size_t)g * (G > 1 ? wstride : 0) + ((size_t)L * 2 + ph) * (nv + 1) + nv];
                if (L > kMaxL) wqwords = std::max<uint64_t>(wqwords, 6 * cnt);  // entries + straggler copies
                else if (variant & 16)
                    qwords = std::max<uint64_t>(qwords, seg_count((cnt + kBlock - 1) / kBlock) * kSegEntries *
                                                            (uint64_t)(1 + 2 * bits_words(L)));
            }
    // walk-queue segment counters per (group, layer, phase) of the unrolled
    // two-pass launches (queue_walk), kSegStride words each
    const size_t nseg_slots = (size_t)G * 2 * (kmax + 1);
    std::vector<uint64_t> segoff(nseg_slots + 1, 0);
    for (size_t i = 0; i < nseg_slots; ++i) {
        const int g = (int)(i / (2 * (size_t)(kmax + 1))), L = (int)((i / 2) % (size_t)(kmax + 1)), ph = (int)(i % 2);
        const uint64_t cnt = h_wk[(size_t)g * (G > 1 ? wstride : 0) + ((size_t)L * 2 + ph) * (nv + 1) + nv];
        const bool queued = L >= 1 && L <= kMaxL && (variant & 16);
        const bool bhdr = queued && (L == 5 || L == 6);  // room for a walk_bucket header
        segoff[i + 1] = segoff[i] + (queued ? seg_count((cnt + kBlock - 1) / kBlock) * kSegStride : 0) +
                        (bhdr && cnt ? kBucketHdrWords : 0);
    }
    // queue counters per (group, layer, phase), then the wide walks' error flag
    const size_t nqc = (size_t)G * 2 * (kmax + 1) + 1;
    if ((variant & 16) || kmax > kMaxL) {
        if ((rc = ensure(c, c->d_queue, (size_t)G * qwords)) || (rc = ensure(c, c->d_qcount, nqc)) ||
            (rc = ensure(c, c->d_wqueue, (size_t)G * wqwords)))
            return rc;
        if ((rc = ensure(c, c->d_qseg, (size_t)std::max<uint64_t>(segoff.back(), 1)))) return rc;
    }
    // bucketed walk launches (walk_bucket, layers 5 and 6): per stream group a
    // key/rank word and a sorted index per queue entry, the (key, segment)
    // offsets and the wave table
    const bool bucket = (variant & 112) == 112 && c->walk_bucket && !wck && kmax >= 5;  // the CMP path queues with keys
    const uint64_t qcap = (qwords / 3 + 255) & ~255ull;  // queue entries per group (an entry is >= 3 words), 256-aligned
    uint64_t nseg_max = 1;
    for (int g = 0; g < G; ++g)
        for (int L = 5; L <= std::min(kmax, 6); ++L)
            for (int ph = 0; ph < 2; ++ph) {
                const uint64_t cnt = h_wk[(size_t)g * (G > 1 ? wstride : 0) + ((size_t)L * 2 + ph) * (nv + 1) + nv];
                nseg_max = std::max<uint64_t>(nseg_max, seg_count((cnt + kBlock - 1) / kBlock));
            }
    const uint64_t wave_cap = qcap / 64 + kBucketMax;  // walk waves of a bucketed launch, at most
    if (bucket) {
        if ((rc = ensure(c, c->d_qkey, (size_t)(G * qcap))) || (rc = ensure(c, c->d_qaux, (size_t)(G * qcap))) ||
            (rc = ensure(c, c->d_qsidx, (size_t)(G * qcap))) ||
            (rc = ensure(c, c->d_qoffs, (size_t)(G * kBucketMax * nseg_max))))
            return rc;
    }
    // zeroed by call_prologue_kernel (the first launch of the sequence below)
    const bool zero_q = (variant & 16) || kmax > kMaxL;
    const uint64_t nqseg = zero_q ? std::max<uint64_t>(segoff.back(), 1) : 0;
    sa.err = zero_q ? c->d_qcount.p + nqc - 1 : nullptr;
    // wide-layer walks: one checked-bitset slice per stream group, allocated
    // before any launch (2^q bits per walking set, q <= kmax + 1)
    uint64_t wslice = 0;
    std::vector<uint64_t> hoff;
    if (kmax > kMaxL) {
        const uint64_t wpl_max = kmax + 1 <= 6 ? 1ull : (1ull << (kmax + 1 - 6));
        wslice = std::max<uint64_t>(kWideBitsWords / (uint64_t)G, wpl_max);
        if ((rc = ensure(c, c->d_wbits, (size_t)(G * wslice))) || (rc = ensure(c, c->d_scount, (size_t)G)) ||
            (rc = ensure(c, c->d_hq, (size_t)G * std::max<uint64_t>(wqwords / 6, 1))) ||
            (rc = ensure(c, c->d_hqc, (size_t)G)))
            return rc;
        // hi-cover tables for the variables that reach a wide layer
        if (c->wide_prune) {
            hoff.assign(nv, ~0ull);
            uint64_t htot = 0;
            for (int i = 0; i < nv; ++i)
                if (std::min(mv[i], max_parents) > kMaxL && mv[i] <= kHiMaxBits) {
                    hoff[i] = htot;
                    htot += 1ull << mv[i];
                }
            if (htot > 0) {
                c->hmax_half = htot;  // d_hmax = [hi-cover maxima][present values]
                if ((rc = ensure(c, c->d_hmax, (size_t)(2 * htot))) || (rc = upload(c, c->d_hoff, c->mir_hoff, hoff)) ||
                    (rc = ensure(c, c->d_hmeta, (size_t)G * (nv + (size_t)(nv + 1) * 8))))
                    return rc;
            } else {
                hoff.clear();
            }
        }
    }
    if (kmax > kMaxL && (int)c->wide_host.size() < 2 * G) {
        if (c->wide_pinned) (void)hipHostFree(c->wide_pinned);
        c->wide_pinned = nullptr;
        ULG_HIP(c, hipHostMalloc((void **)&c->wide_pinned, sizeof(unsigned long long) * 2 * (size_t)G,
                                 hipHostMallocDefault));
        c->wide_host.assign(2 * G, 0);
    }
    // Small layers (L <= Ls, little work, latency-bound): one one-pass launch
    // per phase over all variables on the context stream -- no queue, no walk
    // launch, no stream groups.  The rest: per group, score + queued walk.
    const int Ls = (variant & 16) && !wck ? std::min(kmax, std::min(kMaxL, c->score_small_layers)) : 0;
    const int vsmall = variant & 65;  // the one-pass form (keeping the subset maxima under bit 6)
    // ... of which layers <= Lf in one launch, a workgroup per variable
    // (not under -r: the budget is checked after every layer, and a fused
    // launch would finish layers 2..Lf before the first check)
    const int Lf = vsmall == 65 && c->time_limit_ms == 0 ? std::min(Ls, c->score_fused) : 0;
    bool forked = false;
    // The wide layers variable by variable (wide_pool 1) pay when the
    // variables that reach them differ in size: the long replays of one then
    // hold no other's next layer (C4: 2-hop sets of 10..18 candidates).  On
    // equal candidate sets (C1: a full skeleton) the grouped form's larger
    // launches keep more replays in flight (C1 at lambda 0.5: 10.7 s against
    // 15.2 s).  wide_pool 2 (default) picks the pool when the wide variables'
    // candidate counts span at least 2.
    bool use_pool = c->wide_pool == 1;
    if (c->wide_pool == 2) {
        int lo_m = 64, hi_m = -1;
        for (int i = 0; i < nv; ++i)
            if (std::min(mv[i], max_parents) > kMaxL) {
                lo_m = std::min(lo_m, mv[i]);
                hi_m = std::max(hi_m, mv[i]);
            }
        use_pool = hi_m >= 0 && hi_m - lo_m >= 2;
    }
    // -r (score_calculator.cpp:33-52,78): checked after every complete layer
    const auto t_call = std::chrono::steady_clock::now();
    c->out_of_time = 0;
    int done_L = kmax;
    const int64_t nb = (int64_t)((total_slots + kSlotsPerBlock - 1) / kSlotsPerBlock);
    if ((rc = ensure(c, c->d_blk, (size_t)nb + 2))) return rc;
    // The launch sequence from here to write_kernel has no host sync when
    // every layer is unrolled and no budget / diagnostic is on, and it is the
    // same on every call with the same variables, limits and buffers: it is
    // captured once into a hipGraph (all stream groups, the fork and join
    // events, the profiling events) and replayed, which removes the host
    // launch path of ~40 kernels per call (score_graph, default on).
    const bool use_graph =
        c->score_graph && !c->prof && kmax <= kMaxL && c->time_limit_ms == 0 && !wck;
    std::vector<uint64_t> gkey;
    // An early return between BeginCapture and EndCapture (a failed launch,
    // "layer too large") must not leave the context stream capturing: the
    // guard ends the capture, drops the partial graph and the key.
    struct CaptureGuard {
        ulg_ctx *c;
        bool active;
        ~CaptureGuard() {
            if (!active) return;
            hipGraph_t g = nullptr;
            (void)hipStreamEndCapture(c->stream, &g);
            if (g) (void)hipGraphDestroy(g);
            c->gkey.clear();
            (void)hipGetLastError();
        }
    } capture_guard{c, false};
    if (use_graph) {
        gkey.assign({(uint64_t)nv, (uint64_t)max_parents, (uint64_t)variant, (uint64_t)G, (uint64_t)Ls,
                     (uint64_t)c->score_xcd, (uint64_t)n, (uint64_t)c->N, dbits(c->lambda), (uint64_t)c->prof,
                     (uint64_t)c->walk_small_sets, (uint64_t)c->walk_k6,
                     (uint64_t)c->walk_bucket, (uint64_t)(uintptr_t)c->d_qaux.p, (uint64_t)(uintptr_t)c->d_qsidx.p,
                     (uint64_t)(uintptr_t)c->d_qkey.p,
                     (uint64_t)(uintptr_t)c->d_qoffs.p,
                     (uint64_t)(uintptr_t)c->table.p, (uint64_t)(uintptr_t)c->d_work.p,
                     (uint64_t)(uintptr_t)c->d_workg.p, (uint64_t)(uintptr_t)c->d_queue.p,
                     (uint64_t)(uintptr_t)c->d_qcount.p, (uint64_t)(uintptr_t)c->d_qseg.p, (uint64_t)(uintptr_t)c->d_cand.p,
                     (uint64_t)(uintptr_t)c->d_meta.p, (uint64_t)(uintptr_t)c->d_tbl_off.p,
                     (uint64_t)(uintptr_t)c->out_sets.p, (uint64_t)(uintptr_t)c->out_scores.p,
                     (uint64_t)(uintptr_t)c->out_offsets.p, (uint64_t)(uintptr_t)c->d_blk.p,
                     (uint64_t)(uintptr_t)c->gram.p, (uint64_t)(uintptr_t)c->d_binom.p,
                     (uint64_t)(uintptr_t)c->d_binom64.p, (uint64_t)(uintptr_t)c->d_hsub.p, (uint64_t)total_slots,
                     (uint64_t)c->score_small_layers, (uint64_t)c->score_fused});
        for (int i = 0; i < nv; ++i) gkey.push_back((uint64_t)vars[i]);
        for (int i = 0; i < nv; ++i) gkey.push_back(candidates[i]);
        for (const std::string &nm : c->prof_only) gkey.push_back(std::hash<std::string>{}(nm));
        if (c->gexec && gkey == c->gkey) {
            c->completed_layer = kmax;
            ULG_HIP(c, hipGraphLaunch(c->gexec, c->stream));
            for (const ProfRec &r : c->gprof) c->pending.push_back(r);
            goto launched;
        }
        graph_reset(c);
        ULG_HIP(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed));
        capture_guard.active = true;
    }
    {
    const size_t pend0 = c->pending.size();
    {
        const uint64_t nz = std::max<uint64_t>((uint64_t)nv, std::max<uint64_t>(zero_q ? nqc : 0, nqseg));
        prof_begin(c, "call_prologue");
        call_prologue_kernel<<<(unsigned)((nz + 255) / 256), 256, 0, c->stream>>>(
            c->d_tbl_off.p, nv, S, c->table.p, zero_q ? c->d_qcount.p : nullptr, zero_q ? nqc : 0,
            zero_q ? c->d_qseg.p : nullptr, nqseg);
        prof_end(c);
    }
    for (int L = 1; L <= kmax; ++L) {
        for (int ph = 0; ph < 2; ++ph) {
            if (L <= Lf) {
                if (L == 1 && ph == 0) {
                    ScoreArgs ss = sa;
                    ss.work = nullptr;
                    ss.queue = nullptr;
                    ss.qcount = nullptr;
                    ss.hsub_out = Lf < kmax;  // layer Lf's phase 1 maxima: read only by a layer above
                    const LdsLayout lay = lds_layout(n, nv, S, Lf, 65);
                    const SmallFn kfn = small_kernel(Lf);
                    if (lay.total > 64 * 1024)
                        ULG_HIP(c, hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       lay.total));
                    prof_begin_s(c, "score_small_fused", c->stream);
                    hipLaunchKernelGGL(kfn, dim3((unsigned)nv), dim3(kFusedThreads), (size_t)lay.total, c->stream, ss,
                                       (const uint64_t *)c->d_work.p);
                    prof_end_s(c, c->stream);
                }
                continue;
            }
            if (L <= Ls) {
                const size_t wo = ((size_t)L * 2 + ph) * (nv + 1);
                const uint64_t cnt = work[wo + nv];
                if (cnt == 0) continue;
                ScoreArgs ss = sa;
                ss.work = c->d_work.p + wo;
                ss.queue = nullptr;
                ss.qcount = nullptr;
                ss.hsub_out = !(L == kmax && ph == 1);
                const LdsLayout lay = lds_layout(n, nv, S, L, vsmall);
                const KernelFn kfn = layer_kernel(L, ph, vsmall);
                if (lay.total > 64 * 1024)
                    ULG_HIP(c, hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, lay.total));
                prof_begin_s(c, kLayerNames[ph][L], c->stream);
                hipLaunchKernelGGL(kfn, dim3((unsigned)((cnt + kBlock - 1) / kBlock)), dim3(kBlock), (size_t)lay.total,
                                   c->stream, ss);
                prof_end_s(c, c->stream);
                continue;
            }
            // fork: the side streams start after the uploads / empty-set
            // kernel / small layers
            if (G > 1 && !forked) {
                ULG_HIP(c, hipEventRecord(c->sync_events[0], c->stream));
                for (int g = 1; g < G; ++g) ULG_HIP(c, hipStreamWaitEvent(gst[g], c->sync_events[0], 0));
                forked = true;
            }
            if (L > kMaxL && G > 1 && c->time_limit_ms == 0 && use_pool) {
                // The wide layers variable by variable on G host threads (one
                // stream each): a variable's layers depend only on its own
                // lower layers, and the long LDS replays of one variable no
                // longer hold every other variable's next layer (the grouped
                // form waits for each layer's slowest group).  Largest
                // candidate sets first.
                if ((rc = wide_pool(c, L, G, gst, nv, S, kmax, max_parents, mv, meta, work, wqwords, wslice, hoff,
                                    nqc)))
                    return rc;
                break;
            }
            std::vector<WideGroup> wide;  // a wide layer: every group's part, staged together
            for (int g = 0; g < G; ++g) {
                const size_t wo = (size_t)g * (G > 1 ? wstride : 0) + ((size_t)L * 2 + ph) * (nv + 1);
                const uint64_t cnt = h_wk[wo + nv];
                if (cnt == 0) continue;
                hipStream_t st = gst[g];
                sa.work = d_wk + wo;
                unsigned long long *qc =
                    (variant & 16) ? c->d_qseg.p + segoff[(size_t)g * 2 * (kmax + 1) + (size_t)L * 2 + ph] : nullptr;
                sa.queue = (variant & 16) ? c->d_queue.p + (size_t)g * qwords : nullptr;
                sa.qcount = qc;
                const bool bk = bucket && (L == 5 || L == 6);
                sa.qkey = bk ? c->d_qkey.p + (size_t)g * qcap : nullptr;
                // nothing reads the subset maxima of the top layer's second phase
                sa.hsub_out = !(L == kmax && ph == 1);
                const uint64_t blocks = (cnt + kBlock - 1) / kBlock;
                if (blocks > 0x7fffffffull) return set_err(c, ULG_ERR_UNSUPPORTED, "ulg_cbic_score: layer too large");
                if (L > kMaxL) {
                    WideGroup wg;
                    wg.st = st;
                    wg.d_work = d_wk + wo;
                    wg.h_work = h_wk.data() + wo;
                    wg.cnt = cnt;
                    wg.queue = c->d_wqueue.p + g * wqwords;
                    wg.qc = c->d_qcount.p + (size_t)g * 2 * (kmax + 1) + (L * 2 + ph);
                    wg.scnt = c->d_scount.p + g;
                    wg.bits = c->d_wbits.p + (size_t)g * wslice;
                    wg.d_hmeta = hoff.empty() ? nullptr : c->d_hmeta.p + (size_t)g * (nv + (size_t)(nv + 1) * 8);
                    wg.hq = c->d_hq.p + (size_t)g * std::max<uint64_t>(wqwords / 6, 1);
                    wg.hqc = c->d_hqc.p + g;
                    wide.push_back(std::move(wg));
                    continue;
                }
                const LdsLayout lay = lds_layout(n, nv, S, L, variant);
                const KernelFn kfn = layer_kernel(L, ph, variant);
                if (lay.total > 64 * 1024)
                    ULG_HIP(c, hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, lay.total));
                prof_begin_s(c, kLayerNames[ph][L], st);
                hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(kBlock), (size_t)lay.total, st, sa);
                prof_end_s(c, st);
                if (variant & 16) {
                    // the undecided lanes of this launch, densely packed
                    const int wk = sliced_k(L, cnt, (uint64_t)c->walk_small_sets, c->walk_k6);
                    if (bk) {
                        // counting sort of the queue by walk key, then the table's waves
                        const uint64_t nseg = seg_count(blocks);
                        const int kl = L == 6 ? (wk >= 8 ? 8 : 4) : (wk >= 4 ? 4 : 2);
                        uint32_t *kbase = c->d_qoffs.p + (size_t)g * kBucketMax * nseg_max;
                        uint32_t *sidx = c->d_qsidx.p + (size_t)g * qcap;
                        uint32_t *qaux = c->d_qaux.p + (size_t)g * qcap;
                        const unsigned int *hdr = reinterpret_cast<const unsigned int *>(qc + nseg * kSegStride);
                        // the profiled walk time includes the sort (count + scatter)
                        prof_begin_s(c, kWalkNames[ph][L], st);
                        walk_bucket_count_kernel<<<(unsigned)((nseg + kBucketSegs - 1) / kBucketSegs), 256, 0, st>>>(
                            qc, (uint32_t)nseg, L, sa.qkey, qaux, kbase);
                        const uint64_t items = nseg * (kSegEntries / 256);
                        walk_bucket_scatter_kernel<<<(unsigned)std::min<uint64_t>(items, 2048), 256, 0, st>>>(
                            qc, qaux, kbase, (uint32_t)nseg, L, sidx);
                        hipLaunchKernelGGL(bucket_fn(L, ph, kl), dim3((unsigned)std::min<uint64_t>(wave_cap, 4096)),
                                           dim3(64), 0, st, (const uint64_t *)sa.queue, (const uint32_t *)sidx, hdr,
                                           c->table.p, sa.hsub_out ? sa.hsub : nullptr, total_slots, sa.err);
                        prof_end_s(c, st);
                    } else if ((variant & 32) && sliced_fn(L, ph, wk)) {
                        // one wave per (queue segment, chunk of 64 * K entries)
                        const int kk = L == 7 ? 2 : (L == 8 ? 1 : wk);
                        const uint64_t per = 64ull * (uint64_t)kk;
                        const uint64_t sb = seg_count(blocks) * ((kSegEntries + per - 1) / per);
                        if (wck && (rc = ensure(c, c->d_dump, (size_t)3 * sb))) return rc;
                        if (wck) ULG_HIP(c, hipMemsetAsync(c->d_dump.p, 0, 24 * sb, st));
                        prof_begin_s(c, kWalkNames[ph][L], st);
                        hipLaunchKernelGGL(sliced_fn(L, ph, wk), dim3((unsigned)sb), dim3(64), 0, st, sa.queue, qc,
                                           c->table.p, sa.hsub_out ? sa.hsub : nullptr, wck ? c->d_dump.p : nullptr,
                                           total_slots, sa.err);
                        prof_end_s(c, st);
                        if (wck && (rc = dump_walk_clock(c, st, sb, wck, L, ph))) return rc;
                        if (wck && std::getenv("ULG_WALK_QUEUE_DUMP") &&
                            (rc = dump_walk_queue(c, st, sa.queue, qc, seg_count(blocks), bits_words(L), total_slots, wck, L,
                                                  ph)))
                            return rc;
                    }
                }
            }
            if (!wide.empty() && (rc = score_wide_groups(c, L, ph, wide, nv, S, kmax, c->d_qcount.p + nqc - 1, wslice,
                                                         hoff, meta, c->wide_pinned)))
                return rc;
        }
        if (L > kMaxL && G > 1 && c->time_limit_ms == 0 && use_pool) break;  // the pool ran every wide layer
        if (c->time_limit_ms > 0 && L < kmax) {
            for (int g = 0; g < (forked ? G : 1); ++g) ULG_HIP(c, hipStreamSynchronize(gst[g]));
            const double ms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
            if (ms > (double)c->time_limit_ms) {
                done_L = L;
                c->out_of_time = 1;
                break;
            }
        }
    }
    // join: the compaction on the context stream waits for every group
    for (int g = 1; g < G && forked; ++g) {
        ULG_HIP(c, hipEventRecord(c->sync_events[g], gst[g]));
        ULG_HIP(c, hipStreamWaitEvent(c->stream, c->sync_events[g], 0));
    }
    ULG_HIP(c, hipGetLastError());

    if (done_L < kmax) {
        // out of time: the layers never launched hold no stored set
        scored = 0;
        for (int i = 0; i < nv; ++i) {
            const uint64_t b = toff[(size_t)i * S + done_L + 1], e = toff[(size_t)i * S + S];
            if (e > b) ULG_HIP(c, hipMemsetAsync(c->table.p + b, 0xff, (size_t)(e - b) * 4, c->stream));
            for (int L = 0; L <= done_L; ++L) scored += (int64_t)(toff[(size_t)i * S + L + 1] - toff[(size_t)i * S + L]);
        }
    }
    c->completed_layer = done_L;
    // compaction
    prof_begin(c, "count_stored");
    count_kernel<<<(unsigned)nb, kBlock, 0, c->stream>>>(c->table.p, total_slots, c->d_blk.p);
    prof_end(c);
    prof_begin(c, "scan_stored");
    scan_kernel<<<1, 1024, 0, c->stream>>>(c->d_blk.p, nb, c->out_offsets.p + nv, sa.err);
    prof_end(c);
    WriteArgs wa;
    wa.table = c->table.p;
    wa.blk = c->d_blk.p;
    wa.tbl_off = c->d_tbl_off.p;
    wa.meta = c->d_meta.p;
    wa.cand = c->d_cand.p;
    wa.binom = c->d_binom.p;
    wa.binom64 = c->d_binom64.p;
    wa.total = total_slots;
    wa.nv = nv;
    wa.S = S;
    wa.sets = c->out_sets.p;
    wa.scores = c->out_scores.p;
    wa.offsets = c->out_offsets.p;
    prof_begin(c, "write_stored");
    {
        const size_t nseg = (size_t)nv * (size_t)S;
        const size_t toff_bytes = nseg <= (size_t)kWriteLdsSegs ? (nseg + 1) * sizeof(uint64_t) : 0;
        write_kernel<<<(unsigned)nb, kBlock, toff_bytes, c->stream>>>(wa);
    }
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    if (use_graph) {
        hipGraph_t graph = nullptr;
        capture_guard.active = false;
        ULG_HIP(c, hipStreamEndCapture(c->stream, &graph));
        c->graph = graph;
        ULG_HIP(c, hipGraphInstantiate(&c->gexec, graph, nullptr, nullptr, 0));
        c->gkey = gkey;
        // the profiling events recorded inside the graph belong to it now
        c->gprof.assign(c->pending.begin() + (std::ptrdiff_t)pend0, c->pending.end());
        for (ProfRec &r : c->gprof) r.graph = true;
        c->pending.resize(pend0);
        ULG_HIP(c, hipGraphLaunch(c->gexec, c->stream));
        for (const ProfRec &r : c->gprof) c->pending.push_back(r);
    }
    }
launched:
    if (async && kmax <= kMaxL && c->time_limit_ms == 0) {
        // no host sync on this path: the stored count is copied into pinned
        // memory behind the launches and collected by ulg_cbic_score_finish
        if (!c->async_pinned)
            ULG_HIP(c, hipHostMalloc((void **)&c->async_pinned, 2 * sizeof(unsigned long long), hipHostMallocDefault));
        ULG_HIP(c, hipMemcpyAsync(c->async_pinned, c->d_blk.p + nb, 16, hipMemcpyDeviceToHost, c->stream));
        c->nv = nv;
        c->kmax = kmax;
        c->vars.assign(vars, vars + nv);
        c->m = mv;
        c->tbl_off = toff;
        c->total_slots = (int64_t)total_slots;
        c->total_stored = 0;
        c->total_scored = scored;
        c->scored = true;
        c->async_pending = true;
        return ULG_OK;
    }
    // the stored count and the error word through the context's pinned words
    // (a pageable destination goes through a staging copy)
    if (!c->async_pinned)
        ULG_HIP(c, hipHostMalloc((void **)&c->async_pinned, 2 * sizeof(unsigned long long), hipHostMallocDefault));
    ULG_HIP(c, hipMemcpyAsync(c->async_pinned, c->d_blk.p + nb, 16, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    const uint64_t stored = c->async_pinned[0];
    prof_collect(c);
    if ((rc = call_error(c, c->async_pinned[1]))) return rc;

    c->nv = nv;
    c->kmax = kmax;
    c->vars.assign(vars, vars + nv);
    c->m = mv;
    c->tbl_off = toff;
    c->total_slots = (int64_t)total_slots;
    c->total_stored = (int64_t)stored;
    c->total_scored = scored;
    c->scored = true;
    if (total_stored) *total_stored = (int64_t)stored;
    if (total_scored) *total_scored = scored;
    return ULG_OK;
}

int ulg_cbic_fetch(ulg_ctx *c, uint64_t *sets, float *scores, int64_t *offsets, int device_ptrs) {
    if (!c) return ULG_ERR_ARG;
    if (c->async_pending) {
        int rc0 = ulg_cbic_score_finish(c, nullptr, nullptr);
        if (rc0) return rc0;
    }
    if (!c->scored) return set_err(c, ULG_ERR_STATE, "ulg_cbic_fetch: nothing scored");
    ULG_HIP(c, hipSetDevice(c->device));
    const hipMemcpyKind k = device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const size_t cnt = (size_t)c->total_stored;
    if (sets && cnt) ULG_HIP(c, hipMemcpyAsync(sets, c->out_sets.p, cnt * 8, k, c->stream));
    if (scores && cnt) ULG_HIP(c, hipMemcpyAsync(scores, c->out_scores.p, cnt * 4, k, c->stream));
    if (offsets) ULG_HIP(c, hipMemcpyAsync(offsets, c->out_offsets.p, (size_t)(c->nv + 1) * 8, k, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return ULG_OK;
}

int ulg_cbic_score_vars(ulg_ctx *c, const int *vars, int nv, const uint64_t *candidates, int max_parents,
                        uint64_t *sets, float *scores, int64_t *offsets, int64_t cap) {
    int64_t stored = 0;
    int rc = ulg_cbic_score(c, vars, nv, candidates, max_parents, &stored, nullptr);
    if (rc) return rc;
    if (stored > cap) return set_err(c, ULG_ERR_ARG, "ulg_cbic_score_vars: output capacity too small");
    return ulg_cbic_fetch(c, sets, scores, offsets, 0);
}

int ulg_cbic_score_sets(ulg_ctx *c, int64_t count, const int *vars, const uint64_t *parents, float *neg_scores) {
    if (!c || count < 0 || (count > 0 && (!vars || !parents || !neg_scores))) return ULG_ERR_ARG;
    if (!c->loaded) return set_err(c, ULG_ERR_STATE, "ulg_cbic_score_sets: call ulg_cbic_load first");
    if (count == 0) return ULG_OK;
    const int n = c->n;
    const uint64_t allmask = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    std::vector<uint64_t> pairs((size_t)count * 2);
    for (int64_t i = 0; i < count; ++i) {
        if (vars[i] < 0 || vars[i] >= n) return set_err(c, ULG_ERR_ARG, "ulg_cbic_score_sets: variable out of range");
        if (parents[i] & ~allmask) return set_err(c, ULG_ERR_ARG, "ulg_cbic_score_sets: parent bit >= n");
        if (__builtin_popcountll(parents[i] & ~(1ull << vars[i])) > kWideMax)
            return set_err(c, ULG_ERR_UNSUPPORTED, "ulg_cbic_score_sets: more than ULG_MAX_PARENTS_GPU (31) parents");
        pairs[2 * i] = (uint64_t)vars[i];
        pairs[2 * i + 1] = parents[i];
    }
    ULG_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c, c->d_sets_in, (size_t)count * 2)) || (rc = ensure(c, c->qbuf_out, (size_t)count))) return rc;
    ULG_HIP(c, hipMemcpyAsync(c->d_sets_in.p, pairs.data(), (size_t)count * 16, hipMemcpyHostToDevice, c->stream));
    prof_begin(c, "score_sets");
    score_sets_kernel<<<(unsigned)((count + kBlock - 1) / kBlock), kBlock, (size_t)n * n * 8, c->stream>>>(
        c->gram.p, c->d_sets_in.p, count, n, c->N, c->lambda, c->qbuf_out.p);
    prof_end(c);
    ULG_HIP(c, hipMemcpyAsync(neg_scores, c->qbuf_out.p, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    return ULG_OK;
}

int ulg_quantize_costs(ulg_ctx *c, const float *scores, float *costs, int64_t count) {
    if (!c || count < 0 || (count > 0 && (!scores || !costs))) return ULG_ERR_ARG;
    if (count == 0) return ULG_OK;
    ULG_HIP(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c, c->qbuf_in, (size_t)count)) || (rc = ensure(c, c->qbuf_out, (size_t)count))) return rc;
    ULG_HIP(c, hipMemcpyAsync(c->qbuf_in.p, scores, (size_t)count * 4, hipMemcpyHostToDevice, c->stream));
    prof_begin(c, "quantize");
    quantize_kernel<<<(unsigned)((count + kBlock - 1) / kBlock), kBlock, 0, c->stream>>>(c->qbuf_in.p, c->qbuf_out.p,
                                                                                       count);
    prof_end(c);
    ULG_HIP(c, hipMemcpyAsync(costs, c->qbuf_out.p, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    return ULG_OK;
}

#ifdef ULG_GATHER_STATS
// diagnostic build: the gather counters (2 * (kMaxL + 1) * 16 values), then
// the walk's hits by depth (as many), both zeroed
int ulg_diag_gather_stats(ulg_ctx *c, unsigned long long *out) {
    if (!c || !out) return ULG_ERR_ARG;
    ULG_HIP(c, hipSetDevice(c->device));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    ULG_HIP(c, hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gstats), sizeof(g_gstats)));
    static const unsigned long long zero[2 * (kMaxL + 1) * 16] = {};
    ULG_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(g_gstats), zero, sizeof(zero)));
    ULG_HIP(c, hipMemcpyFromSymbol(out + 2 * (kMaxL + 1) * 16, HIP_SYMBOL(g_wstats), sizeof(g_wstats)));
    ULG_HIP(c, hipMemcpyToSymbol(HIP_SYMBOL(g_wstats), zero, sizeof(zero)));
    return ULG_OK;
}
#endif

}  // extern "C"
