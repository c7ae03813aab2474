// search.hip -- best-score lattice tables and the static pattern database on
// MI355X, plus the device queries the search uses.
//
// Reference path (urlearning/):
//   SparseParentList::initialize/getScore  score_cache/sparse_parent_list.cpp:20-55
//   StaticPatternDatabase                  heuristic/static_pattern_database.cpp:82-247
//
// BestScore table (replaces the sorted-list linear scan): for variable v with
// parent-set support D_v (union of its stored sets, m_v = |D_v|), a dense
// table over all 2^m_v subsets S of D_v holds
//     T_v(S) = min over stored sets P subset of S of ordkey(cost_P)
// (4 B per entry), i.e. the cost of the first entry of the list sorted by
// (cost, file order) that is a subset of S -- what SparseParentList::getScore
// returns.  getParents (the file index behind the min) is needed only for
// the few reconstruction queries; those scan the list with the pinned N7
// (cost, file order) tie-break (bs_key_scan), which finds a set of exactly
// this cost.  The table is filled by a scatter of the stored sets and an
// in-place subset-min ("zeta") transform: bits 0..13 inside LDS tiles, the
// remaining bits in a second pass over strided tiles whose rows are 16
// contiguous entries.  Both passes stream the table once (HBM-bound).
// Lookup: cost = ord_cost(T_v[pext(S, D_v)]).
#include <chrono>
#include <hipcub/hipcub.hpp>
#include <sys/mman.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "search_internal.h"

using namespace ulg;

namespace {

constexpr int kB = 256;
constexpr int kTileBits = 14;  // pass A: 2^14 u32 = 64 KiB LDS
constexpr int kRowBits = 4;    // pass B rows: 16 contiguous u32 = 64 B
constexpr int kColBits = 10;   // pass B: 2^10 rows x 16 = 2^14 u32

// HIP caps blocks x threads along one grid dimension at 2^32 - 1, so launches
// of more blocks spread them over y (n = 28 full skeleton: the last pass B
// has 28 x 2^20 blocks of 1024 threads); flat_block() is the block's index.
constexpr uint64_t kGridX = 1ull << 20;
inline dim3 flat_grid(uint64_t blocks) {
    return dim3((unsigned)std::min<uint64_t>(blocks, kGridX), (unsigned)((blocks + kGridX - 1) / kGridX));
}
__device__ __forceinline__ uint64_t flat_block() { return (uint64_t)blockIdx.y * gridDim.x + blockIdx.x; }

// D_v = union of v's stored sets inside scope (variables outside scope get
// D_v = {} and a one-entry table)
__global__ void __launch_bounds__(kB) support_kernel(const uint64_t *sets, const int64_t *offsets, int n,
                                                     uint64_t scope, unsigned long long *support) {
    const int v = blockIdx.y;
    const int64_t b = offsets[v], e = offsets[v + 1];
    uint64_t acc = 0;
    if ((scope >> v) & 1ull)
        for (int64_t i = b + (int64_t)blockIdx.x * kB + threadIdx.x; i < e; i += (int64_t)gridDim.x * kB)
            if ((sets[i] & ~scope) == 0) acc |= sets[i];
    // wave OR-reduction then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) acc |= __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0 && acc) atomicOr(&support[v], (unsigned long long)acc);
}

__global__ void __launch_bounds__(kB) scatter_kernel(const uint64_t *sets, const float *costs, const int64_t *offsets,
                                                     int n, const uint64_t *support, const uint64_t *tb_off,
                                                     uint32_t *table, uint64_t tvars) {
    const int v = blockIdx.y;
    if (!((tvars >> v) & 1ull)) return;  // no table for v (sharded tables)
    const int64_t b = offsets[v], e = offsets[v + 1];
    const uint64_t D = support[v];
    for (int64_t i = b + (int64_t)blockIdx.x * kB + threadIdx.x; i < e; i += (int64_t)gridDim.x * kB) {
        if (sets[i] & ~D) continue;  // outside the scope
        const uint64_t idx = pext64(sets[i], D);
        table[tb_off[v] + idx] = ordkey(costs[i]);  // stored sets are distinct: one writer per slot
    }
}

// pass A: all subset bits inside a contiguous tile of 2^T entries.
__global__ void __launch_bounds__(1024) zeta_tile_kernel(uint32_t *table, const uint64_t *tb_off, const int *tiles_prefix,
                                                         const int *mbits, int nvar) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *t = reinterpret_cast<uint32_t *>(smem);
    const int64_t blk = (int64_t)flat_block();
    if (blk >= tiles_prefix[nvar]) return;
    // which variable / tile
    int lo = 0, hi = nvar;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tiles_prefix[mid] <= blk) lo = mid; else hi = mid;
    }
    const int v = lo;
    const int m = mbits[v];
    const int T = m < kTileBits ? m : kTileBits;
    const uint64_t size = 1ull << T;
    const uint64_t base = tb_off[v] + ((uint64_t)(blk - tiles_prefix[v]) << T);
    for (uint64_t i = threadIdx.x; i < size; i += 1024) t[i] = table[base + i];
    __syncthreads();
    for (int b = 0; b < T; ++b) {
        const uint64_t bit = 1ull << b;
        for (uint64_t p = threadIdx.x; p < (size >> 1); p += 1024) {
            const uint64_t i = ((p >> b) << (b + 1)) | (p & (bit - 1));
            const uint32_t a = t[i], c = t[i | bit];
            if (a < c) t[i | bit] = a;
        }
        __syncthreads();
    }
    for (uint64_t i = threadIdx.x; i < size; i += 1024) table[base + i] = t[i];
}

// pass B: bits [bit_lo, bit_lo + G) over tiles of 2^G rows x 16 contiguous entries.
struct ZetaBArgs {
    uint32_t *table;
    const uint64_t *tb_off;
    const int *blocks_prefix;
    const int *mbits;
    int nvar;
    int bit_lo;
};
__global__ void __launch_bounds__(1024) zeta_strided_kernel(ZetaBArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *t = reinterpret_cast<uint32_t *>(smem);
    const int64_t blk = (int64_t)flat_block();
    if (blk >= a.blocks_prefix[a.nvar]) return;
    int lo = 0, hi = a.nvar;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a.blocks_prefix[mid] <= blk) lo = mid; else hi = mid;
    }
    const int v = lo;
    const int m = a.mbits[v];
    const int bit_lo = a.bit_lo;
    const int G = std::min(kColBits, m - bit_lo);
    const int nlow = bit_lo - kRowBits;
    const uint64_t bid = (uint64_t)(blk - a.blocks_prefix[v]);
    // tile origin inside v's table; v's table itself starts at tb_off[v], which
    // is not aligned to 2^m when the supports differ in size: add, never OR
    uint32_t *tv = a.table + a.tb_off[v];
    const uint64_t base = ((bid & ((1ull << nlow) - 1)) << kRowBits) | ((bid >> nlow) << (bit_lo + G));
    const int rows = 1 << G;
    const int size = rows << kRowBits;
    for (int e = threadIdx.x; e < size; e += 1024) {
        const uint64_t hc = (uint64_t)(e >> kRowBits), lw = (uint64_t)(e & 15);
        t[e] = tv[base | (hc << bit_lo) | lw];
    }
    __syncthreads();
    for (int j = 0; j < G; ++j) {
        for (int p = threadIdx.x; p < (size >> 1); p += 1024) {
            const int lw = p & 15, q = p >> 4;  // q indexes rows with bit j clear
            const int r0 = ((q >> j) << (j + 1)) | (q & ((1 << j) - 1));
            const int i0 = (r0 << kRowBits) | lw, i1 = ((r0 | (1 << j)) << kRowBits) | lw;
            const uint32_t x = t[i0], y = t[i1];
            if (x < y) t[i1] = x;
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < size; e += 1024) {
        const uint64_t hc = (uint64_t)(e >> kRowBits), lw = (uint64_t)(e & 15);
        tv[base | (hc << bit_lo) | lw] = t[e];
    }
}

// ---- register-blocked subset-min for the big tables ---------------------------
// A 2^14-entry tile (or a 2^10-row x 16-column strided tile) is handled by 1024
// threads holding 16 entries each: the min along 4 index bits at a time runs
// in registers, and LDS only exchanges the entries between the 4-bit windows
// (3 exchanges instead of one LDS sweep per bit).  The subset-min along one
// bit is idempotent, so windows may overlap (bits 0-3, 4-7, 8-11, 10-13).
// LDS rows of 16 entries are padded by one entry against bank conflicts.
constexpr int kRegTileBits = 14;
constexpr int kPadLds = (1 << kRegTileBits) + (1 << (kRegTileBits - 4));

__device__ __forceinline__ int padx(int e) { return e + (e >> 4); }

__device__ __forceinline__ void min4(uint32_t (&r)[16]) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i & (1 << b)) r[i] = r[i ^ (1 << b)] < r[i] ? r[i ^ (1 << b)] : r[i];
}

// one (global table index, packed key) per stored set inside the tables' scope
__global__ void __launch_bounds__(kB) entries_kernel(const uint64_t *sets, const float *costs, const int64_t *offsets,
                                                     int n, const uint64_t *support, const uint64_t *tb_off,
                                                     uint64_t *idx, uint32_t *key, uint64_t tvars) {
    const int v = blockIdx.y;
    const int64_t b = offsets[v], e = offsets[v + 1];
    const uint64_t D = support[v];
    const bool own = (tvars >> v) & 1ull;
    for (int64_t i = b + (int64_t)blockIdx.x * kB + threadIdx.x; i < e; i += (int64_t)gridDim.x * kB) {
        if (!own || (sets[i] & ~D)) {
            idx[i] = ~0ull;  // outside the scope: sorts past every slot
            key[i] = 0xFFFFFFFFu;
            continue;
        }
        idx[i] = tb_off[v] + pext64(sets[i], D);
        key[i] = ordkey(costs[i]);
    }
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t *a, int64_t n, uint64_t x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// pass A for tables of >= 2^14 entries: builds each tile from its sorted
// entries (no fill, no read of the table) and writes it once
__global__ void __launch_bounds__(1024) zeta_tile_reg_kernel(uint32_t *table, uint64_t ntiles_total,
                                                             const uint64_t *eidx, const uint32_t *ekey,
                                                             int64_t nent) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *t = reinterpret_cast<uint32_t *>(smem);
    __shared__ int64_t range[2];
    const int tid = threadIdx.x;
    if (flat_block() >= ntiles_total) return;
    const uint64_t base = flat_block() << kRegTileBits;  // tiles are contiguous over all variables
    if (tid == 0) {
        range[0] = lower_bound_u64(eidx, nent, base);
        range[1] = lower_bound_u64(eidx, nent, base + (1ull << kRegTileBits));
    }
    for (int i = tid; i < (1 << kRegTileBits); i += 1024) t[padx(i)] = 0xFFFFFFFFu;
    __syncthreads();
    for (int64_t k = range[0] + tid; k < range[1]; k += 1024) t[padx((int)(eidx[k] - base))] = ekey[k];
    __syncthreads();
    uint32_t r[16];
    // bits 0-3: entries tid*16 + i
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[padx(tid * 16 + i)];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[padx(tid * 16 + i)] = r[i];
    __syncthreads();
    // bits 4-7
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[padx(((tid >> 4) << 8) | (i << 4) | (tid & 15))];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[padx(((tid >> 4) << 8) | (i << 4) | (tid & 15))] = r[i];
    __syncthreads();
    // bits 8-11
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[padx(((tid >> 8) << 12) | (i << 8) | (tid & 255))];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[padx(((tid >> 8) << 12) | (i << 8) | (tid & 255))] = r[i];
    __syncthreads();
    // bits 10-13, straight to HBM (consecutive threads, consecutive entries)
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[padx((i << 10) | tid)];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) table[base + ((uint64_t)i << 10) + tid] = r[i];
    (void)ntiles_total;
}

// pass B for 10 index bits [bit_lo, bit_lo + 10) of tables with m >= bit_lo + 10:
// a tile is 1024 rows (those bits) x 16 contiguous entries (bits 0-3)
__global__ void __launch_bounds__(1024) zeta_strided_reg_kernel(ZetaBArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *t = reinterpret_cast<uint32_t *>(smem);
    const int64_t blk = (int64_t)flat_block();
    if (blk >= a.blocks_prefix[a.nvar]) return;
    int lo = 0, hi = a.nvar;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a.blocks_prefix[mid] <= blk) lo = mid; else hi = mid;
    }
    const int v = lo;
    const int bit_lo = a.bit_lo;
    const int nlow = bit_lo - kRowBits;
    const uint64_t bid = (uint64_t)(blk - a.blocks_prefix[v]);
    uint32_t *tv = a.table + a.tb_off[v];
    const uint64_t base = ((bid & ((1ull << nlow) - 1)) << kRowBits) | ((bid >> nlow) << (bit_lo + 10));
    const int tid = threadIdx.x, c = tid & 15, q = tid >> 4;
    uint32_t r[16];
    // row bits 0-3: rows (q << 4) | i
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = tv[base | ((uint64_t)((q << 4) | i) << bit_lo) | c];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[padx((((q << 4) | i) << 4) | c)] = r[i];
    __syncthreads();
    // row bits 4-7: rows ((q >> 4) << 8) | (i << 4) | (q & 15)
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[padx(((((q >> 4) << 8) | (i << 4) | (q & 15)) << 4) | c)];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[padx(((((q >> 4) << 8) | (i << 4) | (q & 15)) << 4) | c)] = r[i];
    __syncthreads();
    // row bits 6-9: rows (i << 6) | q, back to HBM
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[padx((((i << 6) | q) << 4) | c)];
    min4(r);
#pragma unroll
    for (int i = 0; i < 16; ++i) tv[base | ((uint64_t)((i << 6) | q) << bit_lo) | c] = r[i];
}

// Successor-cost rows for the dense exact-order search: thread t of a chunk
// fills row r = r0 + t / nl, column li: getScore(scc_li, S) with
// S = pdep(r, scope) (FLT_MAX for scc_li in S) -- one contiguous row per
// popped node instead of one random lattice read per successor.
__global__ void __launch_bounds__(kB) cost_rows_kernel(SearchDev d, const int *meta, int m, int nl, uint64_t r0,
                                                       uint64_t cnt, float *out) {
    __shared__ int bits[64], vars[64];
    for (int i = threadIdx.x; i < m; i += kB) bits[i] = meta[i];
    for (int i = threadIdx.x; i < nl; i += kB) vars[i] = meta[64 + i];
    __syncthreads();
    const uint64_t t = flat_block() * kB + threadIdx.x;
    if (t >= cnt * (uint64_t)nl) return;
    const uint64_t r = r0 + t / (uint64_t)nl;
    const int li = (int)(t % (uint64_t)nl);
    uint64_t S = 0;
    for (uint64_t x = r; x; x &= x - 1) S |= 1ull << bits[__builtin_ctzll(x)];
    const int leaf = vars[li];
    out[t] = ((S >> leaf) & 1ull) ? FLT_MAX : bs_cost(d, leaf, S);
}

__global__ void __launch_bounds__(kB) cost_table_kernel(const uint32_t *table, uint64_t total, float *costs) {
    const uint64_t i = flat_block() * kB + threadIdx.x;
    if (i < total) costs[i] = ord_cost(table[i]);
}

// getScore + getParents for one (variable, S) per block: the block scans the
// variable's list for the first (cost, file order) stored subset of S
// (sparse_parent_list.cpp:44-55 with the pinned N7 tie-break) -- the entry
// whose cost the lattice holds, and the parent set behind it.
__global__ void __launch_bounds__(kB) query_kernel(SearchDev d, int64_t count, const int *vars, const uint64_t *S,
                                                   float *costs, uint64_t *parents) {
    __shared__ uint64_t red[kB / 64];
    const int64_t q = blockIdx.x;
    const int v = vars[q];
    const uint64_t s = S[q];
    const int64_t b = d.offsets[v], e = d.offsets[v + 1];
    uint64_t best = ~0ull;
    for (int64_t i = b + threadIdx.x; i < e; i += kB)
        if ((d.sets[i] & ~s) == 0) {
            const uint64_t k = ((uint64_t)ordkey(d.costs[i]) << 32) | (uint64_t)(i - b);
            best = k < best ? k : best;
        }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(best, off);
        best = o < best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kB / 64; ++w) best = red[w] < best ? red[w] : best;
        costs[q] = bs_cost(d, v, s);  // the lattice read (the scan's key cost where S is outside the tables)
        parents[q] = (best == ~0ull) ? 0ull : d.sets[b + (int64_t)(best & 0xffffffffull)];
    }
}

__global__ void quantize_lists_kernel(const float *scores, float *costs, int64_t count) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i < count) costs[i] = quantize_score(scores[i]);
}

// ---- static pattern database ------------------------------------------------
struct PdbBsArgs {
    SearchDev d;
    uint64_t group;
    int s;
    const int *bitpos;  // s entries
    uint64_t scc, anc;
    float *bsv;         // [2^s][s]
};
// bsv[R][j] = getScore(leaf = bitpos[j], (scc \ (R \ {leaf})) | ancestors) for leaf in R
__global__ void __launch_bounds__(kB) pdb_bs_kernel(PdbBsArgs a) {
    const uint64_t p = (uint64_t)blockIdx.x * kB + threadIdx.x;
    const int s = a.s;
    if (p >= ((uint64_t)s << (s - 1))) return;
    const int j = (int)(p >> (s - 1));
    const uint64_t rr = p & ((1ull << (s - 1)) - 1ull);
    const uint64_t R = ((rr >> j) << (j + 1)) | (1ull << j) | (rr & ((1ull << j) - 1ull));
    uint64_t Rg = 0;
    for (int t = 0; t < s; ++t)
        if ((R >> t) & 1ull) Rg |= 1ull << a.bitpos[t];
    const int leaf = a.bitpos[j];
    const uint64_t removed = Rg & ~(1ull << leaf);
    const uint64_t choices = (a.scc & ~removed) | a.anc;
    a.bsv[R * s + j] = bs_cost(a.d, leaf, choices);
}

// one layer of the reverse BFS (static_pattern_database.cpp:184-207):
// pd[R] = fold over leaves l in R (descending, the oracle's key order) of
//         newG = bs(l, ...) + pd[R \ l], kept if oldG == 0 || newG < oldG.
__global__ void __launch_bounds__(kB) pdb_layer_kernel(const float *bsv, int s, int layer, float *pd) {
    const uint64_t R = (uint64_t)blockIdx.x * kB + threadIdx.x;
    if (R >= (1ull << s) || __popcll(R) != layer) return;
    float cur = 0.0f;
    for (int j = s - 1; j >= 0; --j) {
        if (!((R >> j) & 1ull)) continue;
        const float newG = bsv[R * s + j] + pd[R ^ (1ull << j)];
        if (cur == 0 || newG < cur) cur = newG;
    }
    pd[R] = cur;
}

__global__ void __launch_bounds__(kB) pdb_query_kernel(SearchDev d, int64_t count, const uint64_t *S, float *h,
                                                       int *complete) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= count) return;
    int c = 0;
    h[i] = pdb_h(d, S[i], &c);
    complete[i] = c;
}

}  // namespace

namespace ulg {

int search_build_tables(ulg_ctx *c, uint64_t scope, uint64_t tvars) {
    SearchState &s = *c->search;
    const int n = s.n;
    tvars &= (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    int rc;
    // support D_v
    if ((rc = ensure(c, s.d_support, (size_t)n))) return rc;
    ULG_HIP(c, hipMemsetAsync(s.d_support.p, 0, (size_t)n * 8, c->stream));
    int64_t maxcnt = 1;
    for (int v = 0; v < n; ++v) maxcnt = std::max<int64_t>(maxcnt, s.offsets[v + 1] - s.offsets[v]);
    const unsigned gx = (unsigned)std::min<int64_t>((maxcnt + kB - 1) / kB, 4096);
    prof_begin(c, "bs_support");
    support_kernel<<<dim3(gx, n), kB, 0, c->stream>>>(s.d_sets.p, s.d_offsets.p, n, scope,
                                                     reinterpret_cast<unsigned long long *>(s.d_support.p));
    prof_end(c);
    std::vector<uint64_t> support(n, 0);
    ULG_HIP(c, hipMemcpyAsync(support.data(), s.d_support.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    // memory check before touching the current tables: 4 B ordered cost + 4 B
    // device float cost + 4 B pinned host cost per entry
    // variables outside tvars get no table (0 entries; their lookups scan the lists)
    uint64_t total = 0;
    for (int v = 0; v < n; ++v) {
        const int m = __builtin_popcountll(support[v]);
        if (!((tvars >> v) & 1ull)) continue;
        if (m > 40) return set_err(c, ULG_ERR_UNSUPPORTED, "best-score table over more than 40 candidate parents");
        total += 1ull << m;
    }
    if (total == 0) return set_err(c, ULG_ERR_ARG, "best-score tables for no variable");
    uint64_t budget = c->table_budget_kb << 10;
    if (budget == 0) {
        size_t free_b = 0, tot_b = 0;
        ULG_HIP(c, hipMemGetInfo(&free_b, &tot_b));
        budget = (uint64_t)(free_b / 2) + (uint64_t)s.d_table.cap * 4 + (uint64_t)s.d_cost_table.cap * 4;
    }
    if (total * 12 > budget)
        return set_err(c, ULG_ERR_UNSUPPORTED, "best-score tables for this scope need " +
                                                   std::to_string((total * 12) >> 10) + " KiB (budget " +
                                                   std::to_string(budget >> 10) + " KiB)");
    s.tables_ready = false;
    s.pdb_ready = false;
    s.host_costs_ready = false;
    s.rows_ready = false;
    s.sweep_ready = false;
    s.support = support;
    s.mbits.assign(n, 0);
    s.tb_off.assign(n + 1, 0);
    for (int v = 0; v < n; ++v) {
        const bool own = (tvars >> v) & 1ull;
        s.mbits[v] = own ? __builtin_popcountll(s.support[v]) : 0;
        s.tb_off[v + 1] = s.tb_off[v] + (own ? (1ull << s.mbits[v]) : 0ull);
    }
    s.table_vars = tvars;
    s.table_entries = total;
    if ((rc = ensure(c, s.d_table, total)) || (rc = ensure(c, s.d_tb_off, (size_t)n + 1)) ||
        (rc = ensure(c, s.d_mbits, (size_t)n)))
        return rc;
    ULG_HIP(c, hipMemcpyAsync(s.d_tb_off.p, s.tb_off.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    ULG_HIP(c, hipMemcpyAsync(s.d_mbits.p, s.mbits.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    int minm = 64;
    for (int v = 0; v < n; ++v)
        if ((tvars >> v) & 1ull) minm = std::min(minm, s.mbits[v]);
    std::vector<int> tiles_prefix(n + 1, 0), blocks_prefix(n + 1, 0);
    if ((rc = ensure(c, s.d_prefix, (size_t)2 * (n + 1)))) return rc;
    if (minm >= kRegTileBits) {
        // every table is whole 2^14-entry tiles: sort the stored sets by table
        // index once and build each tile from its entries (no fill, no read)
        const int64_t nsets = s.offsets[n];
        if ((rc = ensure(c, s.e_idx, (size_t)nsets)) || (rc = ensure(c, s.e_key, (size_t)nsets)) ||
            (rc = ensure(c, s.e_idx2, (size_t)nsets)) || (rc = ensure(c, s.e_key2, (size_t)nsets)))
            return rc;
        prof_begin(c, "bs_entries");
        entries_kernel<<<dim3(gx, n), kB, 0, c->stream>>>(s.d_sets.p, s.d_costs.p, s.d_offsets.p, n, s.d_support.p,
                                                         s.d_tb_off.p, s.e_idx.p, s.e_key.p, tvars);
        prof_end(c);
        int end_bit = 1;
        while (end_bit < 64 && (1ull << (end_bit - 1)) <= total) ++end_bit;  // ~0 sorts past every slot
        size_t tmp = 0;
        ULG_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, s.e_idx.p, s.e_idx2.p, s.e_key.p, s.e_key2.p,
                                                      (int)nsets, 0, end_bit, c->stream));
        if ((rc = ensure(c, s.sort_tmp, tmp))) return rc;
        prof_begin(c, "bs_sort");
        ULG_HIP(c, hipcub::DeviceRadixSort::SortPairs(s.sort_tmp.p, tmp, s.e_idx.p, s.e_idx2.p, s.e_key.p, s.e_key2.p,
                                                      (int)nsets, 0, end_bit, c->stream));
        prof_end(c);
        ULG_HIP(c, hipFuncSetAttribute((const void *)zeta_tile_reg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       kPadLds * 4));
        prof_begin(c, "bs_zeta_tile");
        zeta_tile_reg_kernel<<<flat_grid(total >> kRegTileBits), 1024, (size_t)kPadLds * 4, c->stream>>>(
            s.d_table.p, total >> kRegTileBits, s.e_idx2.p, s.e_key2.p, nsets);
        prof_end(c);
        ULG_HIP(c, hipGetLastError());
    } else {
    prof_begin(c, "bs_fill");
    ULG_HIP(c, hipMemsetAsync(s.d_table.p, 0xff, total * 4, c->stream));
    prof_end(c);
    prof_begin(c, "bs_scatter");
    scatter_kernel<<<dim3(gx, n), kB, 0, c->stream>>>(s.d_sets.p, s.d_costs.p, s.d_offsets.p, n, s.d_support.p,
                                                     s.d_tb_off.p, s.d_table.p, tvars);
    prof_end(c);
    // pass A tiles
    for (int v = 0; v < n; ++v) {
        const int m = s.mbits[v];
        tiles_prefix[v + 1] = tiles_prefix[v] + (!((tvars >> v) & 1ull) ? 0 : m <= kTileBits ? 1 : (1 << (m - kTileBits)));
    }
    ULG_HIP(c, hipMemcpyAsync(s.d_prefix.p, tiles_prefix.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    const int maxm0 = *std::max_element(s.mbits.begin(), s.mbits.end());
    const size_t ldsA = (size_t)4 << std::min(maxm0, kTileBits);
    ULG_HIP(c, hipFuncSetAttribute((const void *)zeta_tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4 << kTileBits)));
    prof_begin(c, "bs_zeta_tile");
    zeta_tile_kernel<<<flat_grid((uint64_t)tiles_prefix[n]), 1024, ldsA, c->stream>>>(s.d_table.p, s.d_tb_off.p, s.d_prefix.p, s.d_mbits.p, n);
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    }
    const int maxm = *std::max_element(s.mbits.begin(), s.mbits.end());
    // pass B over the remaining high bits, kColBits at a time
    ULG_HIP(c, hipFuncSetAttribute((const void *)zeta_strided_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4 << (kColBits + kRowBits))));
    for (int bit_lo = kTileBits; bit_lo < maxm; bit_lo += kColBits) {
        std::fill(blocks_prefix.begin(), blocks_prefix.end(), 0);
        for (int v = 0; v < n; ++v) {
            const int m = s.mbits[v];
            int nb = 0;
            if (m > bit_lo) nb = 1 << (m - kRowBits - std::min(kColBits, m - bit_lo));
            blocks_prefix[v + 1] = blocks_prefix[v] + nb;
        }
        if (blocks_prefix[n] == 0) break;
        ULG_HIP(c, hipMemcpyAsync(s.d_prefix.p + (n + 1), blocks_prefix.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice, c->stream));
        ZetaBArgs za{s.d_table.p, s.d_tb_off.p, s.d_prefix.p + (n + 1), s.d_mbits.p, n, bit_lo};
        const int G = std::min(kColBits, maxm - bit_lo);
        bool full_window = kColBits == 10;
        for (int v = 0; v < n; ++v)
            if (s.mbits[v] > bit_lo && s.mbits[v] - bit_lo < 10) full_window = false;
        prof_begin(c, "bs_zeta_strided");
        if (full_window) {
            ULG_HIP(c, hipFuncSetAttribute((const void *)zeta_strided_reg_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kPadLds * 4));
            zeta_strided_reg_kernel<<<flat_grid((uint64_t)blocks_prefix[n]), 1024, (size_t)kPadLds * 4, c->stream>>>(za);
        } else {
            zeta_strided_kernel<<<flat_grid((uint64_t)blocks_prefix[n]), 1024, (size_t)4 << (G + kRowBits), c->stream>>>(za);
        }
        prof_end(c);
        ULG_HIP(c, hipGetLastError());
        // host copy of blocks_prefix must stay valid until the copy ran
        ULG_HIP(c, hipStreamSynchronize(c->stream));
    }
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    s.scope = scope;
    s.tables_ready = true;
    return ULG_OK;
}

int search_ensure_scope(ulg_ctx *c, uint64_t need) {
    SearchState &s = *c->search;
    const uint64_t all = (s.n >= 64) ? ~0ull : ((1ull << s.n) - 1ull);
    if (s.tables_ready && (need & ~s.scope) == 0 && s.table_vars == all) return ULG_OK;
    return search_build_tables(c, need, all);
}

int search_build_pdb(ulg_ctx *c, int pd_count, uint64_t ancestors, uint64_t scc) {
    SearchState &s = *c->search;
    if (!s.lists_ready) return set_err(c, ULG_ERR_STATE, "pattern database needs the parent-set lists");
    if (pd_count < 1 || pd_count > kMaxGroups) return set_err(c, ULG_ERR_ARG, "pd_count must be 1..8");
    // groups: consecutive scc variables, ceil(|scc| / pd_count) each (static_pattern_database.cpp:95-120)
    s.groups.clear();
    const int remaining = __builtin_popcountll(scc);
    const int pds = (int)std::ceil((float)remaining / pd_count);
    int var = scc ? __builtin_ctzll(scc) : -1;
    int x = 0;
    for (int g = 0; g < pd_count; ++g) {
        uint64_t grp = 0;
        int sz;
        for (sz = 0; sz < pds && x < remaining; ++sz) {
            grp |= 1ull << var;
            const uint64_t rest = (var + 1 < 64) ? (scc >> (var + 1)) : 0;
            var = var + (rest ? (__builtin_ctzll(rest) + 1) : 0);
            ++x;
        }
        s.groups.push_back(grp);
    }
    if (ancestors & scc) return set_err(c, ULG_ERR_UNSUPPORTED, "ancestors overlapping the search variables");
    s.ancestors = ancestors;
    s.scc = scc;
    int rc;
    size_t total = 0, maxbsv = 1;
    s.pd_off.assign(pd_count + 1, 0);
    for (int g = 0; g < pd_count; ++g) {
        const int sz = __builtin_popcountll(s.groups[g]);
        if (sz > 24) return set_err(c, ULG_ERR_UNSUPPORTED, "pattern-database group larger than 24 variables");
        s.pd_off[g + 1] = s.pd_off[g] + (1ull << sz);
        maxbsv = std::max(maxbsv, (size_t)sz << sz);
    }
    total = s.pd_off[pd_count];
    if ((rc = ensure(c, s.d_pd, total)) || (rc = ensure(c, s.d_bsv, maxbsv)) || (rc = ensure(c, s.d_bitpos, 64)))
        return rc;
    ULG_HIP(c, hipMemsetAsync(s.d_pd.p, 0, total * 4, c->stream));
    const SearchDev d = s.dev();
    for (int g = 0; g < pd_count; ++g) {
        const uint64_t grp = s.groups[g];
        const int sz = __builtin_popcountll(grp);
        if (sz == 0) continue;
        std::vector<int> bitpos;
        for (int b = 0; b < 64; ++b)
            if ((grp >> b) & 1ull) bitpos.push_back(b);
        ULG_HIP(c, hipMemcpyAsync(s.d_bitpos.p, bitpos.data(), bitpos.size() * 4, hipMemcpyHostToDevice, c->stream));
        PdbBsArgs a{d, grp, sz, s.d_bitpos.p, scc, ancestors, s.d_bsv.p};
        const uint64_t work = (uint64_t)sz << (sz - 1);
        prof_begin(c, "pdb_bs");
        pdb_bs_kernel<<<(unsigned)((work + kB - 1) / kB), kB, 0, c->stream>>>(a);
        prof_end(c);
        float *pd = s.d_pd.p + s.pd_off[g];
        for (int layer = 1; layer <= sz; ++layer) {
            prof_begin(c, "pdb_layer");
            pdb_layer_kernel<<<(unsigned)(((1ull << sz) + kB - 1) / kB), kB, 0, c->stream>>>(s.d_bsv.p, sz, layer, pd);
            prof_end(c);
        }
        ULG_HIP(c, hipStreamSynchronize(c->stream));  // bitpos / bsv reused by the next group
    }
    ULG_HIP(c, hipGetLastError());
    // host copies (small) for the exact-order search and the group table for device h
    s.pd_host.resize(total);
    ULG_HIP(c, hipMemcpyAsync(s.pd_host.data(), s.d_pd.p, total * 4, hipMemcpyDeviceToHost, c->stream));
    std::vector<uint64_t> gmeta(2 * kMaxGroups, 0);
    for (int g = 0; g < pd_count; ++g) {
        gmeta[g] = s.groups[g];
        gmeta[kMaxGroups + g] = s.pd_off[g];
    }
    if ((rc = ensure(c, s.d_groups, gmeta.size()))) return rc;
    ULG_HIP(c, hipMemcpyAsync(s.d_groups.p, gmeta.data(), gmeta.size() * 8, hipMemcpyHostToDevice, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    s.pd_count = pd_count;
    s.pdb_ready = true;
    return ULG_OK;
}

int search_quantize_device(ulg_ctx *c, const float *d_scores, float *d_costs, int64_t count) {
    if (count <= 0) return ULG_OK;
    prof_begin(c, "quantize_lists");
    quantize_lists_kernel<<<(unsigned)((count + kB - 1) / kB), kB, 0, c->stream>>>(d_scores, d_costs, count);
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    return ULG_OK;
}

int search_cost_table_host(ulg_ctx *c) {
    SearchState &s = *c->search;
    if (s.host_costs_ready) return ULG_OK;
    const uint64_t total = s.table_entries;
    int rc;
    if ((rc = ensure(c, s.d_cost_table, total))) return rc;
    prof_begin(c, "bs_cost_table");
    cost_table_kernel<<<flat_grid((total + kB - 1) / kB), kB, 0, c->stream>>>(s.d_table.p, total, s.d_cost_table.p);
    prof_end(c);
    if (s.host_cost_cap < total) {
        if (s.host_costs) (void)hipHostFree(s.host_costs);
        s.host_costs = nullptr;
        ULG_HIP(c, hipHostMalloc((void **)&s.host_costs, total * 4, hipHostMallocDefault));
        s.host_cost_cap = total;
    }
    ULG_HIP(c, hipMemcpyAsync(s.host_costs, s.d_cost_table.p, total * 4, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    s.host_costs_ready = true;
    return ULG_OK;
}

bool HostHuge::reserve(size_t want, bool pin) {
    if (p && bytes >= want && pinned == pin) return true;
    release();
    const size_t huge = (size_t)2 << 20;
    const size_t b = (want + huge - 1) / huge * huge;
    void *q = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (q == MAP_FAILED) return false;
    (void)madvise(q, b, MADV_HUGEPAGE);
    p = q;
    bytes = b;
    pinned = false;
    if (pin) pinned = hipHostRegister(p, b, hipHostRegisterDefault) == hipSuccess;  // else pageable copies
    return true;
}

void HostHuge::zero_prefix(size_t n) {
    if (p && n) std::memset(p, 0, std::min(n, bytes));
}

void HostHuge::release() {
    if (!p) return;
    if (pinned) (void)hipHostUnregister(p);
    munmap(p, bytes);
    p = nullptr;
    bytes = 0;
    pinned = false;
}

int search_cost_rows_host(ulg_ctx *c, uint64_t scope, uint64_t scc, int64_t deadline_ns, bool *timed_out) {
    SearchState &s = *c->search;
    if (timed_out) *timed_out = false;
    if (s.rows_ready && s.rows_scope == scope && s.rows_scc == scc) return ULG_OK;
    const int m = __builtin_popcountll(scope), nl = __builtin_popcountll(scc), W = nl;
    const uint64_t rows = 1ull << m, total = rows * (uint64_t)W;
    if (!s.host_rows.reserve((size_t)total * 4, true))
        return set_err(c, ULG_ERR_HIP, "cannot map the host row table (" + std::to_string(total * 4 >> 20) + " MiB)");
    std::vector<int> meta(128, 0);
    {
        int i = 0;
        for (uint64_t x = scope; x; x &= x - 1) meta[i++] = __builtin_ctzll(x);
        i = 0;
        for (uint64_t x = scc; x; x &= x - 1) meta[64 + i++] = __builtin_ctzll(x);
    }
    // chunks of <= 64 Mi floats through one device staging buffer
    const uint64_t chunk_rows = std::max<uint64_t>(1, std::min<uint64_t>(rows, (64ull << 20) / (uint64_t)W));
    int rc;
    if ((rc = ensure(c, s.d_rows, (size_t)(chunk_rows * W))) || (rc = ensure(c, s.d_rowmeta, 128))) return rc;
    ULG_HIP(c, hipMemcpyAsync(s.d_rowmeta.p, meta.data(), 128 * 4, hipMemcpyHostToDevice, c->stream));
    const SearchDev d = s.dev();
    float *host = static_cast<float *>(s.host_rows.p);
    s.rows_ready = false;
    for (uint64_t r0 = 0; r0 < rows; r0 += chunk_rows) {
        if (deadline_ns &&
            std::chrono::steady_clock::now().time_since_epoch().count() > deadline_ns) {
            ULG_HIP(c, hipStreamSynchronize(c->stream));
            prof_collect(c);
            if (timed_out) *timed_out = true;
            return ULG_OK;
        }
        const uint64_t cnt = std::min(chunk_rows, rows - r0);
        const uint64_t work = cnt * (uint64_t)W;
        prof_begin(c, "bs_cost_rows");
        cost_rows_kernel<<<flat_grid((work + kB - 1) / kB), kB, 0, c->stream>>>(d, s.d_rowmeta.p, m, nl, r0, cnt,
                                                                                  s.d_rows.p);
        prof_end(c);
        ULG_HIP(c, hipGetLastError());
        ULG_HIP(c, hipMemcpyAsync(host + r0 * (uint64_t)W, s.d_rows.p, (size_t)work * 4, hipMemcpyDeviceToHost,
                                  c->stream));
    }
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    s.rows_scope = scope;
    s.rows_scc = scc;
    s.rows_ready = true;
    return ULG_OK;
}

int search_query(ulg_ctx *c, int64_t count, const int *vars, const uint64_t *S, float *costs, uint64_t *parents) {
    SearchState &s = *c->search;
    int rc;
    if ((rc = ensure(c, s.q_vars, (size_t)count)) || (rc = ensure(c, s.q_sets, (size_t)count)) ||
        (rc = ensure(c, s.q_costs, (size_t)count)) || (rc = ensure(c, s.q_par, (size_t)count)))
        return rc;
    ULG_HIP(c, hipMemcpyAsync(s.q_vars.p, vars, (size_t)count * 4, hipMemcpyHostToDevice, c->stream));
    ULG_HIP(c, hipMemcpyAsync(s.q_sets.p, S, (size_t)count * 8, hipMemcpyHostToDevice, c->stream));
    query_kernel<<<(unsigned)count, kB, 0, c->stream>>>(s.dev(), count, s.q_vars.p, s.q_sets.p, s.q_costs.p,
                                                         s.q_par.p);
    ULG_HIP(c, hipGetLastError());
    if (costs) ULG_HIP(c, hipMemcpyAsync(costs, s.q_costs.p, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
    if (parents) ULG_HIP(c, hipMemcpyAsync(parents, s.q_par.p, (size_t)count * 8, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return ULG_OK;
}

int search_pdb_query(ulg_ctx *c, int64_t count, const uint64_t *S, float *h, int *complete) {
    SearchState &s = *c->search;
    int rc;
    if ((rc = ensure(c, s.q_sets, (size_t)count)) || (rc = ensure(c, s.q_costs, (size_t)count)) ||
        (rc = ensure(c, s.q_vars, (size_t)count)))
        return rc;
    ULG_HIP(c, hipMemcpyAsync(s.q_sets.p, S, (size_t)count * 8, hipMemcpyHostToDevice, c->stream));
    pdb_query_kernel<<<(unsigned)((count + kB - 1) / kB), kB, 0, c->stream>>>(s.dev(), count, s.q_sets.p, s.q_costs.p,
                                                                           s.q_vars.p);
    ULG_HIP(c, hipGetLastError());
    ULG_HIP(c, hipMemcpyAsync(h, s.q_costs.p, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
    if (complete) ULG_HIP(c, hipMemcpyAsync(complete, s.q_vars.p, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return ULG_OK;
}

}  // namespace ulg
