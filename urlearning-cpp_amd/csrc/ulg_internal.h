// ulg_internal.h -- shared host-side state of the MI355X URLearning path.
#pragma once

#include <mutex>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <cstring>
#include <set>
#include <vector>

#include "../../include/ulg.h"

namespace ulg {

constexpr int kMaxVars = 63;               // varset = uint64, bit 63 kept free
constexpr int kMaxL = ULG_UNROLLED_PARENTS_GPU;  // unrolled layers on the device
constexpr int kWideMax = ULG_MAX_PARENTS_GPU;   // wide layers kMaxL+1 .. kWideMax (cbic.hip)
constexpr int kBinomK = kMaxL + 2;          // binomial table columns C(a, 0..kBinomK-1)
constexpr uint32_t kAbsentBits = 0xFFFFFFFFu;  // "not in the FloatMap" sentinel (a NaN payload)

// Device buffer that only grows.
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
};

struct SearchState;
struct PssState;

struct ProfRec {
    std::string name;
    hipEvent_t start, stop;
    bool graph = false;  // recorded by a captured graph (its events stay with the graph)
};

// Host copy of what was last uploaded into a device buffer: repeated calls
// with the same layout metadata skip the pageable H2D copies.
struct Mirror {
    const void *dev = nullptr;
    std::vector<unsigned char> bytes;
};

}  // namespace ulg

struct ulg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // ---- data (BIC_OLS ctor) ----
    int n = 0;
    int64_t N = 0;
    int npad = 0;
    double lambda = 0.0;
    bool loaded = false;
    ulg::DevBuf<double> raw, z, gram, partials, colstat;

    // ---- scoring state ----
    int nv = 0;
    int kmax = 0;
    std::vector<int> vars;
    std::vector<int> m;           // candidate count per batch variable
    std::vector<uint64_t> tbl_off;  // [nv][kmax+2] flattened prefix of table slots
    int64_t total_slots = 0;
    int64_t total_stored = 0;
    int64_t total_scored = 0;
    bool scored = false;
    int score_variant = 241;
    int walk_bucket = 1;  // layers 5, 6: walk the queue sorted by walk key (walk_bucket_kernel)
    int score_streams = 3;                  // scorer variable groups on concurrent streams
    int score_small_layers = 4;             // layers <= this run one-pass on one stream (two-pass variants)
    int score_fused = 3;                    // ... and layers <= this (<= small layers) in one launch, a workgroup per variable
    std::vector<hipStream_t> aux_streams;   // created on first use
    std::vector<hipEvent_t> sync_events;
    int64_t time_limit_ms = 0;     // -r: wall-clock budget per scoring call / search (0 = none)
    int out_of_time = 0;           // the last scoring call or search ran out of its budget
    int completed_layer = -1;      // highest fully scored layer of the last scoring call
    int64_t exact_pmu[3] = {-1, -1, -1};  // last exact A*: user-space cycles, instructions, cache misses (-1: n/a)
    uint64_t table_budget_kb = 0;  // best-score table budget in KiB (0 = half the free HBM)
    int sweep_table = 1;
    int wide_prune = 1;            // wide walks: skip absent nodes whose subsets hold no key >= -ts
    int wide_reduced = 1;          // wide walks: skip the recursion's no-op re-tests
    int wide_lds = 1;              // wide walks: long ones replayed with their bitsets in LDS
    int wide_pool = 2;             // wide layers variable by variable on score_streams host threads (2: auto)
    uint64_t wide_host_iters = 1024;     // LDS replays past this many iterations finish on host threads (0: never)
    int wide_host_threads = 16;          // host threads per wide-layer launch for those replays
    uint64_t wide_host_max = 4096;       // ... in launches of at most this many LDS replays
    uint64_t wide_host_first = 0;        // launches of at most this many replays go to the host whole
    int wide_host_q = 0;                 // ... as do launches of <= 128 replays with q >= this (0: off)
    int score_xcd = 1;             // scoring kernels: contiguous runs of sets per XCD
    int score_graph = 1;           // scoring call: replay the captured launch sequence
    hipGraph_t graph = nullptr;    // the captured scoring launches, its instance, its key
    hipGraphExec_t gexec = nullptr;
    std::vector<uint64_t> gkey;
    std::vector<ulg::ProfRec> gprof;  // profiling events inside the graph
    int sweep_xcd = 1;             // GPU sweep launches: contiguous runs of nodes per XCD           // GPU search: successor costs in the sweep's (layer, colex) order
    ulg::DevBuf<float> table;
    ulg::DevBuf<float> d_hsub;    // score_variant bit 6: subset maxima, table layout
    ulg::DevBuf<uint64_t> d_tbl_off, d_work, d_blk;
    ulg::DevBuf<uint8_t> d_cand;  // [nv][64] compact index -> variable
    ulg::DevBuf<int> d_meta;      // [nv][4]: var, m, var0in, pad
    ulg::DevBuf<uint32_t> d_binom;
    ulg::DevBuf<uint64_t> d_binom64;              // [64][64] unclamped C(a, b) for the wide layers
    ulg::DevBuf<uint64_t> d_wqueue;               // wide layers: sets left for the walk
    ulg::DevBuf<uint64_t> d_wbits;                // wide layers: per-walk checked bitsets
    ulg::DevBuf<unsigned long long> d_stats;  // score_variant 13 statistics
    ulg::DevBuf<uint64_t> d_dump;
    ulg::DevBuf<uint64_t> d_queue;                // score_variant bit 4: undecided lanes
    ulg::DevBuf<uint32_t> d_qaux, d_qsidx, d_qoffs;  // walk_bucket: key/rank, sorted index, key bases
    ulg::DevBuf<uint8_t> d_qkey;                            // walk_bucket: each queue entry's walk key
    ulg::DevBuf<unsigned long long> d_qseg;       // ... their per-segment counters (cbic.hip kSegBlocks)
    ulg::DevBuf<unsigned long long> d_qcount;
    ulg::DevBuf<uint64_t> d_workg;                // per stream-group work prefixes
    ulg::DevBuf<uint64_t> d_vwork;                // per-variable work prefixes of the wide-layer pool
    ulg::DevBuf<uint32_t> d_hq;                   // per stream group: replays handed to the host
    ulg::DevBuf<unsigned int> d_hqc;
    ulg::DevBuf<uint64_t> out_sets;
    ulg::DevBuf<float> out_scores;
    ulg::DevBuf<int64_t> out_offsets;

    ulg::DevBuf<float> qbuf_in, qbuf_out;
    ulg::DevBuf<uint64_t> d_sets_in;              // ulg_cbic_score_sets: (variable, parent mask) pairs

    // ---- search side (best-score tables, pattern database, A*) ----
    ulg::SearchState *search = nullptr;

    // ---- .pss text formatting (pss.hip) ----
    ulg::PssState *pss = nullptr;

    // ---- profiling ----
    bool prof = false;
    std::vector<ulg::ProfRec> pending;
    std::set<std::string> prof_only;  // ulg_profile_select: time only these kernels
    std::mutex mu;  // err / pending: the wide scoring layers use one host thread per stream group
    std::vector<hipEvent_t> event_pool;
    ulg::Mirror mir_tbl_off, mir_work, mir_cand, mir_meta, mir_workg, mir_hoff, mir_vwork;
    ulg::DevBuf<float> d_hmax;      // wide walks: hi-cover tables (subset max of the present keys), then the present keys
    uint64_t hmax_half = 0;         // entries of each half of d_hmax
    ulg::DevBuf<uint64_t> d_hoff;   // [nv] table offsets, ~0 = no table
    ulg::DevBuf<int> d_hmeta;       // per stream group: launch variables and tile / block prefixes
    ulg::DevBuf<unsigned long long> d_scount;  // per stream group: long wide walks handed to the LDS kernel
    unsigned long long *wide_pinned = nullptr;  // pinned queue / long-walk counts of the wide stages
    // ulg_cbic_score_async: the stored count lands here when the launches
    // finish; ulg_cbic_score_finish (or any later scorer call) collects it
    unsigned long long *async_pinned = nullptr;  // [stored count, error word] of the last call
    unsigned long long last_err_word = 0;        // the last scoring call's error word (kErr* bits)
    bool async_pending = false;
    std::vector<unsigned long long> wide_host;
    std::map<std::string, std::vector<double>> prof_ms;

    int64_t walk_small_sets = 200000;  // layer-6 launches below this many sets walk one set per lane
    int walk_k6 = 4;                   // sets per lane of the layer-6 walk launches (1, 2, 4 or 8)
};

namespace ulg {

// error helpers -----------------------------------------------------------
int set_err(ulg_ctx *c, int code, const std::string &msg);

#define ULG_HIP(ctx, expr)                                                          \
    do {                                                                            \
        hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess)                                                       \
            return ::ulg::set_err((ctx), ULG_ERR_HIP,                               \
                                  std::string(#expr " failed: ") + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
int ensure(ulg_ctx *c, DevBuf<T> &b, size_t elems) {
    if (elems == 0) elems = 1;
    if (b.cap >= elems) return ULG_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    // 16 bytes of slack: kernels copy whole 16-byte chunks (fill_lds), so the
    // last chunk of an array may read up to 15 bytes past its end
    hipError_t e = hipMalloc(&b.p, elems * sizeof(T) + 16);
    if (e != hipSuccess)
        return set_err(c, ULG_ERR_HIP, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    b.cap = elems;
    return ULG_OK;
}

template <typename T>
int upload(ulg_ctx *c, DevBuf<T> &b, Mirror &m, const std::vector<T> &h) {
    const size_t nbytes = h.size() * sizeof(T);
    if (int rc = ensure(c, b, h.size())) return rc;
    if (m.dev == b.p && m.bytes.size() == nbytes && std::memcmp(m.bytes.data(), h.data(), nbytes) == 0) return ULG_OK;
    hipError_t e = hipMemcpyAsync(b.p, h.data(), nbytes, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return set_err(c, ULG_ERR_HIP, std::string("hipMemcpyAsync failed: ") + hipGetErrorString(e));
    m.dev = b.p;
    m.bytes.assign(reinterpret_cast<const unsigned char *>(h.data()),
                   reinterpret_cast<const unsigned char *>(h.data()) + nbytes);
    return ULG_OK;
}

template <typename T>
void release(DevBuf<T> &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
}

// profiling: bracket a launch with events when enabled
void prof_begin(ulg_ctx *c, const char *name);
void prof_end(ulg_ctx *c);
void prof_begin_s(ulg_ctx *c, const char *name, hipStream_t stream);
void prof_end_s(ulg_ctx *c, hipStream_t stream);
void prof_collect(ulg_ctx *c);  // after a stream sync
void graph_reset(ulg_ctx *c);   // drop the captured scoring graph (cbic.hip)
void pss_release(ulg_ctx *c);    // pss.hip

// binomial table C(a, b), a < 64, b < kBinomK, clamped to uint32
const std::vector<uint32_t> &host_binom();
// C(a, b) for a, b < 64 (saturating at 2^64 - 1), [a * 64 + b]
const std::vector<uint64_t> &host_binom64();
uint64_t binom64(int a, int b);

}  // namespace ulg
