// cbic_pipe.h -- the persistent scoring pipeline (cbic_pipe.hip) as seen by
// the scoring call (cbic.hip): per-(variable, stage) tables, the launch
// arguments and the host entry points.
#pragma once
#include <cstdint>
#include <vector>

#include "ulg_internal.h"

namespace ulg {

constexpr int kPipeMaxL = 6;       // layers the pipeline runs (the bit-sliced walk's unrolled range)
constexpr int kPipeMaxSmall = 4;   // one-pass stages (score_small_layers) at most up to this layer

// per (variable, stage s = 2 (L - 1) + phase), built on the host per call shape
struct PipeStage {
    uint32_t nsets;   // parent sets of the stage
    uint32_t ntiles;  // score tiles (64 x rounds sets each)
    uint32_t foff;    // first walk-chunk fill counter
    uint32_t next;    // the variable's next stage with sets (0xFFFFFFFF: none)
    uint32_t slab;    // first float of the stage's values in the work layout (a 128-byte line)
    uint32_t pad;
    uint64_t qoff;    // first queue word of the stage's walk entries
};

// per (variable, stage) counters, one 64-byte line each, zeroed every call
struct PipeCtr {
    uint32_t claim;   // next score tile to hand out
    uint32_t qlen;    // walk entries reserved
    uint32_t wclaim;  // next walk chunk to hand out
    uint32_t pad0;
    uint64_t units;   // tiles done << 32 + (entries walked - entries queued)
    uint64_t pad[5];
};
static_assert(sizeof(PipeCtr) == 64, "one line per stage counter");

struct PipeArgs {
    const double *gram;
    const uint32_t *binom;
    const uint8_t *cand;
    const int *meta;
    const uint64_t *tbl_off;
    const PipeStage *stages;  // [nv][NS]
    PipeCtr *ctr;             // [nv][NS]
    uint32_t *fill;           // walk-chunk fill counters
    uint32_t *done;           // [0] variables finished, [1] stall flag
    uint32_t *stage_of;       // [nv] each variable's current stage
    uint64_t *queue;
    float *table;             // colex-ordered slabs (read by the compaction after the launch)
    float *ptab, *phsub;      // work layout: values / subset maxima, one line-aligned slab per stage
    double N, lambda;
    int n, nv, S, NS, kmax;
    int Ls;       // layers <= Ls: one-pass tiles
    int R;        // rounds (x 64 sets) per two-pass tile
    int Rsmall;   // rounds per one-pass tile
    int chain;    // the wave that releases a stage starts on it (pipe_chain)
    uint32_t total_slots;  // table slots (a walk entry's slots are checked against them)
    uint32_t work_slots;   // work-layout slots
    uint64_t timeout;  // wall-clock ticks a wave may stay idle before the call fails
    uint64_t *stats;   // ULG_PIPE_STATS: 10 counters summed over waves (nullptr: off)
};

// LDS of one workgroup: the shared read-only tables, then per wave its pool
// of undecided sets (kPipePool entries: compact mask, work slot, ts, children
// max, table slot)
constexpr int kPipePool = 128;
constexpr int kPipePoolBytes = kPipePool * (8 + 4 + 4 + 4 + 4);
struct PipeLds {
    int gram, binom, toff, meta, pool, total;
};
__host__ __device__ inline int pipe_align16(int x) { return (x + 15) & ~15; }
__host__ __device__ inline PipeLds pipe_lds(int n, int nv, int S) {
    PipeLds l;
    l.gram = 0;
    l.binom = pipe_align16(l.gram + n * n * 8);
    l.toff = pipe_align16(l.binom + 64 * kBinomK * 4);
    l.meta = pipe_align16(l.toff + (nv * S + 1) * 8);
    l.pool = pipe_align16(l.meta + nv * 4 * 4);
    l.total = l.pool + 4 * kPipePoolBytes;  // 256-thread workgroups: 4 waves
    return l;
}
int pipe_chunk_sets(int L);
int pipe_entry_words(int L);

// Builds the stage table for this call shape, sizes and uploads the state
// (cached on the context until the shape changes), and fills `a`.
int pipe_prepare(ulg_ctx *c, int nv, int S, int kmax, int max_parents, const std::vector<int> &mv,
                 const std::vector<int> &meta, PipeArgs &a);
// Per call: reset the counters (memset + copy of the initial stages) and
// launch the persistent kernel on stream st.
int pipe_launch(ulg_ctx *c, const PipeArgs &a, hipStream_t st);
// After the call: 0, or ULG_ERR_HIP when a wave reported a stall.
int pipe_check(ulg_ctx *c);
// ULG_PIPE_STATS: print the last call's per-activity wave time on stderr
void pipe_report(ulg_ctx *c);

}  // namespace ulg
