// ulg_ctx.cpp -- context lifecycle, errors, profiling for libulg.so.
#include <mutex>
#include <cstdio>
#include <cstring>

#include "search_internal.h"

namespace ulg {

int set_err(ulg_ctx *c, int code, const std::string &msg) {
    if (c) {
        // the wide scoring layers run one host thread per stream group
        std::lock_guard<std::mutex> lk(c->mu);
        c->err = msg;
    }
    return code;
}

const std::vector<uint32_t> &host_binom() {
    static std::vector<uint32_t> t = [] {
        std::vector<uint32_t> b(64 * kBinomK, 0);
        for (int a = 0; a < 64; ++a)
            for (int k = 0; k < kBinomK; ++k) {
                uint64_t v = binom64(a, k);
                b[a * kBinomK + k] = v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
            }
        return b;
    }();
    return t;
}

const std::vector<uint64_t> &host_binom64() {
    static std::vector<uint64_t> t = [] {
        std::vector<uint64_t> b(64 * 64, 0);
        for (int a = 0; a < 64; ++a)
            for (int k = 0; k < 64; ++k) b[a * 64 + k] = binom64(a, k);
        return b;
    }();
    return t;
}

uint64_t binom64(int a, int b) {
    if (b < 0 || b > a) return 0;
    if (b > a - b) b = a - b;
    unsigned __int128 r = 1;
    for (int i = 1; i <= b; ++i) r = r * (unsigned)(a - b + i) / (unsigned)i;
    return r > ~0ull ? ~0ull : (uint64_t)r;
}

void prof_begin(ulg_ctx *c, const char *name) { prof_begin_s(c, name, c->stream); }
void prof_end(ulg_ctx *c) { prof_end_s(c, c->stream); }

// The record a thread's prof_end_s closes: its own last prof_begin_s (the
// wide scoring layers drive their stream groups from several host threads).
thread_local int64_t t_prof_rec = -1;

void prof_begin_s(ulg_ctx *c, const char *name, hipStream_t stream) {
    t_prof_rec = -1;
    if (!c->prof || (!c->prof_only.empty() && !c->prof_only.count(name))) return;
    std::lock_guard<std::mutex> lk(c->mu);
    ProfRec r;
    r.name = name;
    // events come from a per-context pool: creating two per kernel costs more
    // than the small layers' kernels themselves
    for (hipEvent_t *e : {&r.start, &r.stop}) {
        if (!c->event_pool.empty()) {
            *e = c->event_pool.back();
            c->event_pool.pop_back();
        } else {
            (void)hipEventCreate(e);
        }
    }
    (void)hipEventRecord(r.start, stream);
    t_prof_rec = (int64_t)c->pending.size();
    c->pending.push_back(r);
}

void prof_end_s(ulg_ctx *c, hipStream_t stream) {
    if (t_prof_rec < 0) return;
    std::lock_guard<std::mutex> lk(c->mu);
    if (t_prof_rec < (int64_t)c->pending.size()) (void)hipEventRecord(c->pending[(size_t)t_prof_rec].stop, stream);
    t_prof_rec = -1;
}

void prof_collect(ulg_ctx *c) {
    for (auto &r : c->pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.stop) == hipSuccess && hipEventElapsedTime(&ms, r.start, r.stop) == hipSuccess)
            c->prof_ms[r.name].push_back(ms);
        if (r.graph) continue;  // the graph records these again on every replay
        c->event_pool.push_back(r.start);
        c->event_pool.push_back(r.stop);
    }
    c->pending.clear();
}

void graph_reset(ulg_ctx *c) {
    (void)hipStreamSynchronize(c->stream);
    prof_collect(c);
    if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    c->gexec = nullptr;
    c->graph = nullptr;
    c->gkey.clear();
    for (const ProfRec &r : c->gprof) {
        c->event_pool.push_back(r.start);
        c->event_pool.push_back(r.stop);
    }
    c->gprof.clear();
}

}  // namespace ulg

using namespace ulg;

extern "C" {

const char *ulg_version(void) { return "ulg 0.1 (HIP, gfx950/CDNA4)"; }

int ulg_create(const int *device_ids, int ndev, ulg_ctx **out) {
    if (!out) return ULG_ERR_ARG;
    *out = nullptr;
    if (ndev != 1 || !device_ids) return ULG_ERR_ARG;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) {
        fprintf(stderr, "ulg_create: no HIP device available (%s)\n", hipGetErrorString(e));
        return ULG_ERR_HIP;
    }
    if (device_ids[0] < 0 || device_ids[0] >= count) return ULG_ERR_ARG;
    ulg_ctx *c = new ulg_ctx();
    c->device = device_ids[0];
    if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return ULG_ERR_HIP;
    }
    const auto &b = host_binom();
    if (ensure(c, c->d_binom, b.size()) != ULG_OK ||
        hipMemcpy(c->d_binom.p, b.data(), b.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess ||
        ensure(c, c->d_binom64, host_binom64().size()) != ULG_OK ||
        hipMemcpy(c->d_binom64.p, host_binom64().data(), host_binom64().size() * sizeof(uint64_t),
                  hipMemcpyHostToDevice) != hipSuccess) {
        delete c;
        return ULG_ERR_HIP;
    }
    *out = c;
    return ULG_OK;
}

void ulg_destroy(ulg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    graph_reset(c);
    if (c->wide_pinned) (void)hipHostFree(c->wide_pinned);
    c->wide_pinned = nullptr;
    if (c->async_pinned) (void)hipHostFree(c->async_pinned);
    c->async_pinned = nullptr;
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    c->event_pool.clear();
    for (hipStream_t s : c->aux_streams) (void)hipStreamDestroy(s);
    c->aux_streams.clear();
    for (hipEvent_t e : c->sync_events) (void)hipEventDestroy(e);
    c->sync_events.clear();
    release(c->raw); release(c->z); release(c->gram); release(c->partials); release(c->colstat);
    release(c->table); release(c->d_tbl_off); release(c->d_work); release(c->d_blk);
    release(c->d_cand); release(c->d_meta); release(c->d_binom); release(c->d_binom64); release(c->d_wqueue); release(c->d_wbits); release(c->d_stats); release(c->d_dump); release(c->d_queue); release(c->d_qcount); release(c->d_workg); release(c->d_vwork); release(c->d_hq); release(c->d_hqc); release(c->d_hmax); release(c->d_hoff); release(c->d_hmeta); release(c->d_scount); release(c->d_hsub); release(c->d_qseg);
    release(c->d_qaux); release(c->d_qsidx); release(c->d_qoffs); release(c->d_qkey);
    release(c->out_sets); release(c->out_scores); release(c->out_offsets);
    release(c->qbuf_in); release(c->qbuf_out);
    pss_release(c);
    if (c->search) {
        c->search->release_all();
        delete c->search;
        c->search = nullptr;
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *ulg_last_error(const ulg_ctx *c) { return c ? c->err.c_str() : "null context"; }

int ulg_set_option(ulg_ctx *c, const char *name, int64_t value) {
    if (!c || !name) return ULG_ERR_ARG;
    if (std::strcmp(name, "score_streams") == 0) {
        if (value < 1 || value > 4) return set_err(c, ULG_ERR_ARG, "score_streams must be 1..4");
        c->score_streams = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "score_small_layers") == 0) {
        if (value < 0 || value > ULG_UNROLLED_PARENTS_GPU)
            return set_err(c, ULG_ERR_ARG, "score_small_layers must be 0..8");
        c->score_small_layers = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "score_fused") == 0) {
        if (value < 0 || value > 4) return set_err(c, ULG_ERR_ARG, "score_fused must be 0..4");
        c->score_fused = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "score_variant") == 0) {
        if (value != 1 && value != 49 && value != 65 && value != 113 && value != 241)
            return set_err(c, ULG_ERR_ARG, "score_variant must be 1, 49, 65, 113 or 241");
        c->score_variant = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "time_limit_ms") == 0) {
        if (value < 0) return set_err(c, ULG_ERR_ARG, "time_limit_ms must be >= 0");
        c->time_limit_ms = value;
        return ULG_OK;
    }
    if (std::strcmp(name, "table_budget_kb") == 0) {
        if (value < 0) return set_err(c, ULG_ERR_ARG, "table_budget_kb must be >= 0");
        c->table_budget_kb = (uint64_t)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "sweep_xcd") == 0) {
        if (value < 0 || value > 1) return set_err(c, ULG_ERR_ARG, "sweep_xcd must be 0 or 1");
        c->sweep_xcd = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "walk_k6") == 0) {
        if (value != 1 && value != 2 && value != 4 && value != 8)
            return set_err(c, ULG_ERR_ARG, "walk_k6 must be 1, 2, 4 or 8");
        c->walk_k6 = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "walk_bucket") == 0) {
        if (value != 0 && value != 1) return set_err(c, ULG_ERR_ARG, "walk_bucket must be 0 or 1");
        c->walk_bucket = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "walk_small_sets") == 0) {
        if (value < 0) return set_err(c, ULG_ERR_ARG, "walk_small_sets must be >= 0");
        c->walk_small_sets = value;
        return ULG_OK;
    }
    if (std::strcmp(name, "score_graph") == 0) {
        if (value < 0 || value > 1) return set_err(c, ULG_ERR_ARG, "score_graph must be 0 or 1");
        c->score_graph = (int)value;
        if (!value) graph_reset(c);
        return ULG_OK;
    }
    if (std::strcmp(name, "score_xcd") == 0) {
        if (value < 0 || value > 1) return set_err(c, ULG_ERR_ARG, "score_xcd must be 0 or 1");
        c->score_xcd = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_host") == 0) {
        if (value < 0) return set_err(c, ULG_ERR_ARG, "wide_host must be >= 0");
        c->wide_host_iters = (uint64_t)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_host_max") == 0) {
        if (value < 0) return set_err(c, ULG_ERR_ARG, "wide_host_max must be >= 0");
        c->wide_host_max = (uint64_t)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_host_first") == 0) {
        if (value < 0) return set_err(c, ULG_ERR_ARG, "wide_host_first must be >= 0");
        c->wide_host_first = (uint64_t)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_host_q") == 0) {
        if (value < 0 || value > 32) return set_err(c, ULG_ERR_ARG, "wide_host_q must be 0..32");
        c->wide_host_q = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_host_threads") == 0) {
        if (value < 1 || value > 64) return set_err(c, ULG_ERR_ARG, "wide_host_threads must be 1..64");
        c->wide_host_threads = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_pool") == 0) {
        if (value < 0 || value > 2) return set_err(c, ULG_ERR_ARG, "wide_pool must be 0, 1 or 2");
        c->wide_pool = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_lds") == 0) {
        if (value < 0 || value > 2) return set_err(c, ULG_ERR_ARG, "wide_lds must be 0, 1 or 2");
        c->wide_lds = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_reduced") == 0) {
        if (value < 0 || value > 1) return set_err(c, ULG_ERR_ARG, "wide_reduced must be 0 or 1");
        c->wide_reduced = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "wide_prune") == 0) {
        if (value < 0 || value > 1) return set_err(c, ULG_ERR_ARG, "wide_prune must be 0 or 1");
        c->wide_prune = (int)value;
        return ULG_OK;
    }
    if (std::strcmp(name, "sweep_table") == 0) {
        if (value < 0 || value > 2) return set_err(c, ULG_ERR_ARG, "sweep_table must be 0, 1 or 2");
        c->sweep_table = (int)value;
        return ULG_OK;
    }
    return set_err(c, ULG_ERR_ARG, std::string("unknown option: ") + name);
}

int ulg_get_info(ulg_ctx *c, const char *name, int64_t *value) {
    if (!c || !name || !value) return ULG_ERR_ARG;
    if (std::strcmp(name, "out_of_time") == 0) {
        *value = c->out_of_time;
        return ULG_OK;
    }
    if (std::strcmp(name, "highest_completed_layer") == 0) {
        *value = c->completed_layer;
        return ULG_OK;
    }
    // the last scoring call's device error word: 0 unless a walk over its cap
    // (1), a walk-queue segment overflow (2) or a walk entry past the table (4)
    if (std::strcmp(name, "score_error_word") == 0) {
        *value = (int64_t)c->last_err_word;
        return ULG_OK;
    }
    // the last exact A*'s host counters (user space, the calling thread; -1: not granted)
    if (std::strcmp(name, "exact_cycles") == 0) {
        *value = c->exact_pmu[0];
        return ULG_OK;
    }
    if (std::strcmp(name, "exact_instructions") == 0) {
        *value = c->exact_pmu[1];
        return ULG_OK;
    }
    if (std::strcmp(name, "exact_cache_misses") == 0) {
        *value = c->exact_pmu[2];
        return ULG_OK;
    }
    return set_err(c, ULG_ERR_ARG, std::string("unknown info: ") + name);
}

int ulg_stream_wait_event(ulg_ctx *c, void *event) {
    if (!c || !event) return ULG_ERR_ARG;
    ULG_HIP(c, hipSetDevice(c->device));
    ULG_HIP(c, hipStreamWaitEvent(c->stream, (hipEvent_t)event, 0));
    return ULG_OK;
}

int ulg_profile_enable(ulg_ctx *c, int on) {
    if (!c) return ULG_ERR_ARG;
    c->prof = on != 0;
    return ULG_OK;
}

int ulg_profile_select(ulg_ctx *c, const char *names) {
    if (!c) return ULG_ERR_ARG;
    c->prof_only.clear();
    if (names) {
        std::string cur;
        for (const char *p = names;; ++p) {
            if (*p == ',' || *p == 0) {
                if (!cur.empty()) c->prof_only.insert(cur);
                cur.clear();
                if (*p == 0) break;
            } else {
                cur += *p;
            }
        }
    }
    return ULG_OK;
}

int ulg_profile_reset(ulg_ctx *c) {
    if (!c) return ULG_ERR_ARG;
    (void)hipStreamSynchronize(c->stream);
    prof_collect(c);
    c->prof_ms.clear();
    return ULG_OK;
}

int ulg_profile_get(ulg_ctx *c, const char *name, double *avg_ms, int64_t *count, double *total_ms) {
    if (!c || !name) return ULG_ERR_ARG;
    (void)hipStreamSynchronize(c->stream);
    prof_collect(c);
    auto it = c->prof_ms.find(name);
    if (it == c->prof_ms.end() || it->second.empty()) return ULG_ERR_ARG;
    double t = 0;
    for (double v : it->second) t += v;
    if (avg_ms) *avg_ms = t / (double)it->second.size();
    if (count) *count = (int64_t)it->second.size();
    if (total_ms) *total_ms = t;
    return ULG_OK;
}

int ulg_profile_dump(ulg_ctx *c, char *buf, int64_t cap) {
    if (!c || !buf || cap <= 0) return ULG_ERR_ARG;
    (void)hipStreamSynchronize(c->stream);
    prof_collect(c);
    int64_t len = 0;
    buf[0] = 0;
    for (auto &kv : c->prof_ms) {
        double t = 0;
        for (double v : kv.second) t += v;
        int w = snprintf(buf + len, (size_t)(cap - len), "%s %zu %.6f\n", kv.first.c_str(), kv.second.size(), t);
        if (w < 0 || len + w >= cap) break;
        len += w;
    }
    return ULG_OK;
}

}  // extern "C"
