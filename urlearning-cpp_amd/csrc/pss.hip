// pss.hip -- the .pss score-cache text, formatted on the GPU.
//
// Reference (urlearning/): scoringThread prints one line per stored parent
// set, "%f " of the score followed by each parent's name and a space
// (score/score_main.cpp:173-203), under "VAR name" / "META arity=a" and a
// file-level META block (score_main.cpp:383-400).  At C3 (1.6 M stored sets,
// 124 MB of text) the host printf loop took 20x longer than the scoring it
// reports on; here every line is formatted by its own thread:
//   1. pss_len_kernel   -- byte length of every line
//   2. exclusive scan   -- line offsets (hipcub)
//   3. pss_write_kernel -- the bytes, glibc "%f" digit for digit
// and the host only drops the VAR / META / blank lines into the gaps.
//
// "%f" of (double)x for a float x is exact in glibc: the decimal expansion of
// the binary value rounded to 6 fraction digits, ties to even.  With
// x = M * 2^E: E >= 0 means an integer (up to 2^128, no fraction); E < 0 means
// D = round-half-even(M * 10^6 / 2^-E) < 2^44, integer part D / 10^6 and
// fraction D % 10^6 -- the same exact integer rounding as quantize_score.
#include <hipcub/hipcub.hpp>

#include <cstring>

#include "ulg_internal.h"

using namespace ulg;

namespace {

constexpr int kB = 256;

struct F6 {  // a float as glibc's "%f" prints it
    uint64_t hi, lo;   // integer part (128 bits)
    uint32_t frac;     // 6 fraction digits
    uint8_t neg, kind; // kind: 0 finite, 1 inf, 2 nan
};

__device__ __forceinline__ F6 split_f6(float x) {
    const uint32_t u = __float_as_uint(x);
    F6 r;
    r.neg = (uint8_t)(u >> 31);
    r.hi = r.lo = 0;
    r.frac = 0;
    const uint32_t ex = (u >> 23) & 0xffu;
    if (ex == 0xffu) {
        r.kind = (u & 0x7fffffu) ? 2 : 1;
        return r;
    }
    r.kind = 0;
    uint64_t M;
    int E;
    if (ex == 0) { M = u & 0x7fffffu; E = -149; }
    else { M = (u & 0x7fffffu) | 0x800000u; E = (int)ex - 150; }
    if (E >= 0) {  // an integer M * 2^E < 2^128
        if (E == 0) { r.lo = M; }
        else if (E < 64) { r.lo = M << E; r.hi = M >> (64 - E); }
        else { r.hi = M << (E - 64); }
        return r;
    }
    const int sh = -E;
    const uint64_t num = M * 1000000ull;  // < 2^44
    uint64_t D;
    if (sh >= 64) {
        D = 0;
    } else {
        D = num >> sh;
        const uint64_t rem = num & ((1ull << sh) - 1ull);
        const uint64_t half = 1ull << (sh - 1);
        if (rem > half || (rem == half && (D & 1ull))) ++D;
    }
    r.lo = D / 1000000ull;
    r.frac = (uint32_t)(D % 1000000ull);
    return r;
}

// (hi, lo) /= 10, returns the remainder
__device__ __forceinline__ uint32_t divmod10_128(uint64_t &hi, uint64_t &lo) {
    const uint64_t qh = hi / 10, rh = hi % 10;
    // (rh * 2^64 + lo) / 10 in 32-bit limbs
    const uint64_t a = (rh << 32) | (lo >> 32);
    const uint64_t qa = a / 10, ra = a % 10;
    const uint64_t b = (ra << 32) | (lo & 0xffffffffull);
    const uint64_t qb = b / 10, rb = b % 10;
    hi = qh;
    lo = (qa << 32) | qb;
    return (uint32_t)rb;
}

__device__ __forceinline__ int int_digits(uint64_t hi, uint64_t lo) {
    if (hi == 0) {
        int d = 1;
        uint64_t t = lo;
        while (t >= 10) { t /= 10; ++d; }
        return d;
    }
    int d = 0;
    while (hi || lo) { divmod10_128(hi, lo); ++d; }
    return d;
}

__device__ __forceinline__ int f6_len(const F6 &f) {
    if (f.kind == 1) return 3 + f.neg;             // inf / -inf
    if (f.kind == 2) return 3 + f.neg;             // nan / -nan
    return f.neg + int_digits(f.hi, f.lo) + 7;     // digits '.' 6 digits
}

__device__ __forceinline__ char *f6_write(const F6 &f, char *p) {
    if (f.neg) *p++ = '-';
    if (f.kind) {
        const char *s = f.kind == 1 ? "inf" : "nan";
        p[0] = s[0]; p[1] = s[1]; p[2] = s[2];
        return p + 3;
    }
    const int nd = int_digits(f.hi, f.lo);
    uint64_t hi = f.hi, lo = f.lo;
    for (int i = nd - 1; i >= 0; --i) {
        uint32_t dg;
        if (hi == 0) { dg = (uint32_t)(lo % 10); lo /= 10; }
        else dg = divmod10_128(hi, lo);
        p[i] = (char)('0' + dg);
    }
    p += nd;
    *p++ = '.';
    uint32_t fr = f.frac;
    for (int i = 5; i >= 0; --i) { p[i] = (char)('0' + fr % 10); fr /= 10; }
    return p + 6;
}

struct PssArgs {
    const uint64_t *sets;
    const float *scores;
    const int64_t *offsets;   // [nl+1] list boundaries (list order)
    int nl;
    const char *names;        // concatenated names
    const int *name_off;      // [n+1]
    int64_t total;
};

__device__ __forceinline__ int list_of(const int64_t *off, int nl, int64_t i) {
    int lo = 0, hi = nl;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kB) pss_len_kernel(PssArgs a, uint64_t *len) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i > a.total) return;
    if (i == a.total) { len[i] = 0; return; }
    int L = f6_len(split_f6(a.scores[i])) + 2;  // "%f " ... '\n'
    uint64_t s = a.sets[i];
    while (s) {
        const int p = __builtin_ctzll(s);
        s &= s - 1;
        L += a.name_off[p + 1] - a.name_off[p] + 1;
    }
    len[i] = (uint64_t)L;
}

__global__ void __launch_bounds__(kB) pss_gather_kernel(const uint64_t *pos, const int64_t *offsets, int nl,
                                                        uint64_t *out) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i <= nl) out[i] = pos[offsets[i]];
}

__global__ void __launch_bounds__(kB) pss_write_kernel(PssArgs a, const uint64_t *pos, const int64_t *base,
                                                       char *text) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= a.total) return;
    const int l = list_of(a.offsets, a.nl, i);
    char *p = text + base[l] + pos[i];
    p = f6_write(split_f6(a.scores[i]), p);
    *p++ = ' ';
    uint64_t s = a.sets[i];
    while (s) {
        const int v = __builtin_ctzll(s);
        s &= s - 1;
        for (int c = a.name_off[v]; c < a.name_off[v + 1]; ++c) *p++ = a.names[c];
        *p++ = ' ';
    }
    *p = '\n';
}

}  // namespace

namespace ulg {

struct PssState {
    DevBuf<uint64_t> len, pos, bounds, sets;
    DevBuf<int64_t> base, offsets;
    DevBuf<float> scores;
    DevBuf<char> names, text;
    DevBuf<int> name_off;
    DevBuf<unsigned char> scan_tmp;
    char *host = nullptr;
    size_t host_cap = 0;
};

void pss_release(ulg_ctx *c) {
    if (!c->pss) return;
    PssState &s = *c->pss;
    release(s.len); release(s.pos); release(s.bounds); release(s.sets); release(s.base); release(s.offsets);
    release(s.scores); release(s.names); release(s.text); release(s.name_off); release(s.scan_tmp);
    if (s.host) (void)hipHostFree(s.host);
    delete c->pss;
    c->pss = nullptr;
}

// lists: nl lists in list order; var_of_list[l] = the variable list l belongs
// to; every variable 0..n-1 has exactly one list.
static int pss_format_impl(ulg_ctx *c, int n, int nl, const int *var_of_list, const int64_t *h_offsets,
                           const int64_t *d_offsets, const uint64_t *d_sets, const float *d_scores, const char *header,
                           const char *const *names, const int *arity, const char **text, int64_t *len) {
    if (!c->pss) c->pss = new PssState();
    PssState &s = *c->pss;
    const int64_t total = h_offsets[nl];
    int rc;
    // names
    std::vector<int> name_off(n + 1, 0);
    std::string blob;
    for (int v = 0; v < n; ++v) {
        blob += names[v];
        name_off[v + 1] = (int)blob.size();
    }
    if ((rc = ensure(c, s.names, blob.size() + 1)) || (rc = ensure(c, s.name_off, (size_t)n + 1)) ||
        (rc = ensure(c, s.len, (size_t)total + 1)) || (rc = ensure(c, s.pos, (size_t)total + 1)) ||
        (rc = ensure(c, s.bounds, (size_t)nl + 1)) || (rc = ensure(c, s.base, (size_t)nl)))
        return rc;
    if (!blob.empty())
        ULG_HIP(c, hipMemcpyAsync(s.names.p, blob.data(), blob.size(), hipMemcpyHostToDevice, c->stream));
    ULG_HIP(c, hipMemcpyAsync(s.name_off.p, name_off.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    PssArgs a{d_sets, d_scores, d_offsets, nl, s.names.p, s.name_off.p, total};
    const unsigned g1 = (unsigned)((total + 1 + kB - 1) / kB);
    prof_begin(c, "pss_len");
    pss_len_kernel<<<g1, kB, 0, c->stream>>>(a, s.len.p);
    prof_end(c);
    size_t tmp = 0;
    ULG_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, s.len.p, s.pos.p, (int)(total + 1), c->stream));
    if ((rc = ensure(c, s.scan_tmp, tmp))) return rc;
    prof_begin(c, "pss_scan");
    ULG_HIP(c, hipcub::DeviceScan::ExclusiveSum(s.scan_tmp.p, tmp, s.len.p, s.pos.p, (int)(total + 1), c->stream));
    prof_end(c);
    pss_gather_kernel<<<(unsigned)((nl + 1 + kB - 1) / kB), kB, 0, c->stream>>>(s.pos.p, d_offsets, nl, s.bounds.p);
    std::vector<uint64_t> bounds(nl + 1);
    ULG_HIP(c, hipMemcpyAsync(bounds.data(), s.bounds.p, (size_t)(nl + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    // file layout: header, then per variable "VAR name\nMETA arity=a\n" + lines + "\n"
    std::vector<int> list_of_var(n, -1);
    for (int l = 0; l < nl; ++l) list_of_var[var_of_list[l]] = l;
    std::vector<std::string> vhead(n);
    std::vector<int64_t> vstart(n), base(nl);
    int64_t at = (int64_t)std::strlen(header);
    for (int v = 0; v < n; ++v) {
        const int l = list_of_var[v];
        vhead[v] = std::string("VAR ") + names[v] + "\nMETA arity=" + std::to_string(arity[v]) + "\n";
        vstart[v] = at;
        at += (int64_t)vhead[v].size();
        base[l] = at - (int64_t)bounds[l];
        at += (int64_t)(bounds[l + 1] - bounds[l]) + 1;  // lines + blank line
    }
    const int64_t bytes = at;
    if ((rc = ensure(c, s.text, (size_t)bytes))) return rc;
    ULG_HIP(c, hipMemcpyAsync(s.base.p, base.data(), (size_t)nl * 8, hipMemcpyHostToDevice, c->stream));
    prof_begin(c, "pss_write");
    if (total > 0)
        pss_write_kernel<<<(unsigned)((total + kB - 1) / kB), kB, 0, c->stream>>>(a, s.pos.p, s.base.p, s.text.p);
    prof_end(c);
    ULG_HIP(c, hipGetLastError());
    if (s.host_cap < (size_t)bytes) {
        if (s.host) (void)hipHostFree(s.host);
        s.host = nullptr;
        s.host_cap = 0;
        ULG_HIP(c, hipHostMalloc((void **)&s.host, (size_t)bytes + 1, hipHostMallocDefault));
        s.host_cap = (size_t)bytes;
    }
    ULG_HIP(c, hipMemcpyAsync(s.host, s.text.p, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    prof_collect(c);
    std::memcpy(s.host, header, std::strlen(header));
    for (int v = 0; v < n; ++v) {
        std::memcpy(s.host + vstart[v], vhead[v].data(), vhead[v].size());
        const int l = list_of_var[v];
        s.host[base[l] + (int64_t)bounds[l + 1]] = '\n';
    }
    s.host[bytes] = 0;
    *text = s.host;
    *len = bytes;
    return ULG_OK;
}

}  // namespace ulg

extern "C" {

int ulg_pss_format(ulg_ctx *c, const char *header, const char *const *names, const int *arity, const char **text,
                   int64_t *len) {
    if (!c || !header || !names || !arity || !text || !len) return ULG_ERR_ARG;
    if (c->async_pending) {  // an async scoring call still owns the lists
        const int rc0 = ulg_cbic_score_finish(c, nullptr, nullptr);
        if (rc0) return rc0;
    }
    if (!c->scored) return set_err(c, ULG_ERR_STATE, "ulg_pss_format: call ulg_cbic_score first");
    if (c->nv != c->n) return set_err(c, ULG_ERR_STATE, "ulg_pss_format: every variable must be scored in this context");
    ULG_HIP(c, hipSetDevice(c->device));
    std::vector<int64_t> offs(c->nv + 1);
    ULG_HIP(c, hipMemcpyAsync(offs.data(), c->out_offsets.p, (size_t)(c->nv + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    ULG_HIP(c, hipStreamSynchronize(c->stream));
    return pss_format_impl(c, c->n, c->nv, c->vars.data(), offs.data(), c->out_offsets.p, c->out_sets.p,
                           c->out_scores.p, header, names, arity, text, len);
}

int ulg_pss_format_lists(ulg_ctx *c, int n, const int64_t *offsets, const uint64_t *sets, const float *scores,
                         const char *header, const char *const *names, const int *arity, const char **text,
                         int64_t *len) {
    if (!c || n < 1 || n > 63 || !offsets || !header || !names || !arity || !text || !len) return ULG_ERR_ARG;
    const int64_t total = offsets[n];
    if (total < 0 || (total > 0 && (!sets || !scores))) return ULG_ERR_ARG;
    for (int v = 0; v < n; ++v)
        if (offsets[v + 1] < offsets[v]) return set_err(c, ULG_ERR_ARG, "ulg_pss_format_lists: bad offsets");
    for (int64_t i = 0; i < total; ++i)
        if (sets[i] >> n) return set_err(c, ULG_ERR_ARG, "ulg_pss_format_lists: parent outside the variables");
    ULG_HIP(c, hipSetDevice(c->device));
    if (!c->pss) c->pss = new PssState();
    PssState &s = *c->pss;
    int rc;
    if ((rc = ensure(c, s.sets, (size_t)total)) || (rc = ensure(c, s.scores, (size_t)total)) ||
        (rc = ensure(c, s.offsets, (size_t)n + 1)))
        return rc;
    if (total) {
        ULG_HIP(c, hipMemcpyAsync(s.sets.p, sets, (size_t)total * 8, hipMemcpyHostToDevice, c->stream));
        ULG_HIP(c, hipMemcpyAsync(s.scores.p, scores, (size_t)total * 4, hipMemcpyHostToDevice, c->stream));
    }
    ULG_HIP(c, hipMemcpyAsync(s.offsets.p, offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    std::vector<int> ident(n);
    for (int v = 0; v < n; ++v) ident[v] = v;
    return pss_format_impl(c, n, n, ident.data(), offsets, s.offsets.p, s.sets.p, s.scores.p, header, names, arity,
                           text, len);
}

}  // extern "C"
