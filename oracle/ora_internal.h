/* ora_internal.h -- TEST INFRASTRUCTURE ONLY (see ora.h).
 * Small open-addressing hash containers standing in for the reference's
 * boost::unordered_map<varset,float> (FloatMap, typedefs.h:816),
 * std::unordered_set<varset> (BIC_OLS.cpp:230) and NodeMap.  Lookups and
 * inserts have the same semantics; iteration order is not used. */
#ifndef ULG_ORA_INTERNAL_H
#define ULG_ORA_INTERNAL_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t vs_t;

static inline uint64_t ora_mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}

/* u64 -> u64 map (value holds float bits or an index) */
typedef struct {
    uint64_t *keys;
    uint64_t *vals;
    uint8_t *used;
    size_t cap, size;
} omap;

static inline void omap_init(omap *m, size_t hint) {
    size_t c = 16;
    while (c < hint * 2) c <<= 1;
    m->cap = c; m->size = 0;
    m->keys = (uint64_t *)malloc(c * sizeof(uint64_t));
    m->vals = (uint64_t *)malloc(c * sizeof(uint64_t));
    m->used = (uint8_t *)calloc(c, 1);
}
static inline void omap_free(omap *m) {
    free(m->keys); free(m->vals); free(m->used);
    m->keys = NULL; m->vals = NULL; m->used = NULL; m->cap = m->size = 0;
}
static inline void omap_clear(omap *m) {
    memset(m->used, 0, m->cap); m->size = 0;
}
static inline size_t omap_slot(const omap *m, uint64_t k) {
    size_t i = (size_t)ora_mix64(k) & (m->cap - 1);
    while (m->used[i] && m->keys[i] != k) i = (i + 1) & (m->cap - 1);
    return i;
}
static inline int omap_get(const omap *m, uint64_t k, uint64_t *v) {
    size_t i = omap_slot(m, k);
    if (!m->used[i]) return 0;
    if (v) *v = m->vals[i];
    return 1;
}
static void omap_grow(omap *m);
static inline void omap_put(omap *m, uint64_t k, uint64_t v) {
    if ((m->size + 1) * 2 > m->cap) omap_grow(m);
    size_t i = omap_slot(m, k);
    if (!m->used[i]) { m->used[i] = 1; m->keys[i] = k; m->size++; }
    m->vals[i] = v;
}
static void omap_grow(omap *m) {
    omap n;
    size_t i;
    omap_init(&n, m->cap);
    for (i = 0; i < m->cap; i++)
        if (m->used[i]) omap_put(&n, m->keys[i], m->vals[i]);
    omap_free(m);
    *m = n;
}

static inline uint64_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint64_t v) { uint32_t u = (uint32_t)v; float f; memcpy(&f, &u, 4); return f; }

static inline int popc64(uint64_t x) { return __builtin_popcountll(x); }

#endif
