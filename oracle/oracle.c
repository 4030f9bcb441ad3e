/*
 * oracle.c -- CPU restatement of NthPortal/reservoir (TEST INFRASTRUCTURE ONLY; see oracle.h).
 *
 * Every function cites the reference line it restates.  Reference paths are relative to
 * the NthPortal/reservoir tree: core/src/main/scala/lgbt/princess/reservoir/Sampler.scala.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* java.util.Random (JDK 1.0+ spec; scala.util.Random delegates to it, Sampler.scala:199)      */
/* ------------------------------------------------------------------------------------------ */
#define JR_MULT 0x5DEECE66DULL
#define JR_ADD  0xBULL
#define JR_MASK ((1ULL << 48) - 1)

void or_jr_init(or_jrandom* r, int64_t seed) { r->seed = ((uint64_t)seed ^ JR_MULT) & JR_MASK; }

int32_t or_jr_next(or_jrandom* r, int bits) {
    r->seed = (r->seed * JR_MULT + JR_ADD) & JR_MASK;
    return (int32_t)(uint32_t)(r->seed >> (48 - bits)); /* Java (int) narrowing */
}

int32_t or_jr_next_int(or_jrandom* r) { return or_jr_next(r, 32); }

int32_t or_jr_next_int_bound(or_jrandom* r, int32_t bound) {
    /* Random.nextInt(int bound): power-of-two fast path, else rejection on int overflow */
    int32_t rr = or_jr_next(r, 31);
    int32_t m = bound - 1;
    if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)rr) >> 31);
    for (int32_t u = rr;; u = or_jr_next(r, 31)) {
        rr = u % bound;
        if ((int32_t)((uint32_t)u - (uint32_t)rr + (uint32_t)m) >= 0) break; /* wrapping int */
    }
    return rr;
}

int64_t or_jr_next_long(or_jrandom* r) {
    /* ((long)next(32) << 32) + next(32): the second int is sign-extended */
    int64_t hi = or_jr_next(r, 32);
    int64_t lo = or_jr_next(r, 32);
    return (int64_t)(((uint64_t)hi << 32) + (uint64_t)lo);
}

double or_jr_next_double(or_jrandom* r) {
    int64_t a = or_jr_next(r, 26), b = or_jr_next(r, 27);
    return (double)((a << 27) + b) * 0x1.0p-53;
}

/* JVM d2l: NaN -> 0, saturating at the int64 range (JLS 5.1.3) */
static int64_t jvm_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
static int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* ------------------------------------------------------------------------------------------ */
/* scala.util.hashing.byteswap64 (scala-library 2.13.6, package.scala)                        */
/* ------------------------------------------------------------------------------------------ */
int64_t or_byteswap64(int64_t v) {
    uint64_t hc = (uint64_t)v * 0x9e3779b97f4a7c15ULL;
    hc = __builtin_bswap64(hc);
    return (int64_t)(hc * 0x9e3779b97f4a7c15ULL);
}
int64_t or_java_long_hashcode(int64_t v) {
    return (int64_t)(int32_t)(uint32_t)((uint64_t)v ^ ((uint64_t)v >> 32));
}
int64_t or_java_int_hashcode(int32_t v) { return (int64_t)v; }

/* ------------------------------------------------------------------------------------------ */
/* Algorithm L -- RandomElements (Sampler.scala:196-331)                                       */
/* ------------------------------------------------------------------------------------------ */
static void algo_l_update(or_algo_l* s) {
    /* updateNextSampleCount, Sampler.scala:228-236 (java.lang.Math.log/exp/floor) */
    double W = s->W * exp(log(or_jr_next_double(&s->rand)) / (double)s->k);
    s->W = W;
    double skip = floor(log(or_jr_next_double(&s->rand)) / log(1.0 - W));
    s->next_sample_count = wadd(wadd(s->next_sample_count, jvm_d2l(skip)), 1);
}

int or_algo_l_init(or_algo_l* s, int32_t k, int64_t seed, int64_t event_cap) {
    memset(s, 0, sizeof(*s));
    if (k <= 0) return -1;
    s->k = k;
    s->samples = (int64_t*)calloc((size_t)k, sizeof(int64_t));
    if (!s->samples) return -2;
    if (event_cap > 0) {
        s->ev_pos = (int64_t*)malloc((size_t)event_cap * sizeof(int64_t));
        s->ev_slot = (int32_t*)malloc((size_t)event_cap * sizeof(int32_t));
        s->ev_cap = event_cap;
    }
    /* SamplerTest.useConsistentRandom: rand = Random(seed), W = 1.0, nextSampleCount = k */
    or_jr_init(&s->rand, seed);
    s->W = 1.0;
    s->next_sample_count = k;
    algo_l_update(s);
    return 0;
}

void or_algo_l_free(or_algo_l* s) {
    free(s->samples);
    free(s->ev_pos);
    free(s->ev_slot);
    memset(s, 0, sizeof(*s));
}

static void algo_l_evict(or_algo_l* s, int64_t elem, int64_t pos1) {
    /* sampleWithEviction, Sampler.scala:243-246 */
    int32_t slot = or_jr_next_int_bound(&s->rand, s->k);
    s->samples[slot] = elem;
    if (s->ev_n < s->ev_cap) {
        s->ev_pos[s->ev_n] = pos1;
        s->ev_slot[s->ev_n] = slot;
    }
    s->ev_n++;
    algo_l_update(s);
}

void or_algo_l_sample(or_algo_l* s, int64_t elem) {
    /* sampleImpl, Sampler.scala:248-259 */
    int64_t c = s->count + 1;
    s->count = c;
    if (c <= s->k) s->samples[c - 1] = elem;
    else if (c >= s->next_sample_count) algo_l_evict(s, elem, c);
}

void or_algo_l_sample_all_indexed(or_algo_l* s, const int64_t* elems, int64_t n) {
    /* sampleAllImpl (Sampler.scala:289-312) with the IndexedSeq branch -> sampleIndexed (:261-273).
     * Arrays are Int-indexed in the reference; callers keep n < 2^31. */
    if (n <= 0) return;
    int64_t start_count = s->count, i = 0;
    if (start_count < s->k) {
        int64_t c = start_count;
        while (c < s->k && i < n) { s->samples[c] = elems[i]; c++; i++; }
    }
    int32_t start = (int32_t)i, len = (int32_t)(n - i);
    int64_t cnt = start_count + i;
    while (len > 0) {
        int64_t nsc = s->next_sample_count;
        int64_t off = nsc - cnt;
        if (!((int64_t)len >= off)) break;
        if (off <= 0) break; /* only after nextDouble()==0.0 (p = 2^-53): the JVM would throw */
        int32_t off_i = (int32_t)off; /* .toInt */
        int32_t next_start = start + off_i;
        algo_l_evict(s, elems[next_start - 1], cnt + off_i);
        start = next_start;
        len -= off_i;
        cnt = nsc;
    }
    s->count = start_count + n;
}

/* The same sampleIndexed walk over the virtual sequence seq(i) = base_value + i (e.g. a Range,
 * SamplerTest.scala:117-142 feeds 1 to 3000): no element array, so a 1e9-element stream costs only
 * its ~k ln(n/k) evictions.  Element i is read exactly where or_algo_l_sample_all_indexed reads
 * elems[i]. */
void or_algo_l_sample_all_iota(or_algo_l* s, int64_t base_value, int64_t n) {
    if (n <= 0) return;
    int64_t start_count = s->count, i = 0;
    if (start_count < s->k) {
        int64_t c = start_count;
        while (c < s->k && i < n) { s->samples[c] = base_value + i; c++; i++; }
    }
    int64_t start = i, len = n - i; /* 64-bit: a Range is not limited to Int indices here */
    int64_t cnt = start_count + i;
    while (len > 0) {
        int64_t nsc = s->next_sample_count;
        int64_t off = nsc - cnt;
        if (!(len >= off)) break;
        if (off <= 0) break;
        int64_t next_start = start + off;
        algo_l_evict(s, base_value + next_start - 1, cnt + off);
        start = next_start;
        len -= off;
        cnt = nsc;
    }
    s->count = start_count + n;
}

int64_t or_algo_l_result(const or_algo_l* s, int64_t* out) {
    /* resultImpl, Sampler.scala:318-331: the array is min(count, k) long in every growth state */
    int64_t m = s->count < s->k ? s->count : s->k;
    if (out) memcpy(out, s->samples, (size_t)m * sizeof(int64_t));
    return m;
}

/* ------------------------------------------------------------------------------------------ */
/* RandomValues -- distinct bottom-k (Sampler.scala:383-412)                                   */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int64_t elem, h; } pq_ent;

/* scala.collection.mutable.HashSet[Long] stand-in: open addressing (iteration order is not
 * observable through the oracle's sorted result). */
typedef struct { int64_t* keys; uint8_t* used; uint64_t cap, n; } i64set;

static uint64_t set_slot(uint64_t cap, int64_t k) {
    return ((uint64_t)k * 0x9E3779B97F4A7C15ULL) >> 7 & (cap - 1);
}
static int set_contains(const i64set* s, int64_t k) {
    for (uint64_t p = set_slot(s->cap, k);; p = (p + 1) & (s->cap - 1)) {
        if (!s->used[p]) return 0;
        if (s->used[p] == 1 && s->keys[p] == k) return 1;
    }
}
static void set_add(i64set* s, int64_t k) {
    uint64_t p = set_slot(s->cap, k);
    while (s->used[p] == 1) {
        if (s->keys[p] == k) return;
        p = (p + 1) & (s->cap - 1);
    }
    s->used[p] = 1; s->keys[p] = k; s->n++;
}
static void set_remove(i64set* s, int64_t k) {
    /* backward-shift deletion for linear probing */
    uint64_t p = set_slot(s->cap, k);
    for (;; p = (p + 1) & (s->cap - 1)) {
        if (!s->used[p]) return;
        if (s->keys[p] == k) break;
    }
    s->used[p] = 0; s->n--;
    uint64_t q = p;
    for (;;) {
        q = (q + 1) & (s->cap - 1);
        if (!s->used[q]) return;
        uint64_t home = set_slot(s->cap, s->keys[q]);
        /* move q back to p if home is cyclically outside (p, q] */
        int move = (p <= q) ? (home <= p || home > q) : (home <= p && home > q);
        if (move) {
            s->keys[p] = s->keys[q]; s->used[p] = 1; s->used[q] = 0; p = q;
        }
    }
}

struct or_distinct {
    int32_t k;
    int     hash_kind;
    int64_t r0, r1;
    pq_ent* heap;   /* 1-indexed binary max-heap, like scala mutable.PriorityQueue (resarr) */
    int64_t size;   /* number of heap entries */
    i64set  set;
    int64_t max_hash;
};

int64_t or_distinct_scramble(int64_t r0, int64_t r1, int64_t hashed) {
    /* Sampler.scala:396 */
    return or_byteswap64(r1 ^ or_byteswap64(r0 ^ hashed));
}

static int64_t distinct_hash(const or_distinct* d, int64_t elem) {
    switch (d->hash_kind) {
    case OR_HASH_JAVA_LONG: return or_java_long_hashcode(elem);
    case OR_HASH_JAVA_INT:  return or_java_int_hashcode((int32_t)elem);
    default:                return elem;
    }
}

or_distinct* or_distinct_new(int32_t k, int64_t seed, int hash_kind) {
    if (k <= 0) return NULL;
    or_distinct* d = (or_distinct*)calloc(1, sizeof(*d));
    d->k = k;
    d->hash_kind = hash_kind;
    or_jrandom r;
    or_jr_init(&r, seed);
    d->r0 = or_jr_next_long(&r); /* Sampler.scala:385-388 */
    d->r1 = or_jr_next_long(&r);
    d->heap = (pq_ent*)malloc(((size_t)k + 2) * sizeof(pq_ent));
    uint64_t cap = 16;
    while (cap < 2 * (uint64_t)k + 2) cap <<= 1;
    d->set.cap = cap;
    d->set.keys = (int64_t*)calloc(cap, sizeof(int64_t));
    d->set.used = (uint8_t*)calloc(cap, 1);
    d->max_hash = INT64_MIN; /* Sampler.scala:392 */
    return d;
}

void or_distinct_free(or_distinct* d) {
    if (!d) return;
    free(d->heap); free(d->set.keys); free(d->set.used); free(d);
}

/* scala 2.13 mutable.PriorityQueue.addOne + fixUp (1-indexed; ord.lt on the hash only) */
static void pq_add(or_distinct* d, pq_ent e) {
    int64_t m = ++d->size;
    d->heap[m] = e;
    while (m > 1 && d->heap[m / 2].h < d->heap[m].h) {
        pq_ent t = d->heap[m]; d->heap[m] = d->heap[m / 2]; d->heap[m / 2] = t;
        m /= 2;
    }
}
/* scala 2.13 mutable.PriorityQueue.dequeue + fixDown */
static pq_ent pq_dequeue(or_distinct* d) {
    pq_ent res = d->heap[1];
    d->heap[1] = d->heap[d->size];
    d->size--;
    int64_t n = d->size, k = 1;
    while (n >= 2 * k) {
        int64_t j = 2 * k;
        if (j < n && d->heap[j].h < d->heap[j + 1].h) j++;
        if (d->heap[k].h >= d->heap[j].h) break;
        pq_ent t = d->heap[k]; d->heap[k] = d->heap[j]; d->heap[j] = t;
        k = j;
    }
    return res;
}

void or_distinct_sample(or_distinct* d, int64_t elem) {
    /* RandomValues.sample, Sampler.scala:394-409 */
    int64_t h = or_distinct_scramble(d->r0, d->r1, distinct_hash(d, elem));
    if (d->size < d->k) {
        if (!set_contains(&d->set, elem)) {
            pq_ent e = {elem, h};
            pq_add(d, e);
            set_add(&d->set, elem);
            if (h > d->max_hash) d->max_hash = h;
        }
    } else if (h < d->max_hash && !set_contains(&d->set, elem)) {
        set_remove(&d->set, pq_dequeue(d).elem);
        pq_ent e = {elem, h};
        pq_add(d, e);
        set_add(&d->set, elem);
        d->max_hash = d->heap[1].h;
    }
}

void or_distinct_sample_array(or_distinct* d, const int64_t* elems, int64_t n) {
    for (int64_t i = 0; i < n; i++) or_distinct_sample(d, elems[i]); /* Sampler.scala:50 */
}

static int cmp_ent(const void* a, const void* b) {
    const pq_ent* x = (const pq_ent*)a; const pq_ent* y = (const pq_ent*)b;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    if (x->elem != y->elem) return x->elem < y->elem ? -1 : 1;
    return 0;
}

int64_t or_distinct_result(const or_distinct* d, int64_t* out_keys, int64_t* out_hash) {
    /* Sampler.scala:411 returns the HashSet's order (unspecified); the oracle sorts */
    pq_ent* tmp = (pq_ent*)malloc(((size_t)d->size + 1) * sizeof(pq_ent));
    memcpy(tmp, d->heap + 1, (size_t)d->size * sizeof(pq_ent));
    qsort(tmp, (size_t)d->size, sizeof(pq_ent), cmp_ent);
    for (int64_t i = 0; i < d->size; i++) {
        if (out_keys) out_keys[i] = tmp[i].elem;
        if (out_hash) out_hash[i] = tmp[i].h;
    }
    free(tmp);
    return d->size;
}
int64_t or_distinct_r0(const or_distinct* d) { return d->r0; }
int64_t or_distinct_r1(const or_distinct* d) { return d->r1; }

/* ------------------------------------------------------------------------------------------ */
/* RandomValues over fixed-width byte keys (Sampler.scala:383-412 with B = UUID / a case class) */
/* ------------------------------------------------------------------------------------------ */
/* java.util.UUID.hashCode (JDK): long hilo = mostSigBits ^ leastSigBits;
 * return ((int)(hilo >> 32)) ^ (int) hilo;  -- widened by .toLong (Sampler.scala:75) */
int64_t or_uuid_hashcode(uint64_t msb, uint64_t lsb) {
    uint64_t hilo = msb ^ lsb;
    return (int64_t)(int32_t)((uint32_t)(hilo >> 32) ^ (uint32_t)hilo);
}

/* The element set of B: open addressing over member ids with tombstones (FNV-1a of the key
 * words picks the home slot; equality compares every word), rebuilt when half full. */
typedef struct { int64_t* ids; uint64_t cap, used; } rowset; /* ids: -1 free, -2 tombstone */

struct or_distinct_rows {
    int32_t  k, words, uuid;
    int64_t  r0, r1;
    pq_ent*  heap;     /* 1-indexed max-heap of (member id, h), scala PriorityQueue order */
    int64_t  size;
    uint64_t* store;   /* member id -> key words; ids recycled through `free_ids` */
    int64_t* free_ids;
    int64_t  n_free, n_ids, cap_ids;
    rowset   set;
    int64_t  max_hash;
};

static uint64_t row_fnv(const uint64_t* r, int32_t words) {
    uint64_t x = 0xcbf29ce484222325ULL;
    for (int32_t w = 0; w < words; w++)
        for (int b = 0; b < 8; b++) { x ^= (r[w] >> (8 * b)) & 0xFF; x *= 0x100000001b3ULL; }
    return x;
}
static const uint64_t* drow(const or_distinct_rows* d, int64_t id) { return d->store + (size_t)id * d->words; }
static int rows_equal(const uint64_t* a, const uint64_t* b, int32_t words) {
    return memcmp(a, b, (size_t)words * 8) == 0;
}
static void rowset_init(rowset* s, uint64_t cap) {
    s->cap = cap; s->used = 0;
    s->ids = (int64_t*)malloc(cap * sizeof(int64_t));
    for (uint64_t i = 0; i < cap; i++) s->ids[i] = -1;
}
static void rowset_put(or_distinct_rows* d, int64_t id) {
    uint64_t p = row_fnv(drow(d, id), d->words) & (d->set.cap - 1);
    while (d->set.ids[p] >= 0) p = (p + 1) & (d->set.cap - 1);
    d->set.ids[p] = id; d->set.used++;
}
static void rowset_rebuild(or_distinct_rows* d) {  /* drops tombstones */
    free(d->set.ids);
    uint64_t cap = 16;
    while (cap < 4 * (uint64_t)(d->size + 2)) cap <<= 1;
    rowset_init(&d->set, cap);
    for (int64_t i = 1; i <= d->size; i++) rowset_put(d, d->heap[i].elem);
}
static int rowset_contains(const or_distinct_rows* d, const uint64_t* r) {
    for (uint64_t p = row_fnv(r, d->words) & (d->set.cap - 1);; p = (p + 1) & (d->set.cap - 1)) {
        int64_t id = d->set.ids[p];
        if (id == -1) return 0;
        if (id >= 0 && rows_equal(drow(d, id), r, d->words)) return 1;
    }
}
static void rowset_remove(or_distinct_rows* d, int64_t id) {
    for (uint64_t p = row_fnv(drow(d, id), d->words) & (d->set.cap - 1);; p = (p + 1) & (d->set.cap - 1))
        if (d->set.ids[p] == id) { d->set.ids[p] = -2; return; }
}

or_distinct_rows* or_drows_new(int32_t k, int64_t seed, int32_t words, int uuid) {
    if (k <= 0 || words <= 0) return NULL;
    or_distinct_rows* d = (or_distinct_rows*)calloc(1, sizeof(*d));
    d->k = k; d->words = words; d->uuid = uuid;
    or_jrandom r;
    or_jr_init(&r, seed);
    d->r0 = or_jr_next_long(&r); /* Sampler.scala:385-388 */
    d->r1 = or_jr_next_long(&r);
    d->heap = (pq_ent*)malloc(((size_t)k + 2) * sizeof(pq_ent));
    d->cap_ids = 1024;
    d->store = (uint64_t*)malloc((size_t)d->cap_ids * words * 8);
    d->free_ids = (int64_t*)malloc((size_t)d->cap_ids * 8);
    rowset_init(&d->set, 64);
    d->max_hash = INT64_MIN;
    return d;
}

void or_drows_free(or_distinct_rows* d) {
    if (!d) return;
    free(d->heap); free(d->store); free(d->free_ids); free(d->set.ids); free(d);
}

static int64_t drows_new_id(or_distinct_rows* d, const uint64_t* r) {
    int64_t id;
    if (d->n_free) id = d->free_ids[--d->n_free];
    else {
        if (d->n_ids == d->cap_ids) {
            d->cap_ids *= 2;
            d->store = (uint64_t*)realloc(d->store, (size_t)d->cap_ids * d->words * 8);
            d->free_ids = (int64_t*)realloc(d->free_ids, (size_t)d->cap_ids * 8);
        }
        id = d->n_ids++;
    }
    memcpy(d->store + (size_t)id * d->words, r, (size_t)d->words * 8);
    return id;
}

/* the same heap moves as pq_add / pq_dequeue above (scala 2.13 PriorityQueue), on (id, h) */
static void drows_pq_add(or_distinct_rows* d, pq_ent e) {
    int64_t m = ++d->size;
    d->heap[m] = e;
    while (m > 1 && d->heap[m / 2].h < d->heap[m].h) {
        pq_ent t = d->heap[m]; d->heap[m] = d->heap[m / 2]; d->heap[m / 2] = t;
        m /= 2;
    }
}
static pq_ent drows_pq_dequeue(or_distinct_rows* d) {
    pq_ent res = d->heap[1];
    d->heap[1] = d->heap[d->size];
    d->size--;
    int64_t n = d->size, k = 1;
    while (n >= 2 * k) {
        int64_t j = 2 * k;
        if (j < n && d->heap[j].h < d->heap[j + 1].h) j++;
        if (d->heap[k].h >= d->heap[j].h) break;
        pq_ent t = d->heap[k]; d->heap[k] = d->heap[j]; d->heap[j] = t;
        k = j;
    }
    return res;
}

void or_drows_sample(or_distinct_rows* d, const uint64_t* row, int64_t hash) {
    /* RandomValues.sample, Sampler.scala:394-409 */
    if (d->uuid) hash = or_uuid_hashcode(row[0], row[1]);
    int64_t h = or_distinct_scramble(d->r0, d->r1, hash);
    if (d->size < d->k) {
        if (!rowset_contains(d, row)) {
            if (4 * (d->set.used + 1) > 2 * d->set.cap) rowset_rebuild(d); /* before the new member */
            pq_ent e = {drows_new_id(d, row), h};
            drows_pq_add(d, e);
            rowset_put(d, e.elem);
            if (h > d->max_hash) d->max_hash = h;
        }
    } else if (h < d->max_hash && !rowset_contains(d, row)) {
        pq_ent old = drows_pq_dequeue(d);        /* elements -= samples.dequeue()._1 */
        rowset_remove(d, old.elem);
        d->free_ids[d->n_free++] = old.elem;
        if (4 * (d->set.used + 1) > 2 * d->set.cap) rowset_rebuild(d);
        pq_ent e = {drows_new_id(d, row), h};    /* samples += ((elem, elemHash)) */
        drows_pq_add(d, e);
        rowset_put(d, e.elem);                   /* elements += elem */
        d->max_hash = d->heap[1].h;
    }
}

void or_drows_sample_array(or_distinct_rows* d, const uint64_t* rows, const int64_t* hashes, int64_t n) {
    for (int64_t i = 0; i < n; i++) or_drows_sample(d, rows + (size_t)i * d->words, hashes ? hashes[i] : 0);
}

static const or_distinct_rows* g_cmp_rows; /* qsort context (the oracle is single-threaded here) */
static int cmp_row_ent(const void* a, const void* b) {
    const pq_ent* x = (const pq_ent*)a; const pq_ent* y = (const pq_ent*)b;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    const uint64_t* p = drow(g_cmp_rows, x->elem); const uint64_t* q = drow(g_cmp_rows, y->elem);
    for (int32_t w = 0; w < g_cmp_rows->words; w++)
        if (p[w] != q[w]) return p[w] < q[w] ? -1 : 1;
    return 0;
}

int64_t or_drows_result(const or_distinct_rows* d, uint64_t* out_rows, int64_t* out_hash) {
    pq_ent* tmp = (pq_ent*)malloc(((size_t)d->size + 1) * sizeof(pq_ent));
    memcpy(tmp, d->heap + 1, (size_t)d->size * sizeof(pq_ent));
    g_cmp_rows = d;
    qsort(tmp, (size_t)d->size, sizeof(pq_ent), cmp_row_ent);
    for (int64_t i = 0; i < d->size; i++) {
        if (out_rows) memcpy(out_rows + (size_t)i * d->words, drow(d, tmp[i].elem), (size_t)d->words * 8);
        if (out_hash) out_hash[i] = tmp[i].h;
    }
    free(tmp);
    return d->size;
}

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox.h) and draw format R2                 */
/* ------------------------------------------------------------------------------------------ */
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Draw format R2 (DESIGN.md "Draw format"):
 *   key = (lo32(seed), hi32(seed)); ctr = (lo32(g), hi32(g) | domain bit 31, lo32(stream), hi32(stream))
 *   level 0: g = i >> 4, domain 0; the 128 output bits are 8 bit-planes of 16 bits, plane p =
 *            bits [16 (p & 1), 16 (p & 1) + 16) of word p >> 1; b_i = sum_p bit (i & 15) of plane p << p
 *   level 1: g = i >> 1, domain 1; L_i = (w[2(i&1)] << 32) | w[2(i&1)+1]
 *   U_i = (b_i << 56) | (L_i >> 8);  j_i = floor(U_i * (i+1) / 2^64)                        */
static void philox_at(uint64_t seed, uint64_t stream, uint64_t g, uint32_t dom, uint32_t out[4]) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)g, (uint32_t)(g >> 32) | (dom << 31), (uint32_t)stream,
                       (uint32_t)(stream >> 32)};
    or_philox4x32_10(ctr, key, out);
}

uint64_t or_draw_u64(uint64_t seed, uint64_t stream, uint64_t i) {
    uint32_t w0[4], w1[4];
    philox_at(seed, stream, i >> 4, 0, w0);
    uint64_t b = 0;
    for (int p = 0; p < 8; p++) b |= (uint64_t)((w0[p >> 1] >> (16 * (p & 1) + (i & 15))) & 1) << p;
    philox_at(seed, stream, i >> 1, 1, w1);
    uint64_t L = ((uint64_t)w1[2 * (i & 1)] << 32) | w1[2 * (i & 1) + 1];
    return (b << 56) | (L >> 8);
}

uint64_t or_draw_j(uint64_t seed, uint64_t stream, uint64_t i) {
    unsigned __int128 p = (unsigned __int128)or_draw_u64(seed, stream, i) * ((unsigned __int128)i + 1);
    return (uint64_t)(p >> 64);
}

void or_export_draws(uint64_t seed, uint64_t stream, uint64_t i0, int64_t n, uint64_t* out_j) {
    for (int64_t t = 0; t < n; t++) out_j[t] = or_draw_j(seed, stream, i0 + (uint64_t)t);
}

/* Sequential Algorithm R: slot i for i < k, then slot j_i if j_i < k (last writer wins). */
int64_t or_algo_r(uint64_t seed, uint64_t stream, int32_t k, uint64_t i0, const int64_t* keys,
                  int64_t n, int64_t* res, int64_t* res_idx) {
    int64_t repl = 0;
    for (int64_t t = 0; t < n; t++) {
        uint64_t i = i0 + (uint64_t)t;
        uint64_t j = i < (uint64_t)k ? i : or_draw_j(seed, stream, i);
        if (j < (uint64_t)k) {
            res[j] = keys[t];
            if (res_idx) res_idx[j] = (int64_t)i;
            if (i >= (uint64_t)k) repl++;
        }
    }
    return repl;
}

void or_algo_r_replay(int32_t k, uint64_t i0, const uint64_t* j, const int64_t* keys, int64_t n,
                      int64_t* res) {
    for (int64_t t = 0; t < n; t++) {
        uint64_t i = i0 + (uint64_t)t;
        uint64_t jj = i < (uint64_t)k ? i : j[t];
        if (jj < (uint64_t)k) res[jj] = keys[t];
    }
}

void or_algo_r_segmented(uint64_t seed, uint64_t stream_base, int32_t k, const int64_t* keys,
                         const int64_t* offsets, int64_t S, int64_t* out, int64_t* counts) {
    for (int64_t s = 0; s < S; s++) {
        int64_t a = offsets[s], n = offsets[s + 1] - offsets[s];
        int64_t* res = out + s * (int64_t)k;
        memset(res, 0, (size_t)k * sizeof(int64_t));
        or_algo_r(seed, stream_base + (uint64_t)s, k, 0, keys + a, n, res, NULL);
        counts[s] = n < k ? n : k;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Full-size form of or_algo_r (C2: 1e9 indices): the same last writers, computed by the exact   */
/* shortcut of draw format R2.  j_i = floor(U_i (i+1) / 2^64) with U_i >= b_i 2^56, so j_i < k     */
/* implies b_i (i+1) < 256 k: an index failing that test cannot write any slot and its level-1    */
/* Philox is skipped.  Every index passing it is evaluated exactly (or_draw_j's arithmetic), so    */
/* the result equals or_algo_r's res_idx bit for bit.  Slot j's writer is the LARGEST index that  */
/* draws j (Algorithm R's last writer), so disjoint index ranges reduce by max: threads.         */
/* ------------------------------------------------------------------------------------------ */
#include <pthread.h>
#include <unistd.h>

typedef struct {
    uint64_t seed, stream, lo, hi; /* [lo, hi) */
    int32_t k;
    int64_t* win;                  /* k slots, this thread's */
} lw_job;

static uint32_t r2_byte(const uint32_t w[4], unsigned e) {
    uint32_t b = 0;
    for (int p = 0; p < 8; p++) b |= ((w[p >> 1] >> (16 * (p & 1) + e)) & 1u) << p;
    return b;
}

static void lw_eval(const lw_job* jb, uint64_t i, uint32_t b) {
    uint32_t w1[4];
    philox_at(jb->seed, jb->stream, i >> 1, 1, w1);
    uint64_t L = ((uint64_t)w1[2 * (i & 1)] << 32) | w1[2 * (i & 1) + 1];
    uint64_t U = ((uint64_t)b << 56) | (L >> 8);
    uint64_t j = (uint64_t)(((unsigned __int128)U * ((unsigned __int128)i + 1)) >> 64);
    if (j < (uint64_t)jb->k && (int64_t)i > jb->win[j]) jb->win[j] = (int64_t)i;
}

static void* lw_run(void* arg) {
    lw_job* jb = (lw_job*)arg;
    const uint64_t k = (uint64_t)jb->k, lim = 256 * k;
    for (uint64_t i = jb->lo; i < jb->hi && i < k; i++) jb->win[i] = (int64_t)i; /* fill phase */
    uint64_t start = jb->lo > k ? jb->lo : k;
    for (uint64_t g = start >> 4; (g << 4) < jb->hi; g++) {
        uint32_t w0[4];
        philox_at(jb->seed, jb->stream, g, 0, w0);
        uint64_t i0 = g << 4;
        if (i0 + 1 >= lim) { /* sparse: only b_i == 0 passes -- bit e of every plane clear */
            uint32_t x = w0[0] | w0[1] | w0[2] | w0[3];
            uint32_t zero = ~(x | (x >> 16)) & 0xFFFFu;
            while (zero) {
                unsigned e = (unsigned)__builtin_ctz(zero);
                zero &= zero - 1;
                uint64_t i = i0 + e;
                if (i >= start && i < jb->hi) lw_eval(jb, i, 0);
            }
        } else {
            for (unsigned e = 0; e < 16; e++) {
                uint64_t i = i0 + e;
                if (i < start || i >= jb->hi) continue;
                uint32_t b = r2_byte(w0, e);
                if ((unsigned __int128)b * (i + 1) < lim) lw_eval(jb, i, b);
            }
        }
    }
    return NULL;
}

static int or_threads(int nthreads) {
    if (nthreads > 0) return nthreads;
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    if (c < 1) c = 1;
    return c > 16 ? 16 : (int)c; /* the GPU box grants 16 host cores per GPU */
}

void or_algo_r_last_writers(uint64_t seed, uint64_t stream, int32_t k, uint64_t i0, int64_t n,
                            int64_t* win, int nthreads) {
    for (int32_t j = 0; j < k; j++) win[j] = -1;
    if (n <= 0 || k <= 0) return;
    int T = or_threads(nthreads);
    if ((uint64_t)n < (1u << 20)) T = 1;
    lw_job* jobs = (lw_job*)calloc((size_t)T, sizeof(lw_job));
    pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
    uint64_t per = (((uint64_t)n + (uint64_t)T - 1) / (uint64_t)T + 15) & ~(uint64_t)15;
    for (int t = 0; t < T; t++) {
        uint64_t lo = i0 + per * (uint64_t)t, hi = lo + per;
        if (lo > i0 + (uint64_t)n) lo = i0 + (uint64_t)n;
        if (hi > i0 + (uint64_t)n) hi = i0 + (uint64_t)n;
        jobs[t] = (lw_job){seed, stream, lo, hi, k, (int64_t*)malloc((size_t)k * sizeof(int64_t))};
        for (int32_t j = 0; j < k; j++) jobs[t].win[j] = -1;
        pthread_create(&th[t], NULL, lw_run, &jobs[t]);
    }
    for (int t = 0; t < T; t++) {
        pthread_join(th[t], NULL);
        for (int32_t j = 0; j < k; j++)
            if (jobs[t].win[j] > win[j]) win[j] = jobs[t].win[j];
        free(jobs[t].win);
    }
    free(jobs);
    free(th);
}

/* ------------------------------------------------------------------------------------------ */
uint64_t or_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
void or_fill_splitmix(uint64_t base, int64_t n, int64_t* out) {
    for (int64_t i = 0; i < n; i++) out[i] = (int64_t)or_splitmix64(base + (uint64_t)i);
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline leg of bench.py (single thread, like the reference: Sampler.scala:18-19)       */
/* ------------------------------------------------------------------------------------------ */
#include <time.h>
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* per-element sample() (Sampler.scala:248-259): one stream of reps * n_buf elements */
double or_time_algo_l_per_element(int32_t k, int64_t seed, const int64_t* keys, int64_t n_buf,
                                  int64_t reps, int64_t* out) {
    or_algo_l s;
    if (or_algo_l_init(&s, k, seed, 0)) return -1.0;
    double t0 = now_s();
    for (int64_t r = 0; r < reps; r++)
        for (int64_t i = 0; i < n_buf; i++) or_algo_l_sample(&s, keys[i]);
    double t1 = now_s();
    if (out) or_algo_l_result(&s, out);
    or_algo_l_free(&s);
    return t1 - t0;
}

/* sampleAll(IndexedSeq) skip path (Sampler.scala:261-273): touches ~k ln(n/k) elements */
double or_time_algo_l_indexed(int32_t k, int64_t seed, const int64_t* keys, int64_t n, int64_t* out) {
    or_algo_l s;
    if (or_algo_l_init(&s, k, seed, 0)) return -1.0;
    double t0 = now_s();
    or_algo_l_sample_all_indexed(&s, keys, n);
    double t1 = now_s();
    if (out) or_algo_l_result(&s, out);
    or_algo_l_free(&s);
    return t1 - t0;
}

/* C3 leg: S independent samplers (one reference Sampler per stream of L keys, seed = stream
 * index), split over threads (the reference has no threads of its own: one sampler per core).
 * mode 0: per-element sample() (Sampler.scala:248-259); mode 1: sampleAll(IndexedSeq) (:261-273). */
typedef struct {
    int32_t k;
    const int64_t* keys;
    int64_t s0, s1, L;
    int mode;
    int64_t* out;
} seg_job;

static void* seg_run(void* arg) {
    seg_job* jb = (seg_job*)arg;
    for (int64_t s = jb->s0; s < jb->s1; s++) {
        or_algo_l a;
        if (or_algo_l_init(&a, jb->k, s, 0)) return NULL;
        const int64_t* x = jb->keys + s * jb->L;
        if (jb->mode == 0)
            for (int64_t i = 0; i < jb->L; i++) or_algo_l_sample(&a, x[i]);
        else
            or_algo_l_sample_all_indexed(&a, x, jb->L);
        if (jb->out) or_algo_l_result(&a, jb->out + s * (int64_t)jb->k);
        or_algo_l_free(&a);
    }
    return NULL;
}

double or_time_segmented_algo_l(int32_t k, const int64_t* keys, int64_t S, int64_t L, int mode,
                                int nthreads, int64_t* out) {
    int T = or_threads(nthreads);
    if (T > S) T = (int)(S > 0 ? S : 1);
    seg_job* jobs = (seg_job*)calloc((size_t)T, sizeof(seg_job));
    pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
    double t0 = now_s();
    for (int t = 0; t < T; t++) {
        jobs[t] = (seg_job){k, keys, S * t / T, S * (t + 1) / T, L, mode, out};
        pthread_create(&th[t], NULL, seg_run, &jobs[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    double t1 = now_s();
    free(jobs);
    free(th);
    return t1 - t0;
}

/* distinct RandomValues.sample per element (Sampler.scala:394-409) */
double or_time_distinct(int32_t k, int64_t seed, int hash_kind, const int64_t* keys, int64_t n) {
    or_distinct* d = or_distinct_new(k, seed, hash_kind);
    if (!d) return -1.0;
    double t0 = now_s();
    or_distinct_sample_array(d, keys, n);
    double t1 = now_s();
    or_distinct_free(d);
    return t1 - t0;
}
