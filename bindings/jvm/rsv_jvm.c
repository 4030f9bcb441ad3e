/* rsv_jvm.c -- see rsv_jvm.h.  Plain C11 over include/reservoir_hip.h; no JNI, no HIP headers. */
#include "rsv_jvm.h"

#include <string.h>

/* rsv_last_error() is thread-local inside the engine; the ISE raised here without a downcall gets
 * its message from this file instead (the JNI shim and the FFM binding read it the same way) */
static _Thread_local const char* g_local_error = 0;

const char* rsv_jvm_last_error(void) { return g_local_error ? g_local_error : rsv_last_error(); }

static rsv_status closed(void) {
    g_local_error = "use of sampler after calling `result()`"; /* Sampler.scala:186 */
    return RSV_E_ILLEGAL_STATE;
}

rsv_status rsv_jvm_create(rsv_jvm* s, const rsv_config* cfg) {
    memset(s, 0, sizeof(*s));
    g_local_error = 0;
    /* byte keys travel as k * key_width / 8 Longs in one JVM array (JniSampler / FfmSampler): more
     * than Int.MaxValue of them cannot be allocated there -- refuse the sampler up front */
    if (cfg->key_width > 8 && (int64_t)cfg->max_sample_size * (cfg->key_width / 8) > 2147483647) {
        g_local_error = "requirement failed: maxSampleSize * key words exceeds the JVM array limit";
        return RSV_E_ILLEGAL_ARGUMENT;
    }
    rsv_status st = rsv_create(cfg, &s->h);
    if (st != RSV_OK) return st;
    s->open = 1;
    s->reusable = cfg->reusable != 0;
    s->k = cfg->max_sample_size;
    s->key_width = cfg->key_width;
    s->precomputed = cfg->kind == RSV_KIND_DISTINCT && cfg->hash_kind == RSV_HASH_PRECOMPUTED;
    return RSV_OK;
}

/* hand the keys written so far to the engine (it flushes a full buffer to the GPU asynchronously)
 * and take the next free staging tail */
static rsv_status next_stage(rsv_jvm* s) {
    if (s->filled > 0) {
        rsv_status st = rsv_stage_commit(s->h, s->filled);
        s->filled = s->cap = 0;
        if (st != RSV_OK) return st;
    }
    void* keys = 0;
    int64_t* hashes = 0;
    rsv_status st = rsv_stage_acquire(s->h, &keys, s->precomputed ? &hashes : 0, &s->cap);
    if (st != RSV_OK) {
        s->cap = 0;
        return st;
    }
    s->stage = (uint8_t*)keys;
    s->stage_hash = hashes;
    return RSV_OK;
}

/* the staged keys must reach the engine before any other call on the handle (the staging pointers
 * are valid only until then) */
static rsv_status commit_pending(rsv_jvm* s) {
    rsv_status st = RSV_OK;
    if (s->filled > 0) st = rsv_stage_commit(s->h, s->filled);
    s->filled = s->cap = 0;
    return st;
}

rsv_status rsv_jvm_sample(rsv_jvm* s, const void* key, int64_t hash) {
    g_local_error = 0;
    if (!s->open) return closed();
    if (s->filled == s->cap) {
        rsv_status st = next_stage(s);
        if (st != RSV_OK) return st;
    }
    memcpy(s->stage + s->filled * s->key_width, key, (size_t)s->key_width);
    if (s->precomputed) s->stage_hash[s->filled] = hash;
    ++s->filled;
    return RSV_OK;
}

rsv_status rsv_jvm_stage_span(rsv_jvm* s, void** keys_out, int64_t** hashes_out, int64_t* room) {
    g_local_error = 0;
    if (!s->open) return closed();
    if (s->filled == s->cap) {
        rsv_status st = next_stage(s);
        if (st != RSV_OK) return st;
    }
    *keys_out = s->stage + s->filled * s->key_width;
    *hashes_out = s->precomputed ? s->stage_hash + s->filled : 0;
    *room = s->cap - s->filled;
    return RSV_OK;
}

void rsv_jvm_stage_advance(rsv_jvm* s, int64_t n) { s->filled += n; }

rsv_status rsv_jvm_sample_array(rsv_jvm* s, const void* keys, const int64_t* hashes, int64_t n) {
    g_local_error = 0;
    if (!s->open) return closed();
    if (n < 0) {
        g_local_error = "negative batch size";
        return RSV_E_ILLEGAL_ARGUMENT;
    }
    if (n > 0 && (!keys || (s->precomputed && !hashes))) {
        g_local_error = "keys/hashes is NULL";
        return RSV_E_NULL_POINTER;
    }
    const uint8_t* src = (const uint8_t*)keys;
    while (n > 0) {  /* the JNI shim runs this same loop with Get<Type>ArrayRegion as the copy */
        void* kb = 0;
        int64_t* hb = 0;
        int64_t room = 0;
        rsv_status st = rsv_jvm_stage_span(s, &kb, &hb, &room);
        if (st != RSV_OK) return st;
        const int64_t c = room < n ? room : n;
        memcpy(kb, src, (size_t)(c * s->key_width));
        if (hb) memcpy(hb, hashes, (size_t)c * 8);
        rsv_jvm_stage_advance(s, c);
        src += c * s->key_width;
        if (hashes) hashes += c;
        n -= c;
    }
    return RSV_OK;
}

rsv_status rsv_jvm_sample_indexed(rsv_jvm* s, int64_t n, int64_t* slot_offsets) {
    g_local_error = 0;
    if (!s->open) return closed();
    rsv_status st = commit_pending(s); /* the staged keys come first in index order */
    if (st == RSV_OK) st = rsv_sample_indexed(s->h, n, slot_offsets);
    return st;
}

rsv_status rsv_jvm_fill_slots(rsv_jvm* s, const void* keys) {
    g_local_error = 0;
    if (!s->open) return closed();
    return rsv_fill_slots(s->h, keys);
}

rsv_status rsv_jvm_abort_indexed(rsv_jvm* s) {
    g_local_error = 0;
    if (!s->open) return closed();
    return rsv_abort_indexed(s->h);
}

rsv_status rsv_jvm_commit_indexed(rsv_jvm* s) {
    g_local_error = 0;
    if (!s->open) return closed();
    return rsv_commit_indexed(s->h);
}

rsv_status rsv_jvm_result(rsv_jvm* s, void* out, int64_t cap, int64_t* out_n) {
    g_local_error = 0;
    if (!s->open) return closed();
    rsv_status st = commit_pending(s);
    if (st == RSV_OK) st = rsv_result(s->h, out, cap, out_n);
    if (st != RSV_OK) return st;
    if (!s->reusable) { /* SingleUse.close (S:188-191): the handle goes now, never touched again */
        rsv_destroy(s->h);
        s->h = 0;
        s->open = 0;
    }
    return RSV_OK;
}

rsv_status rsv_jvm_stage_acquire(rsv_jvm* s, void** keys_out, int64_t* capacity) {
    g_local_error = 0;
    if (!s->open) return closed();
    rsv_status st = commit_pending(s);
    if (st == RSV_OK) st = rsv_stage_acquire(s->h, keys_out, 0, capacity);
    return st;
}

rsv_status rsv_jvm_stage_commit(rsv_jvm* s, int64_t n) {
    g_local_error = 0;
    if (!s->open) return closed();
    return rsv_stage_commit(s->h, n);
}

int32_t rsv_jvm_is_open(const rsv_jvm* s) { return s->open; }

void rsv_jvm_destroy(rsv_jvm* s) {
    if (s->h) rsv_destroy(s->h);
    s->h = 0;
    s->open = 0;
    s->cap = s->filled = 0;
}

const char* rsv_jvm_exception_class(rsv_status st) {
    switch (st) {
    case RSV_OK: return 0;
    case RSV_E_ILLEGAL_ARGUMENT: return "java/lang/IllegalArgumentException"; /* Sampler.scala:80-81 */
    case RSV_E_ILLEGAL_STATE: return "java/lang/IllegalStateException";       /* Sampler.scala:186 */
    case RSV_E_NULL_POINTER: return "java/lang/NullPointerException";         /* Sampler.scala:82, :94 */
    case RSV_E_OUT_OF_MEMORY: return "java/lang/OutOfMemoryError";
    case RSV_E_UNSUPPORTED: return "java/lang/UnsupportedOperationException";
    default: return "java/lang/RuntimeException"; /* device error: fails the akka Future (SampleImpl.scala:43-46) */
    }
}
