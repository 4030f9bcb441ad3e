/*
 * rsv_jvm.h -- the JVM side of one GPU-backed Sampler, written in C over the C ABI.
 *
 * This is the per-call logic of the JNI shim (bindings/jni/reservoir_jni.c calls these functions
 * and nothing else) and, statement for statement, of the Panama FFM binding
 * (bindings/scala/ffm/lgbt/princess/reservoir/gpu/ffm/FfmSampler.scala).  It has no JNI types, so the
 * exact call sequence a JVM drives is compiled and run on the GPU without a JDK
 * (tests/cpp/test_ffm_sequence.cpp, tests/test_gpu_ffm.py).
 *
 * Reference (NthPortal/reservoir): S = core/src/main/scala/lgbt/princess/reservoir/Sampler.scala
 *   - isOpen (S:67, SingleUse S:182-194) is tracked HERE: sample() after a single-use result()
 *     throws IllegalStateException (S:186) without a downcall, and the handle is never touched
 *     after the single-use result() destroyed it (isOpen stays callable: SamplerTest.scala:263-267).
 *   - keys are written into the engine's pinned staging buffer (rsv_stage_acquire/commit): one
 *     downcall per ~1 Mi keys, none per element (the akka operator's per-element path,
 *     SampleImpl.scala:27-31).
 */
#ifndef RESERVOIR_RSV_JVM_H
#define RESERVOIR_RSV_JVM_H

#include <stdint.h>

#include "../../include/reservoir_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rsv_jvm {
    rsv_sampler* h;       /* NULL once a single-use result() has destroyed the handle */
    int32_t open;         /* Sampler.isOpen */
    int32_t reusable;     /* MultiResult* (S:353-381, :430-433): result() keeps the handle */
    int32_t k, key_width; /* key_width 4 (Int), 8 (Long) or 16..256 (byte keys: UUID = 16) */
    int32_t precomputed;  /* RSV_HASH_PRECOMPUTED: a caller hash rides beside every key */
    uint8_t* stage;       /* acquired pinned staging (engine-owned): keys */
    int64_t* stage_hash;  /*   and hashes (precomputed only) */
    int64_t cap, filled;  /* acquired capacity / keys written into it so far */
} rsv_jvm;

/* Sampler.apply / Sampler.distinct (S:128-136, :171-180): validation happens in rsv_create */
rsv_status rsv_jvm_create(rsv_jvm* s, const rsv_config* cfg);
/* Sampler.sample (S:37-38): one key (key_width bytes) + its hash when precomputed */
rsv_status rsv_jvm_sample(rsv_jvm* s, const void* key, int64_t hash);
/* Sampler.sampleAll over a primitive array (S:49-50): n keys (+ n hashes when precomputed) */
rsv_status rsv_jvm_sample_array(rsv_jvm* s, const void* keys, const int64_t* hashes, int64_t n);
/* the free tail of the pinned staging (the next buffer once this one is full: that commit may wait
 * for the GPU, so a JNI caller must hold no array pinned here): room for *room keys (+ hashes for
 * RSV_HASH_PRECOMPUTED, else *hashes_out = NULL); rsv_jvm_stage_advance(n) records n keys written */
rsv_status rsv_jvm_stage_span(rsv_jvm* s, void** keys_out, int64_t** hashes_out, int64_t* room);
void rsv_jvm_stage_advance(rsv_jvm* s, int64_t n);
/* Sampler.sampleAll over a known-size IndexedSeq (S:289-312 -> sampleIndexed S:261-273): the n
 * elements seq(0 until n) are sampled by index alone; slot_offsets[k] receives per slot the offset
 * of the element that now holds it, or -1.  The binding maps exactly those elements into
 * keys[slot] (a k-key array, other entries ignored) and passes it to rsv_jvm_fill_slots. */
rsv_status rsv_jvm_sample_indexed(rsv_jvm* s, int64_t n, int64_t* slot_offsets);
rsv_status rsv_jvm_fill_slots(rsv_jvm* s, const void* keys);
/* `map` threw on an element owed after rsv_jvm_sample_indexed: drop that batch (rsv_abort_indexed)
 * so the sampler stays usable; the binding rethrows the exception */
rsv_status rsv_jvm_abort_indexed(rsv_jvm* s);
/* a `Sampler[A, B]` for any other B (ObjectSampler.scala): accept the pending index-only batch
 * without keys -- the binding keeps the B values in its own slot array (rsv_commit_indexed) */
rsv_status rsv_jvm_commit_indexed(rsv_jvm* s);
/* Sampler.result (S:59-60): writes min(count, k) keys; a single-use sampler closes (S:345-350) */
rsv_status rsv_jvm_result(rsv_jvm* s, void* out, int64_t cap, int64_t* out_n);
/* zero-copy form for a producer that writes keys itself (keys-only samplers): the free tail of
 * the engine's staging buffer (the keys staged by rsv_jvm_sample go first), then commit n of them */
rsv_status rsv_jvm_stage_acquire(rsv_jvm* s, void** keys_out, int64_t* capacity);
rsv_status rsv_jvm_stage_commit(rsv_jvm* s, int64_t n);
/* Sampler.isOpen (S:67) */
int32_t rsv_jvm_is_open(const rsv_jvm* s);
/* release the handle if it is still alive (idempotent): a JVM Cleaner / close() */
void rsv_jvm_destroy(rsv_jvm* s);
/* the message of the last failing rsv_jvm_* call on this thread (the engine's rsv_last_error, or
 * this layer's own for the checks it makes without a downcall) */
const char* rsv_jvm_last_error(void);
/* the JVM exception class a status maps to (JNI class name), NULL for RSV_OK */
const char* rsv_jvm_exception_class(rsv_status st);

#ifdef __cplusplus
}
#endif
#endif
