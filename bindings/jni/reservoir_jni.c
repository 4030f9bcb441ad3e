/*
 * reservoir_jni.c -- JNI shim of lgbt.princess.reservoir.gpu.Jni
 * (bindings/scala/core/lgbt/princess/reservoir/gpu/JniSampler.scala)
 * for the reference's CI JDKs 8/11/15 (build.sbt:37-42), where Panama FFM does not exist.
 *
 * Every native method is a few lines over bindings/jvm/rsv_jvm.{h,c} -- the JVM-side session logic
 * (isOpen tracked on the JVM side, keys staged into the engine's pinned buffers, single-use result()
 * destroys the handle) that tests/cpp/test_ffm_sequence.cpp runs on the GPU without a JDK.
 * A session is a malloc'd rsv_jvm passed to the JVM as a jlong.
 *
 * Build (needs a JDK; none exists in this image):  make -C bindings/jni JAVA_HOME=/path/to/jdk
 *   -> bindings/jni/libreservoir_jni.so, linked against reservoir_amd/libreservoir_hip.so
 */
#include <jni.h>
#include <stdlib.h>

#include "../jvm/rsv_jvm.h"

#define JNI_FN(name) Java_lgbt_princess_reservoir_gpu_Jni_00024_##name /* Scala `object Jni` */

static void throw_status(JNIEnv* env, rsv_status st) {
    jclass cls = (*env)->FindClass(env, rsv_jvm_exception_class(st));
    if (cls) (*env)->ThrowNew(env, cls, rsv_jvm_last_error());
}

static rsv_jvm* session(jlong s) { return (rsv_jvm*)(intptr_t)s; }

/* Sampler.apply / Sampler.distinct (Sampler.scala:128-136, :171-180); returns the session */
JNIEXPORT jlong JNICALL JNI_FN(create)(JNIEnv* env, jobject self, jint kind, jint k, jint key_width, jboolean reusable,
                                        jint engine, jint hash_kind, jint order, jlong seed, jlong stream_id,
                                        jint device) {
    (void)self;
    rsv_config cfg;
    rsv_config_init(&cfg);
    cfg.kind = kind;
    cfg.max_sample_size = k;
    cfg.key_width = key_width;
    cfg.reusable = reusable ? 1 : 0;
    cfg.engine = engine;
    cfg.hash_kind = hash_kind;
    cfg.distinct_order = order;
    cfg.seed = (uint64_t)seed;
    cfg.stream_id = (uint64_t)stream_id;
    cfg.device = device;
    rsv_jvm* s = (rsv_jvm*)malloc(sizeof(rsv_jvm));
    if (!s) {
        throw_status(env, RSV_E_OUT_OF_MEMORY);
        return 0;
    }
    rsv_status st = rsv_jvm_create(s, &cfg);
    if (st != RSV_OK) {
        free(s);
        throw_status(env, st);
        return 0;
    }
    return (jlong)(intptr_t)s;
}

/* Sampler.sample (Sampler.scala:37-38), one key: staged, no device call per element */
JNIEXPORT void JNICALL JNI_FN(sampleLong)(JNIEnv* env, jobject self, jlong s, jlong key, jlong hash) {
    (void)self;
    rsv_status st = rsv_jvm_sample(session(s), &key, hash);
    if (st != RSV_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL JNI_FN(sampleInt)(JNIEnv* env, jobject self, jlong s, jint key, jlong hash) {
    (void)self;
    rsv_status st = rsv_jvm_sample(session(s), &key, hash);
    if (st != RSV_OK) throw_status(env, st);
}

/* Sampler.sampleAll (Sampler.scala:49-50) over the first n keys of a primitive array (+ hashes when
 * the sampler takes precomputed hashes, else null).  Copied with Get<Type>ArrayRegion straight into
 * the engine's pinned staging: no array stays pinned (and GC blocked) while a full staging buffer's
 * commit may wait for the GPU (rsv_jvm_stage_span). */
#define SAMPLE_ARRAY(NAME, JARR, GET)                                                                   \
    JNIEXPORT void JNICALL JNI_FN(NAME)(JNIEnv * env, jobject self, jlong s, JARR keys, jlongArray hashes, \
                                        jint n) {                                                     \
        (void)self;                                                                                   \
        jint done = 0;                                                                                \
        while (done < n) {                                                                            \
            void* kb = NULL;                                                                          \
            int64_t* hb = NULL;                                                                       \
            int64_t room = 0;                                                                         \
            rsv_status st = rsv_jvm_stage_span(session(s), &kb, &hb, &room);                          \
            if (st != RSV_OK) {                                                                       \
                throw_status(env, st);                                                                \
                return;                                                                               \
            }                                                                                         \
            const jint c = room < (int64_t)(n - done) ? (jint)room : n - done;                        \
            (*env)->GET(env, keys, done, c, kb);                                                      \
            if (hb && hashes) (*env)->GetLongArrayRegion(env, hashes, done, c, (jlong*)hb);           \
            if ((*env)->ExceptionCheck(env)) return; /* bounds: nothing committed for this span */    \
            if (hb && !hashes) {                                                                      \
                throw_status(env, RSV_E_NULL_POINTER);                                                \
                return;                                                                               \
            }                                                                                         \
            rsv_jvm_stage_advance(session(s), c);                                                     \
            done += c;                                                                                \
        }                                                                                             \
    }

SAMPLE_ARRAY(sampleLongs, jlongArray, GetLongArrayRegion)
SAMPLE_ARRAY(sampleInts, jintArray, GetIntArrayRegion)

/* Sampler.result (Sampler.scala:59-60): fills `out` (length >= k) and returns the sample size;
 * a single-use sampler's handle is destroyed here (never touched again).  The engine writes into a
 * native buffer (its result may wait on the GPU or run the ordered replay: no pinned array), then
 * Set<Type>ArrayRegion copies it out. */
#define RESULT_ARRAY(NAME, JARR, JT, SET)                                                 \
    JNIEXPORT jint JNICALL JNI_FN(NAME)(JNIEnv * env, jobject self, jlong s, JARR out) {  \
        (void)self;                                                                      \
        const jsize len = (*env)->GetArrayLength(env, out);                              \
        JT* buf = (JT*)malloc((size_t)(len > 0 ? len : 1) * sizeof(JT));                 \
        if (!buf) {                                                                      \
            throw_status(env, RSV_E_OUT_OF_MEMORY);                                      \
            return 0;                                                                    \
        }                                                                                \
        int64_t n = 0;                                                                   \
        rsv_status st = rsv_jvm_result(session(s), buf, len, &n);                        \
        if (st == RSV_OK) (*env)->SET(env, out, 0, (jsize)n, buf);                       \
        free(buf);                                                                       \
        if (st != RSV_OK) throw_status(env, st);                                         \
        return (jint)n;                                                                  \
    }

RESULT_ARRAY(resultLongs, jlongArray, jlong, SetLongArrayRegion)
RESULT_ARRAY(resultInts, jintArray, jint, SetIntArrayRegion)

/* Sampler.isOpen (Sampler.scala:67): no downcall into the engine */
JNIEXPORT jboolean JNICALL JNI_FN(isOpen)(JNIEnv* env, jobject self, jlong s) {
    (void)env;
    (void)self;
    return rsv_jvm_is_open(session(s)) ? JNI_TRUE : JNI_FALSE;
}

/* release (JniSession.release, exactly once: a single-use result() or the phantom-reference cleaner):
 * destroys a live handle, frees the session */
JNIEXPORT void JNICALL JNI_FN(destroy)(JNIEnv* env, jobject self, jlong s) {
    (void)env;
    (void)self;
    if (!s) return;
    rsv_jvm_destroy(session(s));
    free(session(s));
}

/* Zero-copy staging for a JVM producer that writes keys itself (e.g. a columnar source): a direct
 * ByteBuffer over the free tail of the engine's pinned staging buffer; stageCommit(n) hands the
 * first n keys written there to the engine.  Both first flush the keys staged by sample(). */
JNIEXPORT jobject JNICALL JNI_FN(stageAcquire)(JNIEnv* env, jobject self, jlong s) {
    (void)self;
    void* keys = NULL;
    int64_t cap = 0;
    rsv_status st = rsv_jvm_stage_acquire(session(s), &keys, &cap);
    if (st != RSV_OK) {
        throw_status(env, st);
        return NULL;
    }
    return (*env)->NewDirectByteBuffer(env, keys, cap * session(s)->key_width);
}

JNIEXPORT void JNICALL JNI_FN(stageCommit)(JNIEnv* env, jobject self, jlong s, jlong n) {
    (void)self;
    rsv_status st = rsv_jvm_stage_commit(session(s), n);
    if (st != RSV_OK) throw_status(env, st);
}

/* Sampler.sampleAll over a known-size IndexedSeq (Sampler.scala:289-312 -> sampleIndexed :261-273):
 * the engine samples indices 0 until n of the sequence and fills `offsets` (length >= k) with the
 * offset of the element each slot now holds, or -1; JniSampler maps exactly those elements and
 * hands their keys back with fillLongs / fillInts (a k-key array in slot order). */
JNIEXPORT void JNICALL JNI_FN(sampleIndexed)(JNIEnv* env, jobject self, jlong s, jlong n, jlongArray offsets) {
    (void)self;
    const jsize len = (*env)->GetArrayLength(env, offsets);
    if (len < session(s)->k) {
        throw_status(env, RSV_E_ILLEGAL_ARGUMENT);
        return;
    }
    int64_t* buf = (int64_t*)malloc((size_t)len * sizeof(int64_t));
    if (!buf) {
        throw_status(env, RSV_E_OUT_OF_MEMORY);
        return;
    }
    rsv_status st = rsv_jvm_sample_indexed(session(s), n, buf);
    if (st == RSV_OK) (*env)->SetLongArrayRegion(env, offsets, 0, session(s)->k, (const jlong*)buf);
    free(buf);
    if (st != RSV_OK) throw_status(env, st);
}

#define FILL_ARRAY(NAME, JARR, JT, GET)                                                  \
    JNIEXPORT void JNICALL JNI_FN(NAME)(JNIEnv * env, jobject self, jlong s, JARR keys) { \
        (void)self;                                                                     \
        const jint k = session(s)->k;                                                   \
        JT* buf = (JT*)malloc((size_t)k * sizeof(JT));                                  \
        if (!buf) {                                                                     \
            throw_status(env, RSV_E_OUT_OF_MEMORY);                                     \
            return;                                                                     \
        }                                                                               \
        (*env)->GET(env, keys, 0, k, buf);                                              \
        rsv_status st = (*env)->ExceptionCheck(env) ? RSV_OK : rsv_jvm_fill_slots(session(s), buf); \
        free(buf);                                                                      \
        if (st != RSV_OK) throw_status(env, st);                                        \
    }

FILL_ARRAY(fillLongs, jlongArray, jlong, GetLongArrayRegion)
FILL_ARRAY(fillInts, jintArray, jint, GetIntArrayRegion)

/* fixed-width byte keys (java.util.UUID: key_width 16) travel as key_width / 8 Longs per key, in
 * key order: sampleWords / resultWords / fillWords are the Long-array forms above with n counting
 * keys, not array elements */
JNIEXPORT void JNICALL JNI_FN(sampleWords)(JNIEnv* env, jobject self, jlong s, jlongArray words, jlongArray hashes,
                                           jint n) {
    (void)self;
    const jint w = session(s)->key_width / 8;
    jint done = 0;
    while (done < n) {
        void* kb = NULL;
        int64_t* hb = NULL;
        int64_t room = 0;
        rsv_status st = rsv_jvm_stage_span(session(s), &kb, &hb, &room);
        if (st != RSV_OK) {
            throw_status(env, st);
            return;
        }
        const jint c = room < (int64_t)(n - done) ? (jint)room : n - done;
        (*env)->GetLongArrayRegion(env, words, done * w, c * w, (jlong*)kb);
        if (hb && hashes) (*env)->GetLongArrayRegion(env, hashes, done, c, (jlong*)hb);
        if ((*env)->ExceptionCheck(env)) return;
        if (hb && !hashes) {
            throw_status(env, RSV_E_NULL_POINTER);
            return;
        }
        rsv_jvm_stage_advance(session(s), c);
        done += c;
    }
}

JNIEXPORT jint JNICALL JNI_FN(resultWords)(JNIEnv* env, jobject self, jlong s, jlongArray out) {
    (void)self;
    const jint w = session(s)->key_width / 8;
    const jsize len = (*env)->GetArrayLength(env, out);
    jlong* buf = (jlong*)malloc((size_t)(len > 0 ? len : 1) * sizeof(jlong));
    if (!buf) {
        throw_status(env, RSV_E_OUT_OF_MEMORY);
        return 0;
    }
    int64_t n = 0;
    rsv_status st = rsv_jvm_result(session(s), buf, len / w, &n);
    if (st == RSV_OK) (*env)->SetLongArrayRegion(env, out, 0, (jsize)(n * w), buf);
    free(buf);
    if (st != RSV_OK) throw_status(env, st);
    return (jint)n;
}

JNIEXPORT void JNICALL JNI_FN(fillWords)(JNIEnv* env, jobject self, jlong s, jlongArray keys) {
    (void)self;
    /* k * key_width / 8 <= Int.MaxValue (rsv_jvm_create refuses larger byte-key samplers) */
    const size_t kw = (size_t)session(s)->k * (size_t)(session(s)->key_width / 8);
    jlong* buf = (jlong*)malloc(kw * sizeof(jlong));
    if (!buf) {
        throw_status(env, RSV_E_OUT_OF_MEMORY);
        return;
    }
    (*env)->GetLongArrayRegion(env, keys, 0, (jsize)kw, buf);
    rsv_status st = (*env)->ExceptionCheck(env) ? RSV_OK : rsv_jvm_fill_slots(session(s), buf);
    free(buf);
    if (st != RSV_OK) throw_status(env, st);
}

/* ObjectSampler (any B): accept the index-only batch; the B values stay in the JVM's slot array */
JNIEXPORT void JNICALL JNI_FN(commitIndexed)(JNIEnv* env, jobject self, jlong s) {
    (void)self;
    rsv_status st = rsv_jvm_commit_indexed(session(s));
    if (st != RSV_OK) throw_status(env, st);
}

/* `map` threw while the keys of an index-only batch were owed: drop the batch (the JVM rethrows) */
JNIEXPORT void JNICALL JNI_FN(abortIndexed)(JNIEnv* env, jobject self, jlong s) {
    (void)self;
    rsv_status st = rsv_jvm_abort_indexed(session(s));
    if (st != RSV_OK) throw_status(env, st);
}
