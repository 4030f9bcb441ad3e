/*
 * reservoir_jni.c -- JNI shim of lgbt.princess.reservoir.gpu.Jni (bindings/scala/.../Jni.scala)
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
 * the sampler takes precomputed hashes, else null): copied straight from the pinned-down array
 * into the engine's staging buffer */
JNIEXPORT void JNICALL JNI_FN(sampleLongs)(JNIEnv* env, jobject self, jlong s, jlongArray keys, jlongArray hashes,
                                            jint n) {
    (void)self;
    jlong* k = (jlong*)(*env)->GetPrimitiveArrayCritical(env, keys, NULL);
    jlong* h = hashes ? (jlong*)(*env)->GetPrimitiveArrayCritical(env, hashes, NULL) : NULL;
    rsv_status st = rsv_jvm_sample_array(session(s), k, (const int64_t*)h, n);
    if (h) (*env)->ReleasePrimitiveArrayCritical(env, hashes, h, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
    if (st != RSV_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL JNI_FN(sampleInts)(JNIEnv* env, jobject self, jlong s, jintArray keys, jlongArray hashes,
                                           jint n) {
    (void)self;
    jint* k = (jint*)(*env)->GetPrimitiveArrayCritical(env, keys, NULL);
    jlong* h = hashes ? (jlong*)(*env)->GetPrimitiveArrayCritical(env, hashes, NULL) : NULL;
    rsv_status st = rsv_jvm_sample_array(session(s), k, (const int64_t*)h, n);
    if (h) (*env)->ReleasePrimitiveArrayCritical(env, hashes, h, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, keys, k, JNI_ABORT);
    if (st != RSV_OK) throw_status(env, st);
}

/* Sampler.result (Sampler.scala:59-60): fills `out` (length >= k) and returns the sample size;
 * a single-use sampler's handle is destroyed here (never touched again) */
JNIEXPORT jint JNICALL JNI_FN(resultLongs)(JNIEnv* env, jobject self, jlong s, jlongArray out) {
    (void)self;
    int64_t n = 0;
    jlong* o = (jlong*)(*env)->GetPrimitiveArrayCritical(env, out, NULL);
    rsv_status st = rsv_jvm_result(session(s), o, (*env)->GetArrayLength(env, out), &n);
    (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
    if (st != RSV_OK) throw_status(env, st);
    return (jint)n;
}

JNIEXPORT jint JNICALL JNI_FN(resultInts)(JNIEnv* env, jobject self, jlong s, jintArray out) {
    (void)self;
    int64_t n = 0;
    jint* o = (jint*)(*env)->GetPrimitiveArrayCritical(env, out, NULL);
    rsv_status st = rsv_jvm_result(session(s), o, (*env)->GetArrayLength(env, out), &n);
    (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
    if (st != RSV_OK) throw_status(env, st);
    return (jint)n;
}

/* Sampler.isOpen (Sampler.scala:67): no downcall into the engine */
JNIEXPORT jboolean JNICALL JNI_FN(isOpen)(JNIEnv* env, jobject self, jlong s) {
    (void)env;
    (void)self;
    return rsv_jvm_is_open(session(s)) ? JNI_TRUE : JNI_FALSE;
}

/* release (the JVM Cleaner, exactly once): destroys a live handle, frees the session */
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
