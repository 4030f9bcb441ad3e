/*
 * oracle.h -- CPU restatement of NthPortal/reservoir's sampling algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (reservoir_amd/, include/,
 * libreservoir_hip.so) may include, link or call this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline ("kind": "port").
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - java.util.Random restatement: pinned by published JDK known answers
 *     (tests/test_oracle_kats.py).
 *   - Philox4x32-10: pinned by the Random123 known-answer vectors.
 *   - Algorithm L (Sampler.scala:196-331) and RandomValues (Sampler.scala:383-412):
 *     pinned by the reference's own test properties (sample == sampleAll over every
 *     collection shape, SamplerTest.scala:117-142; boundary/lifecycle cases) and by the
 *     survey's independently restated vector.  No JVM exists in this
 *     image, so exact JVM outputs are UNCONFIRMED; java.lang.Math.log/exp last-ulp
 *     behaviour and scala-library PriorityQueue/HashSet internals are "parity unpinned".
 */
#ifndef RESERVOIR_ORACLE_H
#define RESERVOIR_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- java.util.Random (JDK spec; used by Sampler.scala:199 via scala.util.Random) ---- */
typedef struct { uint64_t seed; } or_jrandom;
void     or_jr_init(or_jrandom* r, int64_t seed);
int32_t  or_jr_next(or_jrandom* r, int bits);
int32_t  or_jr_next_int(or_jrandom* r);
int32_t  or_jr_next_int_bound(or_jrandom* r, int32_t bound);
int64_t  or_jr_next_long(or_jrandom* r);
double   or_jr_next_double(or_jrandom* r);

/* ---- scala.util.hashing.byteswap64 (scala-library 2.13.6) ---- */
int64_t  or_byteswap64(int64_t v);
/* java.lang.Long.hashCode / Integer.hashCode, widened with .toLong (Sampler.scala:75) */
int64_t  or_java_long_hashcode(int64_t v);
int64_t  or_java_int_hashcode(int32_t v);

/* ---- Algorithm L: RandomElements (Sampler.scala:196-331) ---- */
typedef struct {
    int32_t    k;
    int64_t    count;
    double     W;
    int64_t    next_sample_count;
    or_jrandom rand;
    int64_t*   samples;     /* k slots */
    /* optional event log: (1-based position, slot) of every sampleWithEviction */
    int64_t*   ev_pos;
    int32_t*   ev_slot;
    int64_t    ev_n, ev_cap;
} or_algo_l;

/* Seeds exactly like SamplerTest.useConsistentRandom (SamplerTest.scala:28-36):
 * rand = new Random(seed); W = 1.0; nextSampleCount = k; updateNextSampleCount(). */
int  or_algo_l_init(or_algo_l* s, int32_t k, int64_t seed, int64_t event_cap);
void or_algo_l_free(or_algo_l* s);
/* per-element path, Sampler.scala:248-259 */
void or_algo_l_sample(or_algo_l* s, int64_t elem);
/* sampleAll over an IndexedSeq with knownSize, Sampler.scala:289-312 + sampleIndexed :261-273 */
void or_algo_l_sample_all_indexed(or_algo_l* s, const int64_t* elems, int64_t n);
void or_algo_l_sample_all_iota(or_algo_l* s, int64_t base_value, int64_t n);
/* resultImpl, Sampler.scala:318-331: returns min(count, k) */
int64_t or_algo_l_result(const or_algo_l* s, int64_t* out);

/* ---- RandomValues: distinct bottom-k (Sampler.scala:383-412) ---- */
typedef struct or_distinct or_distinct;
enum { OR_HASH_IDENTITY = 0, OR_HASH_JAVA_LONG = 1, OR_HASH_JAVA_INT = 2 };
/* r0, r1 = Random(seed).nextLong() x2 (SamplerTest.scala:39-42) */
or_distinct* or_distinct_new(int32_t k, int64_t seed, int hash_kind);
void    or_distinct_free(or_distinct* d);
void    or_distinct_sample(or_distinct* d, int64_t elem);
void    or_distinct_sample_array(or_distinct* d, const int64_t* elems, int64_t n);
/* writes the set sorted by (signed scrambled hash, key); returns its size */
int64_t or_distinct_result(const or_distinct* d, int64_t* out_keys, int64_t* out_hash);
int64_t or_distinct_r0(const or_distinct* d);
int64_t or_distinct_r1(const or_distinct* d);
int64_t or_distinct_scramble(int64_t r0, int64_t r1, int64_t hashed);

/* ---- RandomValues over fixed-width byte keys (B with value equality: java.util.UUID, a case
 * class of primitives; `words` 64-bit words per key).  hash(elem) is the caller's per-element
 * value (a JVM `hash: B => Long`), or with uuid != 0 java.util.UUID.hashCode of the key laid out
 * [mostSigBits | leastSigBits].  Equality = equal words (Sampler.scala:398, :403). ---- */
typedef struct or_distinct_rows or_distinct_rows;
or_distinct_rows* or_drows_new(int32_t k, int64_t seed, int32_t words, int uuid);
void    or_drows_free(or_distinct_rows* d);
void    or_drows_sample(or_distinct_rows* d, const uint64_t* row, int64_t hash);
void    or_drows_sample_array(or_distinct_rows* d, const uint64_t* rows, const int64_t* hashes, int64_t n);
/* the set sorted by (signed scrambled hash, key words as unsigned, word 0 first); returns its size */
int64_t or_drows_result(const or_distinct_rows* d, uint64_t* out_rows, int64_t* out_hash);
int64_t or_uuid_hashcode(uint64_t msb, uint64_t lsb);

/* ---- Philox4x32-10 (Random123) and the build's own Algorithm-R draw format "R2" ---- */
void     or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint64_t or_draw_u64(uint64_t seed, uint64_t stream, uint64_t i);          /* U_i */
uint64_t or_draw_j(uint64_t seed, uint64_t stream, uint64_t i);            /* j_i = floor(U_i (i+1) / 2^64) */
void     or_export_draws(uint64_t seed, uint64_t stream, uint64_t i0, int64_t n, uint64_t* out_j);

/* Sequential Algorithm R fed with the R2 draw sequence (the P2 contract).
 * keys[0..n) are the elements at global indices [i0, i0+n); res[k] holds the state
 * (caller initialises it for i0 > 0).  Returns number of replacements. */
int64_t or_algo_r(uint64_t seed, uint64_t stream, int32_t k, uint64_t i0,
                  const int64_t* keys, int64_t n, int64_t* res, int64_t* res_idx);
/* Algorithm R fed with an explicit per-element draw sequence j[0..n) for indices [i0, i0+n). */
void    or_algo_r_replay(int32_t k, uint64_t i0, const uint64_t* j, const int64_t* keys, int64_t n,
                         int64_t* res);
/* Last writer per slot over indices [i0, i0+n) (win[j] = largest index writing slot j, or j
 * itself in the fill phase; -1 = none), identical to or_algo_r's res_idx but evaluated with the
 * exact R2 shortcut (an index with b_i (i+1) >= 256k cannot hit) on nthreads threads (0 = up to
 * 16): the full-size C2 check (1e9 indices) in seconds. */
void    or_algo_r_last_writers(uint64_t seed, uint64_t stream, int32_t k, uint64_t i0, int64_t n,
                               int64_t* win, int nthreads);
/* S independent streams, keys[offsets[s] .. offsets[s+1]), stream id = s (+stream_base). */
void    or_algo_r_segmented(uint64_t seed, uint64_t stream_base, int32_t k, const int64_t* keys,
                            const int64_t* offsets, int64_t S, int64_t* out, int64_t* counts);

/* CPU baseline timings (seconds) for bench.py */
double or_time_algo_l_per_element(int32_t k, int64_t seed, const int64_t* keys, int64_t n_buf,
                                  int64_t reps, int64_t* out);
double or_time_algo_l_indexed(int32_t k, int64_t seed, const int64_t* keys, int64_t n, int64_t* out);
double or_time_distinct(int32_t k, int64_t seed, int hash_kind, const int64_t* keys, int64_t n);
/* S independent Algorithm-L samplers over S x L keys on nthreads threads (0 = up to 16); mode 0 =
 * per-element sample(), 1 = sampleAll(IndexedSeq); out (S x k, optional) receives the reservoirs */
double or_time_segmented_algo_l(int32_t k, const int64_t* keys, int64_t S, int64_t L, int mode,
                                int nthreads, int64_t* out);

/* synthetic inputs */
uint64_t or_splitmix64(uint64_t x);
void     or_fill_splitmix(uint64_t base, int64_t n, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif
