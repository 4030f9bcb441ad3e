/*
 * reservoir_hip.h -- C ABI of libreservoir_hip.so, the MI355X (gfx950) reservoir-sampling engine.
 *
 * This is the drop-in boundary behind the lgbt.princess.reservoir API.  Every entry point names
 * the reference interface it replaces (paths relative to NthPortal/reservoir):
 *   S  = core/src/main/scala/lgbt/princess/reservoir/Sampler.scala
 *   SI = akka-stream/src/main/scala/lgbt/princess/reservoir/akkasupport/SampleImpl.scala
 * A Scala binding (Panama FFM downcalls or JNI) is shown in INTEGRATION.md.
 *
 * Conventions
 *   - plain C: no C++ or torch types; opaque handle; every call returns rsv_status.
 *   - keys are primitive fixed-width values (Int -> key_width 4, Long -> key_width 8, or
 *     fixed-width byte keys of 16..256 bytes in steps of 8: java.util.UUID -> 16 bytes laid out
 *     [mostSigBits | leastSigBits] as little-endian Longs, or a case class of primitives) that the
 *     host extracted with the sampler's `map` (S:115-116: map may be called more than k times).
 *     Byte keys must have value equality (B.equals = equal bytes): a distinct sampler dedups by
 *     the bytes, as the reference's `elements.contains` (S:398, S:403) does for such a B.  An
 *     Array[Byte] (reference equality in a Scala Set) must stay on the JVM sampler.
 *   - "device" pointers are HIP device pointers on the handle's device; "host" pointers are
 *     ordinary (pageable or pinned) memory.  The caller owns every buffer it passes in.
 *   - one handle is single-threaded (S:18-19); distinct handles are independent.
 *   - errors: rsv_last_error() returns a thread-local message for the last failing call.
 */
#ifndef RESERVOIR_HIP_H
#define RESERVOIR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSV_ABI_VERSION 1

/* Status codes; a JVM binding maps them 1:1 onto the reference's exceptions. */
typedef enum rsv_status {
    RSV_OK = 0,
    RSV_E_ILLEGAL_ARGUMENT = 1, /* IllegalArgumentException: k <= 0 or k > Int.MaxValue-2 (S:80-81) */
    RSV_E_ILLEGAL_STATE = 2,    /* IllegalStateException "use of sampler after calling `result()`" (S:186) */
    RSV_E_NULL_POINTER = 3,     /* NullPointerException: a required pointer is NULL (S:82, S:94) */
    RSV_E_DEVICE = 4,           /* HIP runtime / kernel failure -> RuntimeException (fails the akka Future, SI:43-46) */
    RSV_E_OUT_OF_MEMORY = 5,    /* device or pinned allocation failed -> OutOfMemoryError */
    RSV_E_UNSUPPORTED = 6       /* request this build does not implement (message says which): a key_width
                                 * other than 4, 8, 16..256 in steps of 8; a hash kind byte keys lack */
} rsv_status;

typedef enum rsv_kind {
    RSV_KIND_ELEMENTS = 0, /* Sampler.apply   (S:128-136): equal-probability sample, duplicates kept */
    RSV_KIND_DISTINCT = 1  /* Sampler.distinct (S:171-180): bottom-k over the scrambled hash     */
} rsv_kind;

typedef enum rsv_engine {
    /* Algorithm R, data-parallel: element i >= k replaces slot j_i = floor(U_i (i+1) / 2^64) when
     * j_i < k, U_i a counter-based Philox4x32-10 draw of (seed, stream_id, i) (draw
     * format R2).  Bit-identical for any batching and any index-range split over GPUs. */
    RSV_ENGINE_PHILOX_R = 0,
    /* The reference's own Algorithm L (S:224-246) driven by java.util.Random(seed), exactly as
     * SamplerTest.useConsistentRandom seeds it; the eviction events are replayed on the GPU.
     * Bit-identical to the reference Sampler for the same seed. */
    RSV_ENGINE_JAVA_L = 1
} rsv_engine;

typedef enum rsv_hash_kind {
    RSV_HASH_DEFAULT = 0,     /* B#hashCode().toLong (S:75): JAVA_INT for key_width 4, JAVA_LONG for 8,
                               * java.util.UUID.hashCode for 16 ((int)(hilo >>> 32) ^ (int)hilo, hilo =
                               * msb ^ lsb); other byte widths take PRECOMPUTED */
    RSV_HASH_IDENTITY = 1,    /* hash = key as a signed Long (a bijection: bit-exact distinct sets) */
    RSV_HASH_JAVA_LONG = 2,   /* java.lang.Long.hashCode: (int)(v ^ v>>>32), sign-extended */
    RSV_HASH_JAVA_INT = 3,    /* java.lang.Integer.hashCode: v, sign-extended */
    RSV_HASH_PRECOMPUTED = 4  /* caller passes int64 hashes beside the keys (arbitrary JVM `hash`) */
} rsv_hash_kind;

/* How a DISTINCT sampler resolves elements whose scrambled hashes tie.  The reference keeps the
 * elements of its max-heap (S:389-409): with an injective hash that is the bottom-k of the hashes,
 * independent of arrival order; with a colliding hash (Long#hashCode folds to 32 bits) the members of
 * the boundary hash bucket depend on arrival order and on PriorityQueue tie-breaking. */
typedef enum rsv_distinct_order {
    /* ORDERED for RSV_HASH_JAVA_LONG / PRECOMPUTED (may collide), SET for IDENTITY / JAVA_INT */
    RSV_DISTINCT_AUTO = 0,
    /* bottom-k by (hash, key): order-independent and mergeable across GPUs; equal to the
     * reference's set whenever no distinct elements share the final maximum hash */
    RSV_DISTINCT_SET = 1,
    /* the reference's sequential semantics for any hash: the GPU filters each chunk of the batch
     * against the current maximum (a superset of what the reference inserts), the host replays
     * the survivors in arrival order through an exact RandomValues replica (heap + hash set) */
    RSV_DISTINCT_ORDERED = 2
} rsv_distinct_order;

typedef enum rsv_mem { RSV_MEM_HOST = 0, RSV_MEM_DEVICE = 1 } rsv_mem;

typedef struct rsv_config {
    uint32_t struct_size;     /* = sizeof(rsv_config) */
    int32_t  kind;            /* rsv_kind */
    int32_t  max_sample_size; /* k: S:130 maxSampleSize / S:173 */
    int32_t  key_width;       /* 4 (Int), 8 (Long), or fixed-width byte keys: a multiple of 8 in 16..256 */
    int32_t  reusable;        /* S:130/S:173 reusable: result() may be called repeatedly (S:353-381, S:430-433) */
    int32_t  pre_allocate;    /* S:130 preAllocate: accepted; device slots are always preallocated */
    int32_t  engine;          /* rsv_engine (ELEMENTS only) */
    int32_t  hash_kind;       /* rsv_hash_kind (DISTINCT only) */
    int32_t  device;          /* HIP device ordinal; -1 = the calling thread's current device */
    int32_t  distinct_order;  /* rsv_distinct_order (DISTINCT only) */
    uint64_t seed;            /* PHILOX_R: Philox key; JAVA_L / DISTINCT: java.util.Random seed (S:199, S:385-388) */
    uint64_t stream_id;       /* PHILOX_R: Philox stream (independent sampler id) */
} rsv_config;

typedef struct rsv_sampler rsv_sampler;

/* Library / error plumbing */
int32_t     rsv_abi_version(void);
const char* rsv_last_error(void);
const char* rsv_status_string(rsv_status s);
rsv_status  rsv_config_init(rsv_config* cfg); /* defaults: ELEMENTS, k=1, key_width 8, PHILOX_R */

/* Construction = Sampler.apply / Sampler.distinct (S:128-136, S:171-180) incl. validation
 * validateSharedParams (S:77-83).  `map`/`hash` nullness is checked on the JVM side. */
rsv_status rsv_create(const rsv_config* cfg, rsv_sampler** out);
void       rsv_destroy(rsv_sampler* s);

/* Sampler.sample(element) (S:37-38; RandomElements.sampleImpl S:248-259; RandomValues.sample
 * S:394-409).  The key is staged in a pinned host batch and flushed to the GPU in bulk; `hash`
 * is read only for RSV_HASH_PRECOMPUTED (may be NULL otherwise). */
rsv_status rsv_sample(rsv_sampler* s, const void* key, const int64_t* hash);

/* Zero-copy pinned batches (the north-star JVM path: keys extracted straight into pinned memory,
 * e.g. a Panama MemorySegment over the returned pointer).  rsv_stage_acquire returns the free tail
 * of the handle's current pinned staging buffer -- room for *capacity keys (and hashes, for
 * RSV_HASH_PRECOMPUTED, else *hashes_out = NULL) -- and rsv_stage_commit(n) appends the first n
 * keys written there, exactly as n rsv_sample calls would.  A full buffer is flushed to the GPU
 * asynchronously and the next acquire returns the other buffer (double buffering).  The pointers
 * are valid until the next call on the handle. */
rsv_status rsv_stage_acquire(rsv_sampler* s, void** keys_out, int64_t** hashes_out, int64_t* capacity);
rsv_status rsv_stage_commit(rsv_sampler* s, int64_t n);

/* Sampler.sampleAll(elements) (S:49-50, S:289-316): appends n keys at global indices
 * [count, count+n).  mem says where `keys` (and `hashes`) live.  Identical results to n calls of
 * rsv_sample, for any split into batches (SamplerTest.scala:117-142). */
rsv_status rsv_sample_batch(rsv_sampler* s, const void* keys, int64_t n, int32_t mem,
                            const int64_t* hashes);

/* Sampler.sampleAll over a known-size IndexedSeq WITHOUT its keys (sampleAllImpl S:289-312 ->
 * sampleIndexed S:261-273, which reads only seq(nextSampleCount - count - 1) per eviction): the n
 * elements at global indices [count, count+n) are sampled by index alone -- a draw depends only on
 * the index (PHILOX_R), or the eviction events come from java.util.Random (JAVA_L) -- so only the
 * elements that end up in the reservoir need `map`.  slot_offsets_host[k] receives, per slot, the
 * offset in [0, n) of the element that now holds it (fill phase S:253-255 included), or -1 where
 * the slot did not change.  The caller maps exactly those elements (seq(offset)) and passes their
 * keys to rsv_fill_slots; until then every other call on the handle returns RSV_E_ILLEGAL_STATE.
 * ELEMENTS samplers only (Sampler.distinct maps every element: its sampleAll is the trait default,
 * S:50).  One K1 pass over the index range, k x 8 B back over PCIe -- no key crosses the link.
 * `map` then runs once per slot that changed, on its final holder: for a pure map the reservoir is
 * the reference's.  The reference calls map on every fill-phase element and on every evicting
 * element in order (S:241, :244, :269), so an impure map (side effects, call counts) or one that
 * throws midway observes fewer calls here; such a map belongs on the keyed path (rsv_sample_batch
 * with its keys), and a throw while keys are owed is undone with rsv_abort_indexed. */
rsv_status rsv_sample_indexed(rsv_sampler* s, int64_t n, int64_t* slot_offsets_host);
/* The keys owed after rsv_sample_indexed: keys_host holds k keys in slot order; entry j is read
 * only where slot_offsets_host[j] >= 0 (the rest may be anything). */
rsv_status rsv_fill_slots(rsv_sampler* s, const void* keys_host);
/* Drop the pending rsv_sample_indexed batch (the caller's `map` threw on an element it owed the
 * engine): the handle returns to its state before that call -- count, slots, result -- and takes
 * calls again; a binding then rethrows the exception, as the reference's sampleIndexed propagates
 * it (S:261-273).  The batch goes as a whole, where the reference keeps what it mapped before the
 * throw: after a throwing `map` the two differ in which of the batch's elements count.
 * RSV_E_ILLEGAL_STATE without a pending rsv_sample_indexed. */
rsv_status rsv_abort_indexed(rsv_sampler* s);
/* Accept the pending rsv_sample_indexed batch without keys: the caller keeps the elements itself.
 * For a `Sampler[A, B]` whose B has no fixed-width key (a case class, a String, any JVM object:
 * S:128-136 takes any B with a ClassTag), the binding holds the k-slot array of B references
 * (RandomElements.samples, S:200-202) and writes slots[j] = map(seq(slot_offsets[j])) (or the
 * already mapped element of a buffered batch) -- the engine decides WHICH element each slot holds
 * from the indices alone and never sees a B.  Afterwards the handle's slots hold no keys:
 * rsv_result / rsv_result_device / rsv_export_* return RSV_E_ILLEGAL_STATE, and every further batch
 * must be index-only (rsv_sample_indexed + rsv_commit_indexed or rsv_abort_indexed).
 * ELEMENTS samplers; RSV_E_ILLEGAL_STATE without a pending rsv_sample_indexed. */
rsv_status rsv_commit_indexed(rsv_sampler* s);

/* Sampler.result() (S:59-60; resultImpl S:318-331; RandomValues.result S:411).  Writes
 * min(count, k) keys (ELEMENTS: slot order, which is part of the reference result) or the distinct
 * set (DISTINCT: ascending scrambled hash; the reference's order is HashSet order) into host
 * memory `out` of `cap` keys, and the count into *out_n.  Single-use samplers close (S:345-350):
 * any later call but rsv_is_open returns RSV_E_ILLEGAL_STATE. */
rsv_status rsv_result(rsv_sampler* s, void* out, int64_t cap, int64_t* out_n);
/* Same, into device memory (no host round trip of the keys). */
rsv_status rsv_result_device(rsv_sampler* s, void* out_dev, int64_t cap, int64_t* out_n);
/* Same as rsv_result, without the host copy: a single-use sampler whose result is published into
 * its pinned result buffer (ELEMENTS and DISTINCT, k x key_width <= 1 MB) hands that buffer over.
 * *buf holds the *out_n keys (as rsv_result writes them) and belongs to the caller until
 * rsv_host_release(*buf); the sampler closes as after rsv_result.  The copy it saves is a read of
 * memory the GPU just wrote (k = 65536: ~22 us from DRAM).  Anything else (reusable samplers, larger
 * results) returns RSV_E_UNSUPPORTED with the sampler untouched: call rsv_result instead. */
rsv_status rsv_result_take(rsv_sampler* s, void** buf, int64_t* out_n);
void       rsv_host_release(void* buf);

int32_t    rsv_is_open(const rsv_sampler* s); /* Sampler.isOpen (S:67, S:193, S:380) */
int64_t    rsv_count(const rsv_sampler* s);   /* elements sampled so far (S:203) */

/* Streams: every handle owns a non-blocking HIP stream; a caller may substitute its own.  On the
 * handle's own stream every call returns with its device work finished (ownership of caller
 * buffers returns at once); on a caller stream, calls that take or fill DEVICE buffers
 * (rsv_sample_batch with RSV_MEM_DEVICE, rsv_export_state, rsv_merge_state, rsv_result_device) are
 * stream-ordered and return without a host wait.  rsv_set_stream orders the work already queued
 * on the previous stream before the new stream's next work (an event wait, no host wait). */
rsv_status rsv_set_stream(rsv_sampler* s, void* hip_stream);
void*      rsv_get_stream(const rsv_sampler* s);
/* Pipelining several samplers on one stream (ELEMENTS, batches whose K1 runs as its own dispatch:
 * > 2^27 draws): each batch's slot resolve and result publication (a one-workgroup dispatch of a few
 * microseconds) run on `hip_stream` instead, after the batch's K1 (an event), so the NEXT sampler's
 * K1 on the handle's stream does not wait behind them.  The handle's own later work waits for them
 * (an event), and rsv_result waits for the publication as always.  The keys of such a batch are read
 * on `hip_stream`: the caller keeps them unchanged until rsv_result (or rsv_synchronize) returns.
 * NULL = resolve on the handle's stream (the default). */
rsv_status rsv_set_resolve_stream(rsv_sampler* s, void* hip_stream);
rsv_status rsv_synchronize(rsv_sampler* s);

/* Kernel timing: while enabled, HIP events bracket every launch of the handle's hot kernel (K1
 * for PHILOX_R, the event replay K1' for JAVA_L, the K3 filter for DISTINCT) on its stream.
 * rsv_profile_read synchronizes and returns the summed kernel time and the launch count. */
rsv_status rsv_profile_enable(rsv_sampler* s, int32_t on);
rsv_status rsv_profile_read(rsv_sampler* s, double* total_ms, int64_t* launches);
/* Process-wide form (bench.py): while on, the hot-kernel launches of every ELEMENTS handle without
 * its own timing are bracketed by events kept in one process-wide list, so a timed loop that creates and
 * closes samplers pays no per-handle enable/read; rsv_profile_global_read synchronizes those events,
 * returns the totals since the last read and starts a new window.  `on` = 0 turns it off; N > 0
 * times every N-th launch from now on (1 = every launch; a larger N keeps the event packets off
 * most launches of a tight loop while the average stays a live measurement). */
rsv_status rsv_profile_global(int32_t on);
rsv_status rsv_profile_global_read(double* total_ms, int64_t* launches);

/* ---- Multi-GPU (index-range split of one stream; RSV_ENGINE_PHILOX_R / DISTINCT) ---------- */
/* Declare that the next sampled element has global index `index` (>= count): the elements in
 * between belong to other ranks.  PHILOX_R only. */
rsv_status rsv_seek(rsv_sampler* s, int64_t index);
/* Export the partial state into caller device buffers.
 *   ELEMENTS: idx_dev[k] = global index held by each slot (-1 = empty), keys_dev[k].
 *   DISTINCT: up to k (key, hash) pairs in ascending hash order, *out_n = count; idx_dev unused. */
rsv_status rsv_export_state(rsv_sampler* s, int64_t* idx_dev, void* keys_dev, int64_t* hash_dev,
                            int64_t* out_n);
/* Merge `parts` exported states (laid out back to back, `part_len` entries each, e.g. gathered
 * from every rank) into this sampler.  ELEMENTS: per slot the largest global index wins (last
 * writer).  DISTINCT: bottom-k of the union by (hash, key).  total_count sets the merged element
 * count.  An RSV_DISTINCT_ORDERED sampler merges the same way, which is the reference's set
 * unless the boundary hash bucket is oversubscribed (rsv_get_distinct_info `tied`); then the
 * exact set comes from rsv_export_log / rsv_merge_log below (reservoir_amd/distributed.py does
 * both).  With an injective hash the result is always identical. */
rsv_status rsv_merge_state(rsv_sampler* s, const int64_t* idx_dev, const void* keys_dev,
                           const int64_t* hash_dev, const int64_t* part_n_host, int32_t parts,
                           int64_t part_len, int64_t total_count);

/* ---- Exact multi-rank merge of ORDERED distinct samplers (the reference's default hash) ----- *
 * A stream split across ranks in order (rank r holds the r-th contiguous piece) is, to the
 * reference, one sequential RandomValues run (S:394-409): under a colliding hash the members of the
 * boundary hash bucket depend on that run's arrival order and heap ties.  rsv_merge_state gives the
 * (hash, key) bottom-k of the union; when rsv_get_distinct_info then reports `tied` (or a rank's own
 * set was tied at the merged maximum), the exact set comes from replaying every rank's logged
 * candidates in rank order: a rank's log is a superset of what the global run admits from its
 * piece (its local maximum is never below the global one), and the global heap's maximum inside
 * rank r's piece is below the k-th smallest hash of the pieces before it, so rank r exports only
 * candidates under that bound (reservoir_amd/distributed.py computes the bounds). */
typedef struct rsv_distinct_info {
    uint32_t struct_size;  /* = sizeof(rsv_distinct_info) */
    int32_t  ordered;      /* RSV_DISTINCT_ORDERED sampler */
    int32_t  tied;         /* set full and more distinct elements share its maximum hash than it keeps
                            * (ordered: of those the reference could admit; after rsv_merge_state: of
                            * the merged union) -- the boundary bucket needs the arrival order */
    int32_t  log_retained; /* ordered: rsv_export_log can return every candidate logged since creation */
    int64_t  size;         /* set size */
    int64_t  max_hash;     /* the set's largest scrambled hash (INT64_MIN when empty) */
    int64_t  log_entries;  /* ordered: upper bound on rsv_export_log's count */
    int64_t  sched_passes;    /* ordered: batches taken by one verified scheduled pass */
    int64_t  sched_fallbacks; /* ordered: scheduled passes that failed verification or overflowed and
                               * left the batch to the chunk loop (the set restored) */
} rsv_distinct_info;
rsv_status rsv_get_distinct_info(rsv_sampler* s, rsv_distinct_info* out);
/* Keep every logged candidate on the host for rsv_export_log (ORDERED samplers; off by default: the
 * archive holds 12-16 B per replayed candidate, up to 2^27 of them).  Call it before the first
 * sample -- switched on later, the log is reported as not retained. */
rsv_status rsv_retain_log(rsv_sampler* s, int32_t on);
/* Every logged candidate with scrambled hash < bound (all of them for bound = INT64_MAX), in
 * arrival order, into host buffers of cap entries (keys as key_width values); *out_n = the count
 * (RSV_E_ILLEGAL_ARGUMENT when it exceeds cap; cap = 0 is a count-only query, the buffers may be
 * NULL).  RSV_E_UNSUPPORTED if the log was not retained (rsv_retain_log).
 * Stays available after rsv_merge_state until the sampler samples again. */
rsv_status rsv_export_log(rsv_sampler* s, int64_t bound, int64_t* hashes_host, void* keys_host, int64_t cap,
                          int64_t* out_n);
/* Replace the state by a fresh RandomValues replica run over n candidates (host, in global arrival
 * order: rank 0's export, then rank 1's, ...), as if the sampler had seen the whole stream. */
rsv_status rsv_merge_log(rsv_sampler* s, const int64_t* hashes_host, const void* keys_host, int64_t n,
                         int64_t total_count);

/* Packed form of rsv_export_state / rsv_merge_state, the one-collective combine of
 * reservoir_amd/distributed.py.  One kernel, no host wait on a caller stream.
 *   ELEMENTS: row_dev[0..k) = global index per slot (-1 = empty), row_dev[k..2k) = the slot's key
 *     widened to int64 (sign-extended for 4-byte keys); for wide keys (key_width > 8) the k keys
 *     follow as key_width/8 int64 words each.
 *   DISTINCT: [keys (k) | scrambled hashes (k) | n, count, tied, max_hash, log_retained, ordered] --
 *     the set ascending by (hash, key), n entries valid; keys widened to int64 (2k + 6 words), or for
 *     byte keys key_width / 8 words each (k (key_width / 8 + 1) + 6 words, ascending by (hash, key
 *     words compared as unsigned 64-bit, word 0 first)). */
rsv_status rsv_export_packed(rsv_sampler* s, int64_t* row_dev);
/* Merge `parts` packed rows (row p at rows_dev + p*row_stride, row_stride >= the row length), e.g. the output
 * of an all-gather of every rank's rsv_export_packed row.
 *   ELEMENTS: per slot the largest global index wins.
 *   DISTINCT: the bottom-k by (hash, key) of the union with the sampler's set, on the device (four
 *     kernels, no host wait: the set's size and tie state are read back at the next call on the
 *     handle); `tied` as rsv_merge_state.  The rows are the caller's again once the merge has run
 *     in stream order (the engine keeps its own copy for a degenerate hash that overflows the
 *     merge's buckets, redone at the next call).  Byte-key DISTINCT samplers merge before the call
 *     returns (the host reads the rows' meta words). */
rsv_status rsv_merge_packed(rsv_sampler* s, const int64_t* rows_dev, int32_t parts, int64_t row_stride,
                            int64_t total_count);

/* ---- Stateless batch entry points --------------------------------------------------------- */
/* Segmented sampling: S independent Algorithm-R samplers (no reference counterpart; = S separate
 * Sampler instances, S:196-332).  Stream s samples keys_dev[offsets[s] .. offsets[s+1]) with
 * Philox stream id stream_base + s and writes out_dev[s*k .. s*k+k) (slot order; slots >=
 * counts[s] are zero) and counts_dev[s] = min(len, k).  All pointers are device pointers. */
rsv_status rsv_sample_segmented(const void* keys_dev, const int64_t* offsets_dev, int64_t num_streams,
                                int32_t key_width, int32_t k, uint64_t seed, uint64_t stream_base,
                                void* out_dev, int64_t* counts_dev, void* hip_stream);

/* Event replay (K1'): apply eviction events (1-based position, slot) -- the
 * `samples(rand.nextInt(k)) = map(element)` writes of S:243-246 -- for elements at global indices
 * [base_index, base_index+n) held in keys_dev, onto reservoir_dev[k] (in/out, device).  Also
 * performs the fill phase (S:253-255) for indices < k.  The last event per slot wins. */
rsv_status rsv_replay_events(const void* keys_dev, int64_t n, int32_t key_width, int64_t base_index,
                             const int64_t* ev_pos_dev, const int32_t* ev_slot_dev, int64_t n_events,
                             int32_t k, void* reservoir_dev, void* hip_stream);

/* Export the per-element draw sequence j_i (format R2) for indices [i0, i0+n) into j_dev. */
rsv_status rsv_export_draws(uint64_t seed, uint64_t stream_id, uint64_t i0, int64_t n,
                            uint64_t* j_dev, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* RESERVOIR_HIP_H */
