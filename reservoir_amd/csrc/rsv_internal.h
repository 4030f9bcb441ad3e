// rsv_internal.h -- host-side declarations shared between the runtime and the kernel translation
// units of libreservoir_hip.so.  Not part of the public ABI (that is include/reservoir_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace rsv {

// thread-local last error (rsv_last_error)
void set_error(const std::string& msg);

#define RSV_HIP_TRY(expr)                                                                     \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            ::rsv::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));              \
            return _e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;            \
        }                                                                                     \
    } while (0)

// ---- resource pool (rsv_pool.hip): device / pinned host buffers, streams, events ------------
// Allocation is on the current device.  A buffer may only be released once no queued work can
// touch it (synchronize its stream first).
hipError_t pool_device_alloc(void** p, size_t bytes);
void pool_device_free(void* p);
hipError_t pool_host_alloc(void** p, size_t bytes, unsigned flags);
void pool_host_free(void* p);
void pool_trim();  // free every idle cached buffer
hipError_t pool_stream(hipStream_t* out);  // non-blocking stream of the current device
void pool_release_stream(int device, hipStream_t st);
hipError_t pool_event(hipEvent_t* out, unsigned flags);
void pool_release_event(int device, hipEvent_t e, unsigned flags);

// HIP-event timing of a handle's hot kernel (rsv_profile_enable / rsv_profile_read)
struct KernelTimer {
    bool on = false;
    int device = 0;
    std::vector<hipEvent_t> ev;  // start/stop pairs, recycled after each drain
    size_t used = 0;
    double total_ms = 0;
    int64_t launches = 0;
    // Timing-only events (hipEventDisableSystemFence): each record skips the system-scope fence,
    // which costs the timed stream ~5 us per step less than default events and ~9 us less than
    // hipExtLaunchKernelGGL's start/stop events (tools/probe_events.hip, MI355X).
    static constexpr unsigned kFlags = hipEventDisableSystemFence;
    void mark(hipStream_t st) {
        if (!on) return;
        if (used == ev.size()) {
            hipEvent_t e;
            if (pool_event(&e, kFlags) != hipSuccess) return;
            ev.push_back(e);
        }
        (void)hipEventRecord(ev[used++], st);
    }
    hipError_t drain() {
        for (size_t i = 0; i + 1 < used; i += 2) {
            hipError_t e = hipEventSynchronize(ev[i + 1]);
            if (e != hipSuccess) return e;
            float ms = 0;
            e = hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
            if (e != hipSuccess) return e;
            total_ms += ms;
            launches++;
        }
        used = 0;
        return hipSuccess;
    }
    ~KernelTimer() {
        for (hipEvent_t e : ev) pool_release_event(device, e, kFlags);
    }
};

struct DrawParams {
    uint64_t seed;
    uint64_t stream;
};

// ---- elements (Algorithm R, draw format R2) -------------------------------------------------
// K1: per-slot last writer of the index range [lo, hi) (only indices >= k can evict) into
// batch_win[k] (0 = no writer in this batch; atomicMax keeps the largest index).
hipError_t launch_k1_last_writer(const DrawParams& dp, uint32_t k, uint64_t lo, uint64_t hi,
                                 unsigned long long* batch_win, hipStream_t st);
// K1 + resolve_publish as one dispatch (see launch_resolve_publish), when k1_fused_ok: a batch
// whose range K1 covers in one launch, k <= 2048, 4- or 8-byte keys.  ticket: a zeroed device
// word, re-armed by the launch.
bool k1_fused_ok(uint64_t lo, uint64_t hi, uint32_t k, int key_width);
hipError_t launch_k1_resolve_publish(const DrawParams& dp, uint32_t k, uint64_t lo, uint64_t hi,
                                     unsigned long long* batch_win, uint32_t* ticket, const void* keys,
                                     int key_width, int64_t base, int64_t n, void* slot_key, int64_t* slot_idx,
                                     bool fresh, int64_t m, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen,
                                     hipStream_t st);
// Resolve: fill phase for slots in [base, base+n) and winners of batch_win; resets batch_win.
// slot_idx may be null.  init_slots also zeroes `ticket` when non-null.
hipError_t launch_init_slots(void* slot_key, int key_width, int64_t* slot_idx, unsigned long long* win, uint32_t k,
                             hipStream_t st, uint32_t* ticket = nullptr);
hipError_t launch_publish(const void* src, int64_t bytes, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen,
                          hipStream_t st);
// the same from up to 32 workgroups (large buffers); ticket_dev: a zeroed device word, re-armed
hipError_t launch_publish_multi(const void* src, int64_t bytes, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen,
                                uint32_t* ticket_dev, hipStream_t st);
hipError_t launch_resolve(const void* keys, int key_width, int64_t base, int64_t n, uint32_t k,
                          unsigned long long* batch_win, void* slot_key, int64_t* slot_idx, bool fresh,
                          hipStream_t st);
// resolve + publish of the first m slot keys into coherent host memory + flag = gen (k <= 8192;
// slot_idx must be non-null); small: one 256-thread workgroup where k <= 2048 (a resolve running
// beside K1 on a second stream)
hipError_t launch_resolve_publish(const void* keys, int key_width, int64_t base, int64_t n, uint32_t k,
                                  unsigned long long* batch_win, void* slot_key, int64_t* slot_idx, bool fresh,
                                  int64_t m, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st,
                                  bool small = false);
// index-only batches: resolve into slot_idx with offs[k] = the batch offset of each changed slot
// (-1: unchanged); then the caller's keys into the changed slots
hipError_t launch_resolve_indices(int64_t base, int64_t n, uint32_t k, unsigned long long* batch_win, int64_t* slot_idx,
                                  bool fresh, void* slot_key, int key_width, int64_t* offs, hipStream_t st);
hipError_t launch_fill_slots(const int64_t* offs, const void* keys, uint32_t k, int key_width, void* slot_key,
                             hipStream_t st);
// one-dispatch forms (k <= 8192): resolve_indices + offs[] also into coherent host memory + flag = gen;
// fill_slots + the first m slot keys into coherent host memory + flag = gen (4- / 8-byte keys)
bool resolve_indices_publish_ok(uint32_t k);
hipError_t launch_resolve_indices_publish(int64_t base, int64_t n, uint32_t k, unsigned long long* batch_win,
                                          int64_t* slot_idx, bool fresh, void* slot_key, int key_width, int64_t* offs,
                                          int64_t* offs_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st);
bool fill_slots_publish_ok(uint32_t k, int key_width);
hipError_t launch_fill_slots_publish(const int64_t* offs, const void* keys, uint32_t k, int key_width, void* slot_key,
                                     int64_t m, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st);
// K1': events (1-based pos, slot) -> batch_win
hipError_t launch_replay_events(const int64_t* ev_pos, const int32_t* ev_slot, int64_t n_events,
                                uint32_t k, unsigned long long* batch_win, hipStream_t st);
hipError_t launch_export_draws(const DrawParams& dp, uint64_t i0, int64_t n, uint64_t* j,
                               hipStream_t st);
// K2: segmented
hipError_t launch_segmented(const void* keys, int key_width, const int64_t* offsets, int64_t S,
                            uint32_t k, const DrawParams& dp, void* out, int64_t* counts,
                            hipStream_t st);
// merge of exported element states: per slot max index among parts (and current state)
hipError_t launch_merge_slots(const int64_t* idx_parts, const void* key_parts, int key_width,
                              int32_t parts, int64_t part_len, uint32_t k, int64_t* slot_idx,
                              void* slot_key, hipStream_t st);

// packed combine rows: [slot_idx(k) | keys as int64 (k)]
hipError_t launch_export_packed(const int64_t* slot_idx, const void* slot_key, int key_width, uint32_t k,
                                int64_t* row, hipStream_t st);
hipError_t launch_merge_packed(const int64_t* rows, int32_t parts, int64_t stride, uint32_t k, int64_t* slot_idx,
                               void* slot_key, int key_width, hipStream_t st);

// merge of packed rows + publication of the first m keys (k <= 8192, key_width 4 / 8)
hipError_t launch_merge_packed_publish(const int64_t* rows, int32_t parts, int64_t stride, uint32_t k,
                                       int64_t* slot_idx, void* slot_key, int key_width, int64_t m, void* dst_host_dev,
                                       uint32_t* flag_dev, uint32_t gen, hipStream_t st);

// ---- distinct (bottom-k over the scrambled hash) --------------------------------------------
struct DistinctState;  // defined in rsv_distinct.hip
// ordered: RSV_DISTINCT_ORDERED semantics (exact sequential replay; see rsv_distinct.hip)
DistinctState* distinct_create(int32_t k, int key_width, int hash_kind, int64_t r0, int64_t r1, bool ordered,
                               int* status);
void distinct_set_timer(DistinctState* d, KernelTimer* t);
void distinct_destroy(DistinctState* d);
// keys/hashes are device pointers
int distinct_sample_device(DistinctState* d, const void* keys, const int64_t* hashes, int64_t n,
                           hipStream_t st);
int64_t distinct_size(const DistinctState* d);
// RSV_DISTINCT_ORDERED: bring the set arrays to the reference's set (host replay of the logged
// candidates when the tie bucket requires it); a no-op otherwise.  Before size / export / publish.
int distinct_finalize(DistinctState* d, hipStream_t st);
const void* distinct_keys_dev(const DistinctState* d);  // the current set's keys (m of them)
// the set's m keys into coherent host memory (device-mapped pointer) + flag = gen
int distinct_publish(DistinctState* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st);
// Speculative publication (set mode, large batches): the next distinct_sample_device enqueues the
// merged set's publication into dst_host_dev + flag_dev (generation ++*gen_counter) right behind
// its ctl read; distinct_spec_take says whether the last one holds the batch's final set (its
// generation in *gen) and clears the target.
void distinct_spec_target(DistinctState* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t* gen_counter);
bool distinct_is_ordered(const DistinctState* d);
int64_t distinct_spec_min(const DistinctState* d);  // smallest batch that publishes speculatively
bool distinct_spec_take(DistinctState* d, uint32_t* gen);
// copies the set (ascending hash) to device buffers; either may be null
int distinct_export(DistinctState* d, void* keys_dev, int64_t* hash_dev, hipStream_t st);
// merge `parts` external (key, hash) runs (device; run p at p * part_len) into the set
int distinct_merge_parts(DistinctState* d, const void* keys_dev, const int64_t* hash_dev, const int64_t* part_n,
                         int32_t parts, int64_t part_len, hipStream_t st);
void distinct_info(const DistinctState* d, int32_t* ordered, int32_t* tied, int32_t* retained, int64_t* size,
                   int64_t* max_hash, int64_t* log_entries, int64_t* sched_passes, int64_t* sched_fallbacks);
// ordered samplers: every logged candidate with h < bound (all of them for bound = INT64_MAX) in
// arrival order into host buffers; the exact replay of a concatenated candidate run
int distinct_log_export(DistinctState* d, int64_t bound, int64_t* out_h, void* out_k, int64_t cap, int64_t* out_n,
                        hipStream_t st);
int distinct_log_merge(DistinctState* d, const int64_t* h, const void* keys, int64_t n, int64_t seen,
                       hipStream_t st);
// packed rows [keys as int64 (k) | hashes (k) | n, count, tied, max_hash, log_retained, ordered]:
// export of the set (count = the handle's element count), and the device merge of `parts` rows into
// the set -- enqueued without a host wait; `rows` must stay valid until the next call on the state,
// which settles the merge (distinct_settle; every other distinct_* call settles first)
int distinct_export_row(DistinctState* d, int64_t* row, int64_t count, hipStream_t st);
int distinct_merge_rows(DistinctState* d, const int64_t* rows, int32_t parts, int64_t stride, hipStream_t st);
int distinct_settle(DistinctState* d, hipStream_t st);
// ordered samplers: keep every replayed candidate on the host for rsv_export_log (opt-in)
void distinct_retain_log(DistinctState* d, bool on);

// ---- distinct over fixed-width byte keys (rsv_wide.hip; key_width 16..256, a multiple of 8) ------
// The same contract as the distinct_* functions above (which forward here for key_width > 8); keys
// are rows of key_width / 8 int64 words, hashes precomputed (src kWideSrcHashes) or UUID.hashCode of
// 16-byte rows (kWideSrcUuid).  Every call completes its device work before it returns.
struct WideDistinct;
WideDistinct* wide_create(int32_t k, int key_width, int src, int64_t r0, int64_t r1, bool ordered, int* status);
void wide_destroy(WideDistinct* d);
void wide_set_timer(WideDistinct* d, KernelTimer* t);
int64_t wide_size(const WideDistinct* d);
const void* wide_keys_dev(const WideDistinct* d);
bool wide_is_ordered(const WideDistinct* d);
int wide_sample_device(WideDistinct* d, const void* keys, const int64_t* hashes, int64_t n, hipStream_t st);
int wide_finalize(WideDistinct* d, hipStream_t st);
int wide_publish(WideDistinct* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st);
int wide_export(WideDistinct* d, void* keys_dev, int64_t* hash_dev, hipStream_t st);
void wide_info(const WideDistinct* d, int32_t* ordered, int32_t* tied, int32_t* retained, int64_t* size,
               int64_t* max_hash, int64_t* log_entries);
int wide_merge_parts(WideDistinct* d, const void* keys_dev, const int64_t* hash_dev, const int64_t* part_n,
                     int32_t parts, int64_t part_len, hipStream_t st);
int wide_export_row(WideDistinct* d, int64_t* row, int64_t count, hipStream_t st);
int wide_merge_rows(WideDistinct* d, const int64_t* rows, int32_t parts, int64_t stride, hipStream_t st);
void wide_retain_log(WideDistinct* d, bool on);
// set mode's one-pass batches: the merged set published into dst_host_dev + flag_dev (generation
// ++*gen_counter) right behind the merge; wide_spec_take says whether it holds the batch's final set
void wide_spec_target(WideDistinct* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t* gen_counter);
bool wide_spec_take(WideDistinct* d, uint32_t* gen);
int wide_log_export(WideDistinct* d, int64_t bound, int64_t* out_h, void* out_k, int64_t cap, int64_t* out_n,
                    hipStream_t st);
int wide_log_merge(WideDistinct* d, const int64_t* h, const void* keys, int64_t n, int64_t seen, hipStream_t st);

}  // namespace rsv
