// rsv_runtime.hip -- implementation of the C ABI (include/reservoir_hip.h): sampler handles,
// lifecycle (SingleUse / MultiResult, Sampler.scala:182-194, :334-381, :414-433), staging of
// per-element calls into pinned batches, host->device batching, engine dispatch, multi-GPU
// state export/merge.  All data-parallel work runs in the kernels of rsv_elements.hip and
// rsv_distinct.hip; there is no CPU compute path.
#include <cstdlib>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/reservoir_hip.h"
#include "rsv_device.h"
#include "rsv_internal.h"

namespace rsv {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }


// ---------------------------------------------------------------------------------------------
// java.util.Random + Algorithm L event generator for RSV_ENGINE_JAVA_L (product implementation;
// the oracle under oracle/ is an independent restatement used only by the tests).
struct JavaRandom {
    uint64_t seed = 0;
    void init(int64_t s) { seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
    int32_t next(int bits) {
        seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        return (int32_t)(uint32_t)(seed >> (48 - bits));
    }
    double next_double() {  // java.util.Random.nextDouble
        const int64_t a = next(26), b = next(27);
        return (double)((a << 27) + b) * 0x1.0p-53;
    }
    int32_t next_int(int32_t bound) {  // java.util.Random.nextInt(int)
        int32_t r = next(31);
        const int32_t m = bound - 1;
        if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)r) >> 31);
        for (int32_t u = r;; u = next(31)) {
            r = u % bound;
            if ((int32_t)((uint32_t)u - (uint32_t)r + (uint32_t)m) >= 0) break;
        }
        return r;
    }
    int64_t next_long() {
        const int64_t hi = next(32), lo = next(32);
        return (int64_t)(((uint64_t)hi << 32) + (uint64_t)lo);
    }
};

struct AlgoLState {  // RandomElements' private state (Sampler.scala:199-205)
    JavaRandom rand;
    int32_t k = 0;
    double W = 1.0;
    int64_t next_sample_count = 0;

    static int64_t d2l(double d) {  // JVM double -> long (saturating, NaN -> 0)
        if (d != d) return 0;
        if (d >= 9223372036854775807.0) return INT64_MAX;
        if (d <= -9223372036854775808.0) return INT64_MIN;
        return (int64_t)d;
    }
    void update() {  // updateNextSampleCount, Sampler.scala:228-236
        W = W * std::exp(std::log(rand.next_double()) / (double)k);
        const double skip = std::floor(std::log(rand.next_double()) / std::log(1.0 - W));
        next_sample_count = (int64_t)((uint64_t)next_sample_count + (uint64_t)d2l(skip) + 1ULL);
    }
    void init(int32_t kk, int64_t seed) {  // as SamplerTest.useConsistentRandom re-seeds it
        k = kk;
        rand.init(seed);
        W = 1.0;
        next_sample_count = kk;
        update();
    }
    // eviction events for 1-based positions (base, base+n] -- the per-element rule of
    // sampleImpl (Sampler.scala:248-259): position c > k evicts iff c >= nextSampleCount.
    void events(int64_t base, int64_t n, std::vector<int64_t>& pos, std::vector<int32_t>& slot) {
        int64_t cur = base + 1;
        const int64_t end = base + n;
        if (cur <= k) cur = (int64_t)k + 1;
        while (cur <= end) {
            const int64_t p = std::max(next_sample_count, cur);
            if (p > end) break;
            pos.push_back(p);
            slot.push_back(rand.next_int(k));  // sampleWithEviction, Sampler.scala:243-246
            update();
            cur = p + 1;
        }
    }
};

}  // namespace rsv

using namespace rsv;

struct rsv_sampler {
    rsv_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool open = true;
    int64_t count = 0;
    int kw = 8;
    uint32_t k = 0;
    // ELEMENTS
    void* slots = nullptr;  // one pooled block: batch_win[k] | slot_idx[k] | slot_key[k] | k1_ticket
    // device-state knowledge, in stream order: batch_win all zero (resolve leaves it so) / slot
    // arrays initialised.  Creation enqueues no device work; the first batch initialises.
    bool win_zero = false;
    bool slots_init = false;
    void* slot_key = nullptr;
    int64_t* slot_idx = nullptr;
    unsigned long long* batch_win = nullptr;
    uint32_t* k1_ticket = nullptr;  // fused K1 + resolve_publish: zero between launches
    AlgoLState algo_l;
    std::vector<int64_t> ev_pos_h;
    std::vector<int32_t> ev_slot_h;
    int64_t* ev_pos_d = nullptr;
    int32_t* ev_slot_d = nullptr;
    int64_t ev_cap = 0;
    // index-only batches (rsv_sample_indexed): per slot the batch offset of its new element, and
    // whether the caller still owes those elements' keys (rsv_fill_slots)
    int64_t* idx_offs_d = nullptr;
    bool keys_owed = false;
    // rsv_commit_indexed: the caller keeps the elements (any JVM B); the slots hold no keys
    bool keys_external = false;
    // rsv_abort_indexed: the slot indices before the pending index-only batch, and its start
    int64_t* idx_bak_d = nullptr;
    bool idx_fresh = false;
    int64_t idx_base = 0;
    AlgoLState idx_algo_l;  // JAVA_L: java.util.Random and W before the batch's events
    // the index-only batch's offsets in host memory: k <= 8192 coherent + mapped, published by the
    // resolve kernel with flag offs_flag = offs_gen; larger k a pinned D2H target
    int64_t* offs_h = nullptr;
    int64_t* offs_dev = nullptr;
    uint32_t* offs_flag = nullptr;
    uint32_t* offs_flag_dev = nullptr;
    uint32_t offs_gen = 0;
    // the winners' keys in slot order (host gather of a winners-only batch, rsv_fill_slots): pinned,
    // coherent and mapped, read by the fill kernel across PCIe (no H2D copy, no host wait)
    uint8_t* gath_h = nullptr;
    void* gath_dev = nullptr;
    // DISTINCT
    DistinctState* distinct = nullptr;
    int hash_kind = kHashIdentity;
    // host staging: per-element calls and host batches
    // per-element sample(): two pinned staging buffers; a full one is flushed asynchronously
    // (H2D + kernels, no host wait) while the other fills; an event says when it is free again
    uint8_t* stage_h[2] = {nullptr, nullptr};
    void* stage_dev[2] = {nullptr, nullptr};  // device aliases (winners-only flushes read them in place)
    int64_t* stage_hash_h[2] = {nullptr, nullptr};
    hipEvent_t stage_free[2] = {nullptr, nullptr};
    // java_l staged flushes: the batch's Algorithm-L events in pinned memory owned by the staging
    // buffer (free again with stage_free[b]), so their H2D copies need no host wait
    int64_t* stage_ev_pos[2] = {nullptr, nullptr};
    int32_t* stage_ev_slot[2] = {nullptr, nullptr};
    int64_t stage_ev_cap[2] = {0, 0};
    bool stage_pending[2] = {false, false};
    int stage_cur = 0;
    int64_t stage_n = 0;
    int64_t stage_cap = 0;
    void* chunk_d = nullptr;     // device chunk for host batches
    int64_t* chunk_hash_d = nullptr;
    int64_t chunk_cap = 0;
    void* result_h = nullptr;  // pinned staging for result() (k keys)
    // small reservoirs: result_h is coherent + mapped and publish_kernel writes it directly,
    // followed by result_gen in result_flag (same allocation); the host spins on the flag
    bool result_publish = false;
    void* result_dev = nullptr;  // device alias of result_h
    uint32_t* result_flag = nullptr;
    uint32_t* result_flag_dev = nullptr;
    uint32_t result_gen = 0;
    // small reservoirs: every batch's resolve also publishes the reservoir (resolve_publish
    // kernel), so result() only waits for generation pub_gen -- while pub_valid says no other
    // kernel (merge, init) has changed the slots since
    uint32_t pub_gen = 0;
    bool pub_valid = false;
    KernelTimer timer;
    hipEvent_t handover = nullptr;  // rsv_set_stream's event (kept until destroy: see there)
    // rsv_set_resolve_stream: each batch's resolve + publication on this caller stream, forked from
    // `stream` after K1 (side_fork) and joined back (side_join) before the handle's next device work
    hipStream_t rstream = nullptr;
    hipEvent_t side_fork = nullptr, side_join = nullptr;
    bool side_pending = false;
    // device work enqueued on `stream` by this handle, in groups, vs the groups known complete
    // (a stream synchronize, or the host flag of a publication that was the last group)
    uint64_t ops = 0, ops_done = 0, pub_ops = 0;
};

namespace {

// process-wide hot-kernel timer (rsv_profile_global); guarded by g_prof_mu
std::mutex g_prof_mu;
std::atomic<bool> g_prof_on{false};
KernelTimer& global_timer() {
    static auto* t = new KernelTimer();  // leaked on purpose, like the pool
    return *t;
}

// a new group of device work on the handle's stream / everything enqueued so far is complete
// the forked resolve (rsv_set_resolve_stream) ordered before the handle's next work on its stream
inline void join_side(rsv_sampler* s) {
    if (!s->side_pending) return;
    (void)hipStreamWaitEvent(s->stream, s->side_join, 0);
    s->side_pending = false;
}
inline void touch(rsv_sampler* s) {
    join_side(s);
    ++s->ops;
}
inline hipError_t sync_stream(rsv_sampler* s) {
    join_side(s);
    hipError_t e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) s->ops_done = s->ops;
    return e;
}

// Timing marks around the handle's hot kernel: its own timer (every launch), else the process-wide
// one, which times every g_prof_every-th launch (rsv_profile_global).  prof_begin's return value
// goes to the matching prof_end.
std::atomic<int64_t> g_prof_every{1};
int64_t g_prof_seq = 0;  // guarded by g_prof_mu

bool prof_begin(rsv_sampler* s, hipStream_t st) {
    if (s->timer.on) {
        s->timer.mark(st);
        return true;
    }
    if (!g_prof_on) return false;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (g_prof_seq++ % g_prof_every != 0) return false;
    KernelTimer& t = global_timer();
    t.on = true;
    t.device = s->device;
    t.mark(st);
    return true;
}

void prof_end(rsv_sampler* s, hipStream_t st, bool marked) {
    if (!marked) return;
    if (s->timer.on) {
        s->timer.mark(st);
        return;
    }
    std::lock_guard<std::mutex> lk(g_prof_mu);
    global_timer().mark(st);
}

constexpr int32_t kMaxSize = 2147483647 - 2;  // Sampler.scala:71 (hotspot VM array limit)
constexpr int64_t kStageKeys = 1 << 20;
constexpr int64_t kChunkKeys = 1 << 22;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

rsv_status fail(rsv_status st, const std::string& msg) {
    set_error(msg);
    return st;
}

rsv_status check_open(const rsv_sampler* s) {  // SingleUse.checkOpen, Sampler.scala:185-186
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    if (!s->open) return fail(RSV_E_ILLEGAL_STATE, "use of sampler after calling `result()`");
    if (s->keys_owed) return fail(RSV_E_ILLEGAL_STATE, "rsv_fill_slots is pending after rsv_sample_indexed");
    return RSV_OK;
}

// entry points that read or write keys: not on a handle whose caller keeps the elements
rsv_status check_keyed(const rsv_sampler* s) {
    if (rsv_status st = check_open(s)) return st;
    if (s->keys_external)
        return fail(RSV_E_ILLEGAL_STATE, "the slots hold no keys (rsv_commit_indexed): index-only batches only");
    return RSV_OK;
}

rsv_status ensure_events(rsv_sampler* s, int64_t n) {
    if (n <= s->ev_cap) return RSV_OK;
    int64_t cap = std::max<int64_t>(n, 2 * s->ev_cap);
    if (s->ev_pos_d || s->ev_slot_d) RSV_HIP_TRY(sync_stream(s));  // before reuse elsewhere
    pool_device_free(s->ev_pos_d);
    pool_device_free(s->ev_slot_d);
    s->ev_pos_d = nullptr;
    s->ev_slot_d = nullptr;
    s->ev_cap = 0;
    RSV_HIP_TRY(pool_device_alloc((void**)&s->ev_pos_d, cap * 8));
    RSV_HIP_TRY(pool_device_alloc((void**)&s->ev_slot_d, cap * 4));
    s->ev_cap = cap;
    return RSV_OK;
}

// slot arrays of a fresh handle: slot_key = 0, slot_idx = -1 (empty), batch_win = 0, on the
// handle's current stream before its first use (creation itself enqueues no device work)
rsv_status ensure_slots(rsv_sampler* s) {
    if (s->slots_init || s->cfg.kind != RSV_KIND_ELEMENTS) return RSV_OK;
    touch(s);
    RSV_HIP_TRY(launch_init_slots(s->slot_key, s->kw, s->slot_idx, s->batch_win, s->k, s->stream, s->k1_ticket));
    s->slots_init = s->win_zero = true;
    s->pub_valid = false;
    return RSV_OK;
}

// Slot blocks whose batch_win is known zero (their last sampler ended on a resolve): a new handle
// of the same (k, key width) takes one and skips the init kernel -- its first resolve marks the
// untouched slots empty instead (resolve_kernel `fresh`).
struct CleanSlots {
    void* p;
    uint32_t k;
    int kw;
    int device;
};
std::mutex g_clean_mu;
std::vector<CleanSlots>& clean_slots() {
    static auto* v = new std::vector<CleanSlots>();  // leaked on purpose, like the pool
    return *v;
}

void* take_clean_slots(uint32_t k, int kw, int device) {
    std::lock_guard<std::mutex> lk(g_clean_mu);
    auto& v = clean_slots();
    for (size_t i = v.size(); i-- > 0;)
        if (v[i].k == k && v[i].kw == kw && v[i].device == device) {
            void* p = v[i].p;
            v.erase(v.begin() + (ptrdiff_t)i);
            return p;
        }
    return nullptr;
}

bool give_clean_slots(void* p, uint32_t k, int kw, int device) {
    if ((uint64_t)k * (16 + kw) > (64ull << 20)) return false;
    std::lock_guard<std::mutex> lk(g_clean_mu);
    auto& v = clean_slots();
    if (v.size() >= 32) return false;
    v.push_back(CleanSlots{p, k, kw, device});
    return true;
}

constexpr int64_t kPublishMaxBytes = 1 << 20;

rsv_status ensure_result_buffer(rsv_sampler* s) {
    if (s->result_h) return RSV_OK;
    const size_t bytes = (size_t)s->k * s->kw;
    if ((int64_t)bytes <= kPublishMaxBytes) {
        const size_t flag_off = (bytes + 63) & ~(size_t)63;
        RSV_HIP_TRY(pool_host_alloc(&s->result_h, flag_off + 64, hipHostMallocCoherent | hipHostMallocMapped));
        void* dev = nullptr;
        RSV_HIP_TRY(hipHostGetDevicePointer(&dev, s->result_h, 0));
        s->result_dev = dev;
        s->result_flag = (uint32_t*)((uint8_t*)s->result_h + flag_off);
        s->result_flag_dev = (uint32_t*)((uint8_t*)dev + flag_off);
        *s->result_flag = s->result_gen;
        s->result_publish = true;
    } else {
        RSV_HIP_TRY(pool_host_alloc(&s->result_h, bytes, hipHostMallocDefault));
    }
    return RSV_OK;
}

constexpr uint32_t kFusedPublishMaxK = 8192;  // resolve_publish: one workgroup, <= 8 slots per lane

// a resolve forked onto the resolve stream runs as ONE 256-thread workgroup (beside the next K1;
// RSV_RESOLVE_SMALL=0: the 1024-thread form, for A/B)
bool resolve_small() {
    static const bool v = [] {
        const char* e = std::getenv("RSV_RESOLVE_SMALL");
        return !(e && e[0] == '0');
    }();
    return v;
}

// The batch's resolve: fill phase + winners into the slots; for reservoirs of <= 8192 keys it
// also writes the first min(count, k) keys into the coherent result buffer and publishes
// generation ++result_gen there (one dispatch instead of resolve now + publish at result()).
rsv_status resolve_batch(rsv_sampler* s, const void* keys, int64_t base, int64_t n, bool fresh,
                         hipStream_t rst = nullptr) {
    if (!rst) rst = s->stream;
    if (s->k <= kFusedPublishMaxK) {
        if (rsv_status st = ensure_result_buffer(s)) return st;
        if (s->result_publish) {
            const uint32_t gen = ++s->result_gen;
            const int64_t m = std::min<int64_t>(base + n, (int64_t)s->k);
            RSV_HIP_TRY(launch_resolve_publish(keys, s->kw, base, n, s->k, s->batch_win, s->slot_key, s->slot_idx,
                                               fresh, m, s->result_dev, s->result_flag_dev, gen, rst,
                                               rst != s->stream && resolve_small()));
            s->pub_ops = s->ops;  // the last work of this group
            s->pub_gen = gen;
            s->pub_valid = true;
            return RSV_OK;
        }
    }
    RSV_HIP_TRY(launch_resolve(keys, s->kw, base, n, s->k, s->batch_win, s->slot_key, s->slot_idx, fresh, rst));
    s->pub_valid = false;
    return RSV_OK;
}

// one batch of n keys already in device memory, at global indices [count, count+n); stage_b >= 0:
// the batch is staging buffer stage_b, whose pinned event buffers carry java_l's events
rsv_status process_device_batch(rsv_sampler* s, const void* keys, const int64_t* hashes, int64_t n,
                                int stage_b = -1) {
    if (n <= 0) return RSV_OK;
    touch(s);
    const int64_t base = s->count;
    bool fresh = false;
    if (s->cfg.kind == RSV_KIND_ELEMENTS) {
        if (!s->win_zero) {  // never-used block: full init
            RSV_HIP_TRY(launch_init_slots(s->slot_key, s->kw, s->slot_idx, s->batch_win, s->k, s->stream, s->k1_ticket));
            s->slots_init = s->win_zero = true;
        }
        fresh = !s->slots_init;
        s->win_zero = false;  // until this batch's resolve is enqueued
    }
    if (s->cfg.kind == RSV_KIND_DISTINCT) {
        // large batches publish the merged set speculatively (distinct_spec_target: set mode behind
        // its last merge, ordered mode behind the scheduled pass) -- only where a publication can
        // happen at all (a coherent result buffer of k keys); other samplers (huge k, device-only
        // consumers) keep the result buffer lazy
        if ((int64_t)s->k * s->kw <= kPublishMaxBytes && n >= distinct_spec_min(s->distinct)) {
            if (rsv_status st = ensure_result_buffer(s)) return st;
            if (s->result_publish) distinct_spec_target(s->distinct, s->result_dev, s->result_flag_dev, &s->result_gen);
        }
        int rc = distinct_sample_device(s->distinct, keys, hashes, n, s->stream);
        uint32_t gen = 0;
        const bool published = distinct_spec_take(s->distinct, &gen);
        if (rc != RSV_OK) return (rsv_status)rc;
        s->pub_valid = published;  // result() waits for it instead of publishing
        if (published) {
            s->pub_ops = s->ops;
            s->pub_gen = gen;
        }
    } else if (s->cfg.engine == RSV_ENGINE_JAVA_L) {
        s->ev_pos_h.clear();
        s->ev_slot_h.clear();
        s->algo_l.events(base, n, s->ev_pos_h, s->ev_slot_h);
        const int64_t ne = (int64_t)s->ev_pos_h.size();
        if (ne) {
            if (rsv_status st = ensure_events(s, ne)) return st;
            const void* pos_src = s->ev_pos_h.data();
            const void* slot_src = s->ev_slot_h.data();
            if (stage_b >= 0) {  // pinned: stage_b's previous flush has completed (stage_slow waited for it)
                if (s->stage_ev_cap[stage_b] < ne) {
                    const int64_t cap = std::max<int64_t>(ne, 2 * s->stage_ev_cap[stage_b]);
                    pool_host_free(s->stage_ev_pos[stage_b]);
                    pool_host_free(s->stage_ev_slot[stage_b]);
                    s->stage_ev_pos[stage_b] = nullptr;
                    s->stage_ev_slot[stage_b] = nullptr;
                    s->stage_ev_cap[stage_b] = 0;
                    RSV_HIP_TRY(pool_host_alloc((void**)&s->stage_ev_pos[stage_b], cap * 8, hipHostMallocDefault));
                    RSV_HIP_TRY(pool_host_alloc((void**)&s->stage_ev_slot[stage_b], cap * 4, hipHostMallocDefault));
                    s->stage_ev_cap[stage_b] = cap;
                }
                memcpy(s->stage_ev_pos[stage_b], pos_src, ne * 8);
                memcpy(s->stage_ev_slot[stage_b], slot_src, ne * 4);
                pos_src = s->stage_ev_pos[stage_b];
                slot_src = s->stage_ev_slot[stage_b];
            }
            RSV_HIP_TRY(hipMemcpyAsync(s->ev_pos_d, pos_src, ne * 8, hipMemcpyHostToDevice, s->stream));
            RSV_HIP_TRY(hipMemcpyAsync(s->ev_slot_d, slot_src, ne * 4, hipMemcpyHostToDevice, s->stream));
            const bool pm = prof_begin(s, s->stream);
            RSV_HIP_TRY(launch_replay_events(s->ev_pos_d, s->ev_slot_d, ne, s->k, s->batch_win, s->stream));
            prof_end(s, s->stream, pm);
        }
        if (rsv_status st = resolve_batch(s, keys, base, n, fresh)) return st;
        // pageable host event vectors are reused by the next batch (a staged batch's pinned copies
        // are released by its stage_free event instead)
        if (ne && stage_b < 0) RSV_HIP_TRY(sync_stream(s));
    } else {
        const DrawParams dp{s->cfg.seed, s->cfg.stream_id};
        const uint64_t lo = std::max<uint64_t>((uint64_t)base, s->k), hi = (uint64_t)(base + n);
        // Fused (one dispatch, the last workgroup resolves) for batches up to 2^27 draws, where the
        // saved dispatch is a visible share of the step; above that the two-dispatch form is faster
        // (C2: 112.5 vs 114.0 us per step, r02aa: the fused tail runs on one workgroup of the
        // otherwise idle chip, while resolve_publish_kernel's dispatch overlaps K1's drain; round 6,
        // the two-group K1: 96.7 vs 83.0-83.7 us per launch, 97.2 vs 88.6-89.5 us per step --
        // every workgroup's ticket wait holds its slot, profiles/r06/bench_k1_fuse_ab.jsonl).
        // RSV_K1_FUSE=0 / =1 forces either form (A/B measurements).
        static const int fuse_mode = [] {
            const char* e = std::getenv("RSV_K1_FUSE");
            return e && e[0] == '0' ? 0 : e && e[0] == '1' ? 1 : 2;
        }();
        constexpr uint64_t kFuseMaxDraws = 1ull << 27;
        const bool fuse = (fuse_mode == 1 || (fuse_mode == 2 && (hi <= lo || hi - lo <= kFuseMaxDraws))) &&
                          k1_fused_ok(lo, hi, s->k, s->kw);
        if (fuse) {
            if (rsv_status st = ensure_result_buffer(s)) return st;
        }
        if (fuse && s->result_publish) {
            // one dispatch: K1, then the last workgroup resolves and publishes (resolve_batch's form)
            const uint32_t gen = ++s->result_gen;
            const int64_t m = std::min<int64_t>(base + n, (int64_t)s->k);
            const bool pm = prof_begin(s, s->stream);
            RSV_HIP_TRY(launch_k1_resolve_publish(dp, s->k, lo, hi, s->batch_win, s->k1_ticket, keys, s->kw, base, n,
                                                  s->slot_key, s->slot_idx, fresh, m, s->result_dev,
                                                  s->result_flag_dev, gen, s->stream));
            prof_end(s, s->stream, pm);
            s->pub_ops = s->ops;
            s->pub_gen = gen;
            s->pub_valid = true;
        } else {
            const bool pm = prof_begin(s, s->stream);
            RSV_HIP_TRY(launch_k1_last_writer(dp, s->k, lo, hi, s->batch_win, s->stream));
            prof_end(s, s->stream, pm);
            if (s->rstream) {  // the resolve + publication forked onto the resolve stream (see there)
                if (!s->side_fork) RSV_HIP_TRY(pool_event(&s->side_fork, hipEventDisableTiming));
                if (!s->side_join) RSV_HIP_TRY(pool_event(&s->side_join, hipEventDisableTiming));
                RSV_HIP_TRY(hipEventRecord(s->side_fork, s->stream));
                RSV_HIP_TRY(hipStreamWaitEvent(s->rstream, s->side_fork, 0));
                if (rsv_status st = resolve_batch(s, keys, base, n, fresh, s->rstream)) return st;
                RSV_HIP_TRY(hipEventRecord(s->side_join, s->rstream));
                s->side_pending = true;
            } else if (rsv_status st = resolve_batch(s, keys, base, n, fresh)) {
                return st;
            }
        }
    }
    if (s->cfg.kind == RSV_KIND_ELEMENTS) s->slots_init = s->win_zero = true;
    s->count = base + n;
    return RSV_OK;
}

rsv_status ensure_chunk(rsv_sampler* s) {
    if (s->chunk_d) return RSV_OK;
    RSV_HIP_TRY(pool_device_alloc(&s->chunk_d, kChunkKeys * s->kw));
    if (s->cfg.kind == RSV_KIND_DISTINCT && s->hash_kind == kHashPrecomputed)
        RSV_HIP_TRY(pool_device_alloc((void**)&s->chunk_hash_d, kChunkKeys * 8));
    s->chunk_cap = kChunkKeys;
    return RSV_OK;
}

// Wait until a kernel has published `gen` into the coherent host word `flag` (acquire).  Spins for
// up to ~2 ms -- the K1 pass of a 1e9-element batch still in flight ahead of it is ~0.1 ms -- then
// falls back to a blocking stream synchronize, which also reports a failed kernel instead of
// waiting forever.
rsv_status spin_flag(rsv_sampler* s, const uint32_t* flag, uint32_t gen, const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == gen) return RSV_OK;
        __builtin_ia32_pause();
        if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
    }
    RSV_HIP_TRY(sync_stream(s));
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == gen) return RSV_OK;
    return fail(RSV_E_DEVICE, std::string(what) + " flag not set after stream synchronize");
}

// One index-only batch of n elements at global indices [count, count + n) (the reference's
// sampleIndexed, Sampler.scala:261-273, which reads only the elements it keeps): K1 (philox_r) or
// the host's Algorithm-L events (java_l) over the indices alone, the resolve into slot_idx, and per
// slot the batch offset of its new element (-1: unchanged) in host memory, *offs_out (k entries,
// valid until the handle's next index-only batch).  No key is read.  The caller then supplies the
// winners' keys (fill_gathered) or undoes the batch (rsv_abort_indexed).
rsv_status index_batch(rsv_sampler* s, int64_t n, const int64_t** offs_out) {
    if (!s->idx_offs_d) RSV_HIP_TRY(pool_device_alloc((void**)&s->idx_offs_d, (size_t)s->k * 8));
    if (!s->idx_bak_d) RSV_HIP_TRY(pool_device_alloc((void**)&s->idx_bak_d, (size_t)s->k * 8));
    const bool publish = resolve_indices_publish_ok(s->k);
    if (!s->offs_h) {
        if (publish) {  // k offsets + one 64-B flag line, coherent and mapped
            const size_t flag_off = ((size_t)s->k * 8 + 63) & ~(size_t)63;
            RSV_HIP_TRY(pool_host_alloc((void**)&s->offs_h, flag_off + 64, hipHostMallocCoherent | hipHostMallocMapped));
            void* dev = nullptr;
            RSV_HIP_TRY(hipHostGetDevicePointer(&dev, s->offs_h, 0));
            s->offs_dev = (int64_t*)dev;
            s->offs_flag = (uint32_t*)((uint8_t*)s->offs_h + flag_off);
            s->offs_flag_dev = (uint32_t*)((uint8_t*)dev + flag_off);
            *s->offs_flag = s->offs_gen;
        } else {
            RSV_HIP_TRY(pool_host_alloc((void**)&s->offs_h, (size_t)s->k * 8, hipHostMallocDefault));
        }
    }
    touch(s);
    const int64_t base = s->count;
    if (!s->win_zero) {  // never-used block: full init
        RSV_HIP_TRY(launch_init_slots(s->slot_key, s->kw, s->slot_idx, s->batch_win, s->k, s->stream, s->k1_ticket));
        s->slots_init = s->win_zero = true;
    }
    const bool fresh = !s->slots_init;
    s->win_zero = false;
    // the state rsv_abort_indexed restores (a throwing `map` leaves the slots consistent)
    s->idx_fresh = fresh;
    s->idx_base = base;
    s->idx_algo_l = s->algo_l;
    if (!fresh)
        RSV_HIP_TRY(hipMemcpyAsync(s->idx_bak_d, s->slot_idx, (size_t)s->k * 8, hipMemcpyDeviceToDevice, s->stream));
    if (s->cfg.engine == RSV_ENGINE_JAVA_L) {  // the reference's own events (S:261-273 skips by them)
        s->ev_pos_h.clear();
        s->ev_slot_h.clear();
        s->algo_l.events(base, n, s->ev_pos_h, s->ev_slot_h);
        const int64_t ne = (int64_t)s->ev_pos_h.size();
        if (ne) {
            if (rsv_status st = ensure_events(s, ne)) return st;
            RSV_HIP_TRY(hipMemcpyAsync(s->ev_pos_d, s->ev_pos_h.data(), ne * 8, hipMemcpyHostToDevice, s->stream));
            RSV_HIP_TRY(hipMemcpyAsync(s->ev_slot_d, s->ev_slot_h.data(), ne * 4, hipMemcpyHostToDevice, s->stream));
            const bool pm = prof_begin(s, s->stream);
            RSV_HIP_TRY(launch_replay_events(s->ev_pos_d, s->ev_slot_d, ne, s->k, s->batch_win, s->stream));
            prof_end(s, s->stream, pm);
        }
    } else {
        const DrawParams dp{s->cfg.seed, s->cfg.stream_id};
        const uint64_t lo = std::max<uint64_t>((uint64_t)base, s->k), hi = (uint64_t)(base + n);
        const bool pm = prof_begin(s, s->stream);
        RSV_HIP_TRY(launch_k1_last_writer(dp, s->k, lo, hi, s->batch_win, s->stream));
        prof_end(s, s->stream, pm);
    }
    if (publish) {  // the offsets straight into coherent host memory + flag: no copy, no stream sync
        const uint32_t gen = ++s->offs_gen;
        RSV_HIP_TRY(launch_resolve_indices_publish(base, n, s->k, s->batch_win, s->slot_idx, fresh, s->slot_key, s->kw,
                                                   s->idx_offs_d, s->offs_dev, s->offs_flag_dev, gen, s->stream));
        // the event vectors above were read by copies that precede the flag in stream order
        if (rsv_status st = spin_flag(s, s->offs_flag, gen, "index batch")) return st;
        if (s->offs_gen == gen) s->ops_done = s->ops;  // the publication was this handle's last work
    } else {
        RSV_HIP_TRY(launch_resolve_indices(base, n, s->k, s->batch_win, s->slot_idx, fresh, s->slot_key, s->kw,
                                           s->idx_offs_d, s->stream));
        RSV_HIP_TRY(hipMemcpyAsync(s->offs_h, s->idx_offs_d, (size_t)s->k * 8, hipMemcpyDeviceToHost, s->stream));
        RSV_HIP_TRY(sync_stream(s));
    }
    s->slots_init = s->win_zero = true;
    s->pub_valid = false;
    s->count = base + n;
    *offs_out = s->offs_h;
    return RSV_OK;
}

rsv_status ensure_gather(rsv_sampler* s) {
    if (s->gath_h) return RSV_OK;
    RSV_HIP_TRY(pool_host_alloc((void**)&s->gath_h, (size_t)s->k * s->kw, hipHostMallocCoherent | hipHostMallocMapped));
    RSV_HIP_TRY(hipHostGetDevicePointer(&s->gath_dev, s->gath_h, 0));
    return RSV_OK;
}

// The winners' keys, gathered by the host into gath_h (slot order; only the slots index_batch
// changed are read), into the reservoir: one kernel reading them across PCIe, which for small
// reservoirs also publishes the result -- enqueued, no host wait.  The gather buffer is rewritten
// only after the handle's next index_batch has waited for its own publication, which follows this
// kernel in stream order.
rsv_status fill_gathered(rsv_sampler* s) {
    touch(s);
    if (fill_slots_publish_ok(s->k, s->kw)) {
        if (rsv_status st = ensure_result_buffer(s)) return st;
        if (s->result_publish) {
            const uint32_t gen = ++s->result_gen;
            const int64_t m = std::min<int64_t>(s->count, (int64_t)s->k);
            RSV_HIP_TRY(launch_fill_slots_publish(s->idx_offs_d, s->gath_dev, s->k, s->kw, s->slot_key, m,
                                                  s->result_dev, s->result_flag_dev, gen, s->stream));
            s->pub_ops = s->ops;
            s->pub_gen = gen;
            s->pub_valid = true;
            s->keys_owed = false;
            return RSV_OK;
        }
    }
    RSV_HIP_TRY(launch_fill_slots(s->idx_offs_d, s->gath_dev, s->k, s->kw, s->slot_key, s->stream));
    s->pub_valid = false;
    s->keys_owed = false;
    return RSV_OK;
}

// A host batch of an ELEMENTS sampler moves only its winners: the batch is sampled by index
// (index_batch), the host copies the <= k winning keys out of the caller's buffer, and they reach
// the slots across PCIe (fill_gathered) -- 8 B per winner instead of 8 B per element.
rsv_status host_batch_elements(rsv_sampler* s, const void* keys, int64_t n) {
    const int64_t* offs = nullptr;
    if (rsv_status st = index_batch(s, n, &offs)) return st;
    if (rsv_status st = ensure_gather(s)) return st;
    const uint8_t* src = (const uint8_t*)keys;
    const size_t kw = (size_t)s->kw;
    if (kw == 8) {
        for (uint32_t j = 0; j < s->k; ++j)
            if (offs[j] >= 0) memcpy(s->gath_h + (size_t)j * 8, src + (size_t)offs[j] * 8, 8);
    } else {
        for (uint32_t j = 0; j < s->k; ++j)
            if (offs[j] >= 0) memcpy(s->gath_h + (size_t)j * kw, src + (size_t)offs[j] * kw, kw);
    }
    return fill_gathered(s);
}

rsv_status process_host_batch(rsv_sampler* s, const void* keys, const int64_t* hashes, int64_t n) {
    if (n <= 0) return RSV_OK;
    if (s->cfg.kind == RSV_KIND_ELEMENTS) return host_batch_elements(s, keys, n);
    if (rsv_status st = ensure_chunk(s)) return st;
    join_side(s);  // (a forked resolve reads its batch's keys; none for DISTINCT, kept for symmetry)
    for (int64_t off = 0; off < n; off += s->chunk_cap) {
        const int64_t c = std::min(s->chunk_cap, n - off);
        RSV_HIP_TRY(hipMemcpyAsync(s->chunk_d, (const uint8_t*)keys + off * s->kw, c * s->kw,
                                   hipMemcpyHostToDevice, s->stream));
        if (s->chunk_hash_d && hashes)
            RSV_HIP_TRY(hipMemcpyAsync(s->chunk_hash_d, hashes + off, c * 8, hipMemcpyHostToDevice, s->stream));
        if (rsv_status st = process_device_batch(s, s->chunk_d, s->chunk_hash_d, c)) return st;
    }
    // the caller may reuse its buffer after return (ownership stays with the caller)
    RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

// Flush the current staging buffer: H2D into the device chunk, record "buffer free", launch the
// batch's kernels -- all stream-ordered, no host wait -- and switch to the other buffer.
// Expected number of slots a batch of n elements at global indices [base, base + n) changes: the
// fill of slots [base, k), then ~k/(i+1) evictions per index i >= k (Algorithm R; Algorithm L has
// the same expectation), at most k.
double expected_changes(const rsv_sampler* s, int64_t base, int64_t n) {
    const double k = s->k;
    const double fill = std::min<double>(std::max<double>(k - (double)base, 0.0), (double)n);
    const double lo = std::max<double>((double)base, k), hi = (double)base + (double)n;
    const double ev = hi > lo ? k * std::log(hi / lo) : 0.0;
    return std::min(fill + ev, std::min<double>((double)n, k));
}

// A staged batch of an ELEMENTS sampler is sampled in place when its expected winners are few
// against its size: the resolve reads the <= k winning keys straight from the pinned staging
// buffer across PCIe instead of a DMA of the whole batch.  RSV_STAGE_ZC_RATIO (default 16): in
// place when expected changes x ratio <= n; 0 = always copy.
bool stage_in_place(const rsv_sampler* s, int64_t n) {
    static const double ratio = [] {
        const char* e = std::getenv("RSV_STAGE_ZC_RATIO");
        return e ? std::atof(e) : 16.0;
    }();
    if (s->cfg.kind != RSV_KIND_ELEMENTS || ratio <= 0) return false;
    return expected_changes(s, s->count, n) * ratio <= (double)n;
}

rsv_status flush_stage(rsv_sampler* s) {
    if (s->stage_n == 0) return RSV_OK;
    const int64_t n = s->stage_n;
    const int b = s->stage_cur;
    s->stage_n = 0;
    if (stage_in_place(s, n)) {
        s->stage_pending[b] = true;
        s->stage_cur = b ^ 1;
        if (rsv_status st = process_device_batch(s, s->stage_dev[b], nullptr, n, b)) return st;
        // the buffer is free once the resolve that reads it has run (on the resolve stream if forked)
        RSV_HIP_TRY(hipEventRecord(s->stage_free[b], s->side_pending ? s->rstream : s->stream));
        return RSV_OK;
    }
    if (rsv_status st = ensure_chunk(s)) return st;
    join_side(s);  // a forked resolve may still read the chunk's previous batch
    RSV_HIP_TRY(hipMemcpyAsync(s->chunk_d, s->stage_h[b], n * s->kw, hipMemcpyHostToDevice, s->stream));
    if (s->chunk_hash_d && s->stage_hash_h[b])
        RSV_HIP_TRY(hipMemcpyAsync(s->chunk_hash_d, s->stage_hash_h[b], n * 8, hipMemcpyHostToDevice, s->stream));
    s->stage_pending[b] = true;
    s->stage_cur = b ^ 1;
    if (s->cfg.kind == RSV_KIND_ELEMENTS && s->cfg.engine == RSV_ENGINE_JAVA_L) {
        // the batch's events travel from stage b's pinned event buffers: free after their copies
        if (rsv_status st = process_device_batch(s, s->chunk_d, nullptr, n, b)) return st;
        RSV_HIP_TRY(hipEventRecord(s->stage_free[b], s->stream));
        return RSV_OK;
    }
    RSV_HIP_TRY(hipEventRecord(s->stage_free[b], s->stream));
    return process_device_batch(s, s->chunk_d, s->chunk_hash_d, n);
}

void free_all(rsv_sampler* s) {
    // callers have synchronized the stream: nothing queued touches these any more
    if (s->slots && s->win_zero && give_clean_slots(s->slots, s->k, s->kw, s->device)) s->slots = nullptr;
    void* ds[] = {s->slots, s->ev_pos_d, s->ev_slot_d, s->chunk_d, s->chunk_hash_d, s->idx_offs_d, s->idx_bak_d};
    for (void* p : ds) pool_device_free(p);
    for (int b = 0; b < 2; ++b) {
        pool_host_free(s->stage_h[b]);
        pool_host_free(s->stage_hash_h[b]);
        pool_host_free(s->stage_ev_pos[b]);
        pool_host_free(s->stage_ev_slot[b]);
        pool_release_event(s->device, s->stage_free[b], hipEventDisableTiming);
    }
    pool_host_free(s->result_h);
    pool_host_free(s->offs_h);
    pool_host_free(s->gath_h);
    // the handover record has completed: the stream waiting on it was synchronized, or its
    // publication seen, before this
    if (s->handover) pool_release_event(s->device, s->handover, hipEventDisableTiming);
    if (s->side_fork) pool_release_event(s->device, s->side_fork, hipEventDisableTiming);
    if (s->side_join) pool_release_event(s->device, s->side_join, hipEventDisableTiming);
    if (s->distinct) distinct_destroy(s->distinct);
    if (s->stream && s->own_stream) pool_release_stream(s->device, s->stream);
}

int resolve_hash_kind(int32_t hk, int kw) {
    switch (hk) {
    case RSV_HASH_IDENTITY: return kHashIdentity;
    case RSV_HASH_JAVA_LONG: return kHashJavaLong;
    case RSV_HASH_JAVA_INT: return kHashJavaInt;
    case RSV_HASH_PRECOMPUTED: return kHashPrecomputed;
    default:  // B#hashCode (Sampler.scala:75): Integer / Long / java.util.UUID
        return kw == 4 ? kHashJavaInt : kw == 16 ? kHashUuid : kHashJavaLong;
    }
}

}  // namespace

extern "C" {

int32_t rsv_abi_version(void) { return RSV_ABI_VERSION; }

const char* rsv_last_error(void) { return g_last_error.c_str(); }

const char* rsv_status_string(rsv_status s) {
    switch (s) {
    case RSV_OK: return "ok";
    case RSV_E_ILLEGAL_ARGUMENT: return "illegal argument";
    case RSV_E_ILLEGAL_STATE: return "illegal state";
    case RSV_E_NULL_POINTER: return "null pointer";
    case RSV_E_DEVICE: return "device error";
    case RSV_E_OUT_OF_MEMORY: return "out of memory";
    case RSV_E_UNSUPPORTED: return "unsupported";
    }
    return "unknown status";
}

rsv_status rsv_config_init(rsv_config* cfg) {
    if (!cfg) return fail(RSV_E_NULL_POINTER, "config is NULL");
    memset(cfg, 0, sizeof(*cfg));
    cfg->struct_size = sizeof(rsv_config);
    cfg->kind = RSV_KIND_ELEMENTS;
    cfg->max_sample_size = 1;
    cfg->key_width = 8;
    cfg->engine = RSV_ENGINE_PHILOX_R;
    cfg->hash_kind = RSV_HASH_DEFAULT;
    cfg->device = -1;
    return RSV_OK;
}

rsv_status rsv_create(const rsv_config* cfg, rsv_sampler** out) {
    if (!cfg || !out) return fail(RSV_E_NULL_POINTER, "config/out is NULL");
    *out = nullptr;
    if (cfg->struct_size != sizeof(rsv_config))
        return fail(RSV_E_ILLEGAL_ARGUMENT, "rsv_config.struct_size mismatch (ABI version)");
    // validateSharedParams, Sampler.scala:79-83
    if (cfg->max_sample_size > kMaxSize) return fail(RSV_E_ILLEGAL_ARGUMENT, "maxSampleSize exceeds VM limit");
    if (cfg->max_sample_size <= 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "maxSampleSize must be positive");
    if (cfg->kind != RSV_KIND_ELEMENTS && cfg->kind != RSV_KIND_DISTINCT)
        return fail(RSV_E_ILLEGAL_ARGUMENT, "unknown sampler kind");
    // key widths: Int (4), Long (8), fixed-width byte keys (a multiple of 8 in 16..256: UUID = 16).
    // Any other width is a request this build does not implement (the reference has no width).
    const bool wide = cfg->key_width > 8 && cfg->key_width <= 256 && cfg->key_width % 8 == 0;
    if (cfg->key_width != 4 && cfg->key_width != 8 && !wide)
        return fail(RSV_E_UNSUPPORTED, "key_width must be 4, 8 or a multiple of 8 in 16..256 bytes");
    // byte keys have no Long/Int hashCode: DISTINCT takes the caller's hash (PRECOMPUTED) or, for
    // 16-byte keys, java.util.UUID.hashCode (DEFAULT)
    if (wide && cfg->kind == RSV_KIND_DISTINCT && cfg->hash_kind != RSV_HASH_PRECOMPUTED &&
        !(cfg->hash_kind == RSV_HASH_DEFAULT && cfg->key_width == 16))
        return fail(RSV_E_UNSUPPORTED, "DISTINCT over byte keys needs RSV_HASH_PRECOMPUTED (or RSV_HASH_DEFAULT = "
                                       "java.util.UUID.hashCode for 16-byte keys)");
    if (cfg->kind == RSV_KIND_ELEMENTS && cfg->engine != RSV_ENGINE_PHILOX_R && cfg->engine != RSV_ENGINE_JAVA_L)
        return fail(RSV_E_ILLEGAL_ARGUMENT, "unknown engine");
    if (cfg->hash_kind < RSV_HASH_DEFAULT || cfg->hash_kind > RSV_HASH_PRECOMPUTED)
        return fail(RSV_E_ILLEGAL_ARGUMENT, "unknown hash kind");
    if (cfg->distinct_order < RSV_DISTINCT_AUTO || cfg->distinct_order > RSV_DISTINCT_ORDERED)
        return fail(RSV_E_ILLEGAL_ARGUMENT, "unknown distinct order");

    rsv_sampler* s = new rsv_sampler();
    s->cfg = *cfg;
    s->kw = cfg->key_width;
    s->k = (uint32_t)cfg->max_sample_size;
    int dev = cfg->device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    s->device = dev;
    DeviceGuard g(dev);
    auto bail = [&](rsv_status st, const std::string& msg) {
        free_all(s);
        delete s;
        return fail(st, msg);
    };
    s->timer.device = dev;
    hipError_t e = pool_stream(&s->stream);
    if (e != hipSuccess) return bail(RSV_E_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    s->own_stream = true;
    if (cfg->kind == RSV_KIND_ELEMENTS) {
        const size_t k = s->k;
        s->slots = take_clean_slots(s->k, s->kw, dev);
        if (s->slots)
            s->win_zero = true;
        else
            e = pool_device_alloc(&s->slots, k * 16 + ((k * s->kw + 7) & ~(size_t)7) + 8);
        if (e == hipSuccess) {
            s->batch_win = (unsigned long long*)s->slots;
            s->slot_idx = (int64_t*)((uint8_t*)s->slots + k * 8);
            s->slot_key = (uint8_t*)s->slots + k * 16;
            s->k1_ticket = (uint32_t*)((uint8_t*)s->slots + k * 16 + ((k * s->kw + 7) & ~(size_t)7));
        }
        if (e != hipSuccess)
            return bail(e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE,
                        std::string("allocating reservoir: ") + hipGetErrorString(e));
        if (cfg->engine == RSV_ENGINE_JAVA_L) s->algo_l.init((int32_t)s->k, (int64_t)cfg->seed);
    } else {
        // RandomValues r0, r1 (Sampler.scala:385-388) from java.util.Random(seed)
        JavaRandom r;
        r.init((int64_t)cfg->seed);
        const int64_t r0 = r.next_long(), r1 = r.next_long();
        s->hash_kind = resolve_hash_kind(cfg->hash_kind, s->kw);
        int st = RSV_OK;
        bool ordered;
        switch (cfg->distinct_order) {
        case RSV_DISTINCT_SET: ordered = false; break;
        case RSV_DISTINCT_ORDERED: ordered = true; break;
        default:  // hashes that may collide
            ordered = s->hash_kind == kHashJavaLong || s->hash_kind == kHashPrecomputed || s->hash_kind == kHashUuid;
        }
        s->distinct = distinct_create((int32_t)s->k, s->kw, s->hash_kind, r0, r1, ordered, &st);
        if (!s->distinct) {
            std::string msg = g_last_error;
            return bail((rsv_status)st, msg);
        }
        distinct_set_timer(s->distinct, &s->timer);
    }
    *out = s;
    return RSV_OK;
}

void rsv_destroy(rsv_sampler* s) {
    if (!s) return;
    DeviceGuard g(s->device);
    // the buffers go back to the pool: nothing this handle enqueued may still touch them.  On a
    // caller stream whose last group of work was a publication the host has seen, that holds
    // already (the flag store is the last memory operation of that group).
    if (s->stream && (s->own_stream || s->ops != s->ops_done)) {
        join_side(s);
        (void)hipStreamSynchronize(s->stream);
    } else if (s->side_pending && s->rstream) {
        // the publication was seen (its flag store is the resolve's last memory operation): only the
        // events and buffers remain, and they outlive the queued work by the join below
        (void)hipEventSynchronize(s->side_join);
    }
    free_all(s);
    delete s;
}

// Slow part of rsv_sample: (re)arm a staging buffer, or flush a full one.  Runs once per batch.
static rsv_status stage_slow(rsv_sampler* s, bool pre) {
    DeviceGuard g(s->device);
    if (s->stage_n == s->stage_cap && s->stage_cap) {
        if (rsv_status st = flush_stage(s)) return st;
    }
    if (!s->stage_h[0]) {
        for (int b = 0; b < 2; ++b) {
            // coherent + mapped: a winners-only flush's resolve reads the keys in place (flush_stage)
            RSV_HIP_TRY(pool_host_alloc((void**)&s->stage_h[b], kStageKeys * s->kw,
                                        hipHostMallocCoherent | hipHostMallocMapped));
            RSV_HIP_TRY(hipHostGetDevicePointer(&s->stage_dev[b], s->stage_h[b], 0));
            if (pre) RSV_HIP_TRY(pool_host_alloc((void**)&s->stage_hash_h[b], kStageKeys * 8, hipHostMallocDefault));
            RSV_HIP_TRY(pool_event(&s->stage_free[b], hipEventDisableTiming));
        }
        s->stage_cap = kStageKeys;
    }
    const int b = s->stage_cur;
    if (s->stage_n == 0 && s->stage_pending[b]) {  // its previous batch's H2D must have read it
        RSV_HIP_TRY(hipEventSynchronize(s->stage_free[b]));
        s->stage_pending[b] = false;
    }
    return RSV_OK;
}

rsv_status rsv_sample(rsv_sampler* s, const void* key, const int64_t* hash) {
    // per-element hot path (the akka operator calls this per element): no HIP call here
    if (!s || !s->open || s->keys_external) return check_keyed(s);
    if (!key) return fail(RSV_E_NULL_POINTER, "key is NULL");
    const bool pre = s->hash_kind == kHashPrecomputed && s->cfg.kind == RSV_KIND_DISTINCT;
    if (pre && !hash) return fail(RSV_E_NULL_POINTER, "hash is NULL for RSV_HASH_PRECOMPUTED");
    if (s->stage_n == 0 || s->stage_n == s->stage_cap) {
        if (rsv_status st = stage_slow(s, pre)) return st;
    }
    const int b = s->stage_cur;
    if (s->kw == 8) memcpy(s->stage_h[b] + s->stage_n * 8, key, 8);
    else if (s->kw == 4) memcpy(s->stage_h[b] + s->stage_n * 4, key, 4);
    else memcpy(s->stage_h[b] + s->stage_n * s->kw, key, (size_t)s->kw);
    if (pre) s->stage_hash_h[b][s->stage_n] = *hash;
    ++s->stage_n;
    return RSV_OK;
}

rsv_status rsv_stage_acquire(rsv_sampler* s, void** keys_out, int64_t** hashes_out, int64_t* capacity) {
    if (!s || !s->open || s->keys_external) return check_keyed(s);
    if (!keys_out || !capacity) return fail(RSV_E_NULL_POINTER, "keys_out/capacity is NULL");
    const bool pre = s->hash_kind == kHashPrecomputed && s->cfg.kind == RSV_KIND_DISTINCT;
    if (s->stage_n == 0 || s->stage_n == s->stage_cap) {
        if (rsv_status st = stage_slow(s, pre)) return st;
    }
    const int b = s->stage_cur;
    *keys_out = s->stage_h[b] + s->stage_n * s->kw;
    if (hashes_out) *hashes_out = pre ? s->stage_hash_h[b] + s->stage_n : nullptr;
    *capacity = s->stage_cap - s->stage_n;
    return RSV_OK;
}

rsv_status rsv_stage_commit(rsv_sampler* s, int64_t n) {
    if (!s || !s->open || s->keys_external) return check_keyed(s);
    if (n < 0 || n > s->stage_cap - s->stage_n)
        return fail(RSV_E_ILLEGAL_ARGUMENT, "commit exceeds the acquired staging capacity");
    s->stage_n += n;
    if (s->stage_n == s->stage_cap && n > 0) {  // full: start its flush now, overlapping the next fill
        DeviceGuard g(s->device);
        if (rsv_status st = flush_stage(s)) return st;
    }
    return RSV_OK;
}

rsv_status rsv_sample_batch(rsv_sampler* s, const void* keys, int64_t n, int32_t mem, const int64_t* hashes) {
    if (rsv_status st = check_keyed(s)) return st;
    if (n < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative batch size");
    if (n == 0) return RSV_OK;
    if (!keys) return fail(RSV_E_NULL_POINTER, "keys is NULL");
    const bool pre = s->cfg.kind == RSV_KIND_DISTINCT && s->hash_kind == kHashPrecomputed;
    if (pre && !hashes) return fail(RSV_E_NULL_POINTER, "hashes is NULL for RSV_HASH_PRECOMPUTED");
    DeviceGuard g(s->device);
    if (rsv_status st = flush_stage(s)) return st;  // keep global index order
    if (mem == RSV_MEM_DEVICE) return process_device_batch(s, keys, pre ? hashes : nullptr, n);
    if (mem == RSV_MEM_HOST) return process_host_batch(s, keys, pre ? hashes : nullptr, n);
    return fail(RSV_E_ILLEGAL_ARGUMENT, "mem must be RSV_MEM_HOST or RSV_MEM_DEVICE");
}

rsv_status rsv_sample_indexed(rsv_sampler* s, int64_t n, int64_t* slot_offsets_host) {
    if (rsv_status st = check_open(s)) return st;
    if (s->cfg.kind != RSV_KIND_ELEMENTS)
        return fail(RSV_E_UNSUPPORTED, "rsv_sample_indexed needs an ELEMENTS sampler (distinct maps every element, S:50)");
    if (n < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative batch size");
    if (!slot_offsets_host) return fail(RSV_E_NULL_POINTER, "slot_offsets_host is NULL");
    if (n == 0) {
        for (uint32_t j = 0; j < s->k; ++j) slot_offsets_host[j] = -1;
        return RSV_OK;
    }
    DeviceGuard g(s->device);
    if (rsv_status st = flush_stage(s)) return st;  // keep global index order
    const int64_t* offs = nullptr;
    if (rsv_status st = index_batch(s, n, &offs)) return st;
    memcpy(slot_offsets_host, offs, (size_t)s->k * 8);
    s->keys_owed = true;
    return RSV_OK;
}

rsv_status rsv_fill_slots(rsv_sampler* s, const void* keys_host) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    if (!s->keys_owed) return fail(RSV_E_ILLEGAL_STATE, "rsv_fill_slots without a pending rsv_sample_indexed");
    if (s->keys_external)
        return fail(RSV_E_ILLEGAL_STATE, "the slots hold no keys (rsv_commit_indexed): commit or abort the batch");
    if (!keys_host) return fail(RSV_E_NULL_POINTER, "keys_host is NULL");
    DeviceGuard g(s->device);
    if (rsv_status st = ensure_gather(s)) return st;
    // the changed slots' keys into the pinned gather buffer: the caller's buffer is theirs again on
    // return, and no copy or host wait follows
    const int64_t* offs = s->offs_h;
    const size_t kw = (size_t)s->kw;
    const uint8_t* src = (const uint8_t*)keys_host;
    for (uint32_t j = 0; j < s->k; ++j)
        if (offs[j] >= 0) memcpy(s->gath_h + (size_t)j * kw, src + (size_t)j * kw, kw);
    return fill_gathered(s);
}

rsv_status rsv_abort_indexed(rsv_sampler* s) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    if (!s->keys_owed) return fail(RSV_E_ILLEGAL_STATE, "rsv_abort_indexed without a pending rsv_sample_indexed");
    DeviceGuard g(s->device);
    touch(s);
    if (s->idx_fresh)  // the slots were never initialised before the batch: empty them again
        RSV_HIP_TRY(launch_init_slots(s->slot_key, s->kw, s->slot_idx, s->batch_win, s->k, s->stream, s->k1_ticket));
    else  // the changed slots still hold their old keys: their old indices make them whole again
        RSV_HIP_TRY(hipMemcpyAsync(s->slot_idx, s->idx_bak_d, (size_t)s->k * 8, hipMemcpyDeviceToDevice, s->stream));
    RSV_HIP_TRY(sync_stream(s));
    s->slots_init = s->win_zero = true;
    s->pub_valid = false;
    s->count = s->idx_base;
    s->algo_l = s->idx_algo_l;
    s->keys_owed = false;
    return RSV_OK;
}

rsv_status rsv_commit_indexed(rsv_sampler* s) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    if (!s->keys_owed) return fail(RSV_E_ILLEGAL_STATE, "rsv_commit_indexed without a pending rsv_sample_indexed");
    // the slot indices are final (index_batch); the keys stay with the caller
    s->keys_owed = false;
    s->keys_external = true;
    s->pub_valid = false;
    return RSV_OK;
}

// Wait until a publication kernel has stored `gen` in the result flag (spin_flag)
static rsv_status wait_flag(rsv_sampler* s, uint32_t gen) { return spin_flag(s, s->result_flag, gen, "result publish"); }

static rsv_status result_impl(rsv_sampler* s, void* out, int64_t cap, int64_t* out_n, bool device_out,
                              bool take = false) {
    if (rsv_status st = check_keyed(s)) return st;
    if (!out_n) return fail(RSV_E_NULL_POINTER, "out_n is NULL");
    DeviceGuard g(s->device);
    if (rsv_status st = flush_stage(s)) return st;
    int64_t m;
    const void* src;
    if (s->cfg.kind == RSV_KIND_DISTINCT) {
        if (int rc = distinct_finalize(s->distinct, s->stream)) return (rsv_status)rc;
        m = distinct_size(s->distinct);
        if (m > cap) return fail(RSV_E_ILLEGAL_ARGUMENT, "result buffer too small");
        if (m && !out && !take) return fail(RSV_E_NULL_POINTER, "out is NULL");
        if (m) {
            if (device_out) {
                if (int rc = distinct_export(s->distinct, out, nullptr, s->stream)) return (rsv_status)rc;
            } else {
                if (rsv_status st = ensure_result_buffer(s)) return st;
                const void* set_k = distinct_keys_dev(s->distinct);
                if (s->result_publish) {  // the set straight into coherent host memory + flag spin
                    uint32_t gen = s->pub_gen;
                    if (!(s->pub_valid && s->pub_ops == s->ops)) {  // no speculative publication of it
                        touch(s);
                        gen = ++s->result_gen;
                        if (int rc = distinct_publish(s->distinct, s->result_dev, s->result_flag_dev, gen, s->stream))
                            return (rsv_status)rc;
                    }
                    s->pub_valid = false;
                    if (rsv_status st = wait_flag(s, gen)) return st;
                    // the publication was the handle's last work: no stream synchronize
                    if (s->result_gen == gen) s->ops_done = s->ops;
                    if (!take) memcpy(out, s->result_h, (size_t)m * s->kw);
                    *out_n = m;
                    if (!s->cfg.reusable) s->open = false;
                    return RSV_OK;
                } else {
                    touch(s);
                    RSV_HIP_TRY(hipMemcpyAsync(s->result_h, set_k, m * s->kw, hipMemcpyDeviceToHost, s->stream));
                    RSV_HIP_TRY(sync_stream(s));
                }
                memcpy(out, s->result_h, (size_t)m * s->kw);
            }
        }
        src = nullptr;
    } else {
        m = std::min<int64_t>(s->count, (int64_t)s->k);  // resultImpl, Sampler.scala:318-331
        if (m > cap) return fail(RSV_E_ILLEGAL_ARGUMENT, "result buffer too small");
        if (m && !out && !take) return fail(RSV_E_NULL_POINTER, "out is NULL");
        src = s->slot_key;
        if (m && !out && take) out = s->result_h;  // checked: a published result (see rsv_result_take)
        if (m && device_out) {
            touch(s);
            RSV_HIP_TRY(hipMemcpyAsync(out, src, m * s->kw, hipMemcpyDeviceToDevice, s->stream));
        } else if (m) {
            if (rsv_status st = ensure_result_buffer(s)) return st;
            if (s->result_publish) {  // publish kernel + flag spin (no D2H copy, no stream sync)
                uint32_t gen = s->pub_gen;
                if (!s->pub_valid) {  // the last batch's resolve did not publish the current slots
                    gen = ++s->result_gen;
                    touch(s);
                    RSV_HIP_TRY(launch_publish(src, m * s->kw, s->result_dev, s->result_flag_dev, gen, s->stream));
                    s->pub_ops = s->ops;
                    s->pub_gen = gen;
                    s->pub_valid = true;
                }
                if (rsv_status st = wait_flag(s, gen)) return st;
                if (s->pub_valid && s->pub_ops == s->ops && s->result_gen == gen) s->ops_done = s->ops;
                if (!take) memcpy(out, s->result_h, (size_t)m * s->kw);
                *out_n = m;
                if (!s->cfg.reusable) s->open = false;
                return RSV_OK;
            }
            // large reservoirs through a pinned buffer: a pageable D2H costs a staged copy
            touch(s);
            RSV_HIP_TRY(hipMemcpyAsync(s->result_h, src, m * s->kw, hipMemcpyDeviceToHost, s->stream));
        }
    }
    RSV_HIP_TRY(sync_stream(s));
    if (m && !device_out && s->cfg.kind != RSV_KIND_DISTINCT) memcpy(out, s->result_h, (size_t)m * s->kw);
    *out_n = m;
    if (!s->cfg.reusable) s->open = false;  // SingleUse.close, Sampler.scala:188-191, :345-350
    return RSV_OK;
}

rsv_status rsv_result(rsv_sampler* s, void* out, int64_t cap, int64_t* out_n) {
    return result_impl(s, out, cap, out_n, false);
}

rsv_status rsv_result_device(rsv_sampler* s, void* out_dev, int64_t cap, int64_t* out_n) {
    return result_impl(s, out_dev, cap, out_n, true);
}

rsv_status rsv_result_take(rsv_sampler* s, void** buf, int64_t* out_n) {
    if (rsv_status st = check_keyed(s)) return st;
    if (!buf || !out_n) return fail(RSV_E_NULL_POINTER, "buf / out_n is NULL");
    if (s->cfg.reusable || (int64_t)s->k * s->kw > kPublishMaxBytes)
        return fail(RSV_E_UNSUPPORTED, "rsv_result_take: single-use samplers with a published result only");
    {
        DeviceGuard g(s->device);
        if (rsv_status st = ensure_result_buffer(s)) return st;
    }
    // the published path of rsv_result, with the buffer handed over instead of copied
    void* h = s->result_h;
    const int64_t cap = s->k;
    rsv_status st = result_impl(s, nullptr, cap, out_n, false, /*take=*/true);
    if (st != RSV_OK) return st;
    *buf = h;
    s->result_h = nullptr;  // the caller's now: a closed single-use handle publishes nothing more
    s->result_dev = nullptr;
    s->result_flag = nullptr;
    s->result_flag_dev = nullptr;
    s->result_publish = false;
    return RSV_OK;
}

void rsv_host_release(void* buf) {
    if (buf) pool_host_free(buf);
}

int32_t rsv_is_open(const rsv_sampler* s) { return s && s->open ? 1 : 0; }

int64_t rsv_count(const rsv_sampler* s) { return s ? s->count + s->stage_n : 0; }

rsv_status rsv_set_stream(rsv_sampler* s, void* hip_stream) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    DeviceGuard g(s->device);
    if (s->side_pending) {  // the hand-over covers the forked resolve too
        join_side(s);
        ++s->ops;
    }
    if (s->ops != s->ops_done && (hipStream_t)hip_stream != s->stream) {
        // stream-ordered hand-over, no host wait: the new stream waits for the work queued so far
        // (e.g. a combine moved to a communication stream while the next batch samples on the
        // first).  The event is the handle's own until rsv_destroy: handed back to the pool at
        // once, its next record elsewhere could land before the wait binds
        if (!s->handover) RSV_HIP_TRY(pool_event(&s->handover, hipEventDisableTiming));
        RSV_HIP_TRY(hipEventRecord(s->handover, s->stream));
        RSV_HIP_TRY(hipStreamWaitEvent((hipStream_t)hip_stream, s->handover, 0));
    }
    if (s->own_stream) pool_release_stream(s->device, s->stream);
    s->stream = (hipStream_t)hip_stream;
    s->own_stream = false;
    return RSV_OK;
}

void* rsv_get_stream(const rsv_sampler* s) { return s ? (void*)s->stream : nullptr; }

rsv_status rsv_set_resolve_stream(rsv_sampler* s, void* hip_stream) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    if (s->cfg.kind != RSV_KIND_ELEMENTS) return fail(RSV_E_UNSUPPORTED, "rsv_set_resolve_stream: ELEMENTS samplers only");
    DeviceGuard g(s->device);
    if (s->side_pending) {
        join_side(s);
        ++s->ops;
    }
    s->rstream = (hipStream_t)hip_stream;
    return RSV_OK;
}

rsv_status rsv_synchronize(rsv_sampler* s) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    DeviceGuard g(s->device);
    RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

rsv_status rsv_profile_enable(rsv_sampler* s, int32_t on) {
    if (!s) return fail(RSV_E_NULL_POINTER, "sampler is NULL");
    s->timer.on = on != 0;
    return RSV_OK;
}

rsv_status rsv_profile_read(rsv_sampler* s, double* total_ms, int64_t* launches) {
    if (!s || !total_ms || !launches) return fail(RSV_E_NULL_POINTER, "NULL argument");
    DeviceGuard g(s->device);
    RSV_HIP_TRY(s->timer.drain());
    *total_ms = s->timer.total_ms;
    *launches = s->timer.launches;
    return RSV_OK;
}

rsv_status rsv_profile_global(int32_t on) {
    if (on < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "rsv_profile_global: negative sampling stride");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (on) {
        g_prof_every = on;
        // the first timed launch is the (on / 2)-th, not the first: a region's first launch finds the
        // GPU idle, so its start event is stamped before the host has even submitted the kernel and
        // the pair would time the host's launch latency too (the 20-step bench: ~85 vs ~83 us)
        g_prof_seq = on - on / 2;
        // the timing events up front (128 pairs, on the current device), so that no event is
        // created inside the region being timed: at a 20-step bench region the lazily created
        // events of its 3 timed launches cost ~3 us per step (tools/probe_region.py)
        KernelTimer& t = global_timer();
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && (t.ev.empty() || t.device == dev)) {
            t.device = dev;
            hipEvent_t last = nullptr;
            while (t.ev.size() < 256) {
                hipEvent_t e;
                if (pool_event(&e, KernelTimer::kFlags) != hipSuccess) break;
                (void)hipEventRecord(e, nullptr);  // an event's first record may set it up
                t.ev.push_back(e);
                last = e;
            }
            if (last) (void)hipEventSynchronize(last);
        }
    }
    g_prof_on = on != 0;
    return RSV_OK;
}

rsv_status rsv_profile_global_read(double* total_ms, int64_t* launches) {
    if (!total_ms || !launches) return fail(RSV_E_NULL_POINTER, "NULL argument");
    std::lock_guard<std::mutex> lk(g_prof_mu);
    KernelTimer& t = global_timer();
    DeviceGuard g(t.device);
    RSV_HIP_TRY(t.drain());
    *total_ms = t.total_ms;
    *launches = t.launches;
    t.total_ms = 0;
    t.launches = 0;
    return RSV_OK;
}

rsv_status rsv_seek(rsv_sampler* s, int64_t index) {
    if (rsv_status st = check_open(s)) return st;
    if (s->cfg.kind != RSV_KIND_ELEMENTS || s->cfg.engine != RSV_ENGINE_PHILOX_R)
        return fail(RSV_E_UNSUPPORTED, "rsv_seek needs an ELEMENTS sampler on RSV_ENGINE_PHILOX_R");
    if (s->stage_n) {  // only staged per-element samples need the device here
        DeviceGuard g(s->device);
        if (rsv_status st = flush_stage(s)) return st;
    }
    if (index < s->count) return fail(RSV_E_ILLEGAL_ARGUMENT, "rsv_seek cannot move backwards");
    // a publication holds min(count, k) keys: once the count crosses k it covers too few
    if (std::min<int64_t>(index, s->k) != std::min<int64_t>(s->count, s->k)) s->pub_valid = false;
    s->count = index;
    return RSV_OK;
}

rsv_status rsv_export_state(rsv_sampler* s, int64_t* idx_dev, void* keys_dev, int64_t* hash_dev,
                            int64_t* out_n) {
    if (rsv_status st = check_keyed(s)) return st;
    if (!out_n) return fail(RSV_E_NULL_POINTER, "out_n is NULL");
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    if (s->cfg.kind == RSV_KIND_DISTINCT) {
        if (int rc = distinct_finalize(s->distinct, s->stream)) return (rsv_status)rc;
        if (int rc = distinct_export(s->distinct, keys_dev, hash_dev, s->stream)) return (rsv_status)rc;
        *out_n = distinct_size(s->distinct);
    } else {
        if (rsv_status st = ensure_slots(s)) return st;
        if (idx_dev) RSV_HIP_TRY(hipMemcpyAsync(idx_dev, s->slot_idx, s->k * 8ull, hipMemcpyDeviceToDevice, s->stream));
        if (keys_dev)
            RSV_HIP_TRY(hipMemcpyAsync(keys_dev, s->slot_key, (size_t)s->k * s->kw, hipMemcpyDeviceToDevice, s->stream));
        *out_n = s->k;
    }
    // on the handle's private stream the caller cannot order against it: wait; on a caller
    // stream (rsv_set_stream) the copies are stream-ordered for the caller's next work
    if (s->own_stream) RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

rsv_status rsv_merge_state(rsv_sampler* s, const int64_t* idx_dev, const void* keys_dev, const int64_t* hash_dev,
                           const int64_t* part_n_host, int32_t parts, int64_t part_len, int64_t total_count) {
    if (rsv_status st = check_keyed(s)) return st;
    if (parts < 0 || part_len < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative parts/part_len");
    if (parts > 0 && !keys_dev) return fail(RSV_E_NULL_POINTER, "keys_dev is NULL");
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    if (s->cfg.kind == RSV_KIND_DISTINCT) {
        if (parts > 0 && (!hash_dev || !part_n_host)) return fail(RSV_E_NULL_POINTER, "hash_dev/part_n is NULL");
        if (parts > 0)
            if (int rc = distinct_merge_parts(s->distinct, keys_dev, hash_dev, part_n_host, parts, part_len, s->stream))
                return (rsv_status)rc;
    } else {
        if (part_len < (int64_t)s->k) return fail(RSV_E_ILLEGAL_ARGUMENT, "part_len < k");
        if (parts > 0 && !idx_dev) return fail(RSV_E_NULL_POINTER, "idx_dev is NULL");
        if (rsv_status st = ensure_slots(s)) return st;
        RSV_HIP_TRY(launch_merge_slots(idx_dev, keys_dev, s->kw, parts, part_len, s->k, s->slot_idx, s->slot_key,
                                       s->stream));
        s->pub_valid = false;
    }
    if (total_count > s->count) s->count = total_count;
    if (s->own_stream) RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

static rsv_status check_distinct(rsv_sampler* s, const char* what) {
    if (rsv_status st = check_open(s)) return st;
    if (s->cfg.kind != RSV_KIND_DISTINCT) return fail(RSV_E_UNSUPPORTED, std::string(what) + " needs a DISTINCT sampler");
    return RSV_OK;
}

rsv_status rsv_get_distinct_info(rsv_sampler* s, rsv_distinct_info* out) {
    if (rsv_status st = check_distinct(s, "rsv_get_distinct_info")) return st;
    if (!out) return fail(RSV_E_NULL_POINTER, "out is NULL");
    if (out->struct_size < sizeof(rsv_distinct_info)) return fail(RSV_E_ILLEGAL_ARGUMENT, "struct_size too small");
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    if (int rc = distinct_settle(s->distinct, s->stream)) return (rsv_status)rc;
    distinct_info(s->distinct, &out->ordered, &out->tied, &out->log_retained, &out->size, &out->max_hash,
                  &out->log_entries, &out->sched_passes, &out->sched_fallbacks);
    return RSV_OK;
}

rsv_status rsv_export_log(rsv_sampler* s, int64_t bound, int64_t* hashes_host, void* keys_host, int64_t cap,
                          int64_t* out_n) {
    if (rsv_status st = check_distinct(s, "rsv_export_log")) return st;
    if (!out_n) return fail(RSV_E_NULL_POINTER, "out_n is NULL");
    if (cap < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative cap");
    if (cap > 0 && (!hashes_host || !keys_host)) return fail(RSV_E_NULL_POINTER, "hashes_host/keys_host is NULL");
    if (cap == 0) hashes_host = nullptr, keys_host = nullptr;  // count-only query
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    return (rsv_status)distinct_log_export(s->distinct, bound, hashes_host, keys_host, cap, out_n, s->stream);
}

rsv_status rsv_merge_log(rsv_sampler* s, const int64_t* hashes_host, const void* keys_host, int64_t n,
                         int64_t total_count) {
    if (rsv_status st = check_distinct(s, "rsv_merge_log")) return st;
    if (n < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative n");
    if (n > 0 && (!hashes_host || !keys_host)) return fail(RSV_E_NULL_POINTER, "hashes_host/keys_host is NULL");
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    if (int rc = distinct_log_merge(s->distinct, hashes_host, keys_host, n, total_count, s->stream))
        return (rsv_status)rc;
    if (total_count > s->count) s->count = total_count;
    s->pub_valid = false;
    if (s->own_stream) RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

rsv_status rsv_retain_log(rsv_sampler* s, int32_t on) {
    if (rsv_status st = check_distinct(s, "rsv_retain_log")) return st;
    distinct_retain_log(s->distinct, on != 0);
    return RSV_OK;
}

rsv_status rsv_export_packed(rsv_sampler* s, int64_t* row_dev) {
    if (rsv_status st = check_keyed(s)) return st;
    if (!row_dev) return fail(RSV_E_NULL_POINTER, "row_dev is NULL");
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    if (s->cfg.kind == RSV_KIND_DISTINCT) {
        if (int rc = distinct_export_row(s->distinct, row_dev, s->count, s->stream)) return (rsv_status)rc;
        if (s->own_stream) RSV_HIP_TRY(sync_stream(s));
        return RSV_OK;
    }
    if (rsv_status st = ensure_slots(s)) return st;
    RSV_HIP_TRY(launch_export_packed(s->slot_idx, s->slot_key, s->kw, s->k, row_dev, s->stream));
    if (s->own_stream) RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

rsv_status rsv_merge_packed(rsv_sampler* s, const int64_t* rows_dev, int32_t parts, int64_t row_stride,
                            int64_t total_count) {
    if (rsv_status st = check_keyed(s)) return st;
    if (parts < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative parts");
    if (s->cfg.kind == RSV_KIND_DISTINCT) {
        // [keys (k, as int64 words: key_width / 8 each for byte keys) | hashes (k) | 6 meta words]
        const int64_t row_len = (int64_t)s->k * (1 + (s->kw > 8 ? s->kw / 8 : 1)) + 6;
        if (row_stride < row_len) return fail(RSV_E_ILLEGAL_ARGUMENT, "row_stride shorter than a packed row");
        if (parts > 0 && !rows_dev) return fail(RSV_E_NULL_POINTER, "rows_dev is NULL");
        DeviceGuard g(s->device);
        touch(s);
        if (rsv_status st = flush_stage(s)) return st;
        if (int rc = distinct_merge_rows(s->distinct, rows_dev, parts, row_stride, s->stream)) return (rsv_status)rc;
        if (total_count > s->count) s->count = total_count;
        s->pub_valid = false;
        if (s->own_stream) {  // the call returns with its work done: settle now, while the rows are the caller's
            RSV_HIP_TRY(sync_stream(s));
            if (int rc = distinct_settle(s->distinct, s->stream)) return (rsv_status)rc;
        }
        return RSV_OK;
    }
    const int64_t row_min = (int64_t)s->k * (1 + (s->kw > 8 ? s->kw / 8 : 1));  // [idx(k) | keys]
    if (row_stride < row_min) return fail(RSV_E_ILLEGAL_ARGUMENT, "row_stride shorter than a packed row");
    if (parts > 0 && !rows_dev) return fail(RSV_E_NULL_POINTER, "rows_dev is NULL");
    DeviceGuard g(s->device);
    touch(s);
    if (rsv_status st = flush_stage(s)) return st;
    if (rsv_status st = ensure_slots(s)) return st;
    if (total_count > s->count) s->count = total_count;
    if (parts > 0) {
        bool fused = false;
        if (s->k <= kFusedPublishMaxK && s->kw <= 8) {  // merge + publish in one dispatch
            if (rsv_status st = ensure_result_buffer(s)) return st;
            if (s->result_publish) {
                const uint32_t gen = ++s->result_gen;
                const int64_t m = std::min<int64_t>(s->count, (int64_t)s->k);
                RSV_HIP_TRY(launch_merge_packed_publish(rows_dev, parts, row_stride, s->k, s->slot_idx, s->slot_key,
                                                        s->kw, m, s->result_dev, s->result_flag_dev, gen, s->stream));
                s->pub_gen = gen;
                s->pub_valid = true;
                s->pub_ops = s->ops;
                fused = true;
            }
        }
        if (!fused) {
            RSV_HIP_TRY(launch_merge_packed(rows_dev, parts, row_stride, s->k, s->slot_idx, s->slot_key, s->kw,
                                            s->stream));
            s->pub_valid = false;
        }
    }
    if (s->own_stream) RSV_HIP_TRY(sync_stream(s));
    return RSV_OK;
}

rsv_status rsv_sample_segmented(const void* keys_dev, const int64_t* offsets_dev, int64_t num_streams,
                                int32_t key_width, int32_t k, uint64_t seed, uint64_t stream_base, void* out_dev,
                                int64_t* counts_dev, void* hip_stream) {
    if (k <= 0 || k > kMaxSize) return fail(RSV_E_ILLEGAL_ARGUMENT, "k out of range");
    if (key_width != 4 && key_width != 8) return fail(RSV_E_ILLEGAL_ARGUMENT, "key_width must be 4 or 8");
    if (num_streams < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative stream count");
    if (num_streams == 0) return RSV_OK;
    if (!offsets_dev || !out_dev || !counts_dev) return fail(RSV_E_NULL_POINTER, "NULL buffer");
    const DrawParams dp{seed, stream_base};
    RSV_HIP_TRY(launch_segmented(keys_dev, key_width, offsets_dev, num_streams, (uint32_t)k, dp, out_dev, counts_dev,
                                 (hipStream_t)hip_stream));
    return RSV_OK;
}

rsv_status rsv_replay_events(const void* keys_dev, int64_t n, int32_t key_width, int64_t base_index,
                             const int64_t* ev_pos_dev, const int32_t* ev_slot_dev, int64_t n_events, int32_t k,
                             void* reservoir_dev, void* hip_stream) {
    if (k <= 0 || k > kMaxSize) return fail(RSV_E_ILLEGAL_ARGUMENT, "k out of range");
    if (key_width != 4 && key_width != 8) return fail(RSV_E_ILLEGAL_ARGUMENT, "key_width must be 4 or 8");
    if (n < 0 || n_events < 0 || base_index < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative size");
    if (!reservoir_dev || (n && !keys_dev) || (n_events && (!ev_pos_dev || !ev_slot_dev)))
        return fail(RSV_E_NULL_POINTER, "NULL buffer");
    hipStream_t st = (hipStream_t)hip_stream;
    unsigned long long* win = nullptr;
    RSV_HIP_TRY(hipMallocAsync((void**)&win, (size_t)k * 8, st));
    hipError_t e = hipMemsetAsync(win, 0, (size_t)k * 8, st);
    if (e == hipSuccess) e = launch_replay_events(ev_pos_dev, ev_slot_dev, n_events, (uint32_t)k, win, st);
    if (e == hipSuccess) e = launch_resolve(keys_dev, key_width, base_index, n, (uint32_t)k, win, reservoir_dev, nullptr, false, st);
    hipError_t e2 = hipFreeAsync(win, st);
    RSV_HIP_TRY(e);
    RSV_HIP_TRY(e2);
    return RSV_OK;
}

rsv_status rsv_export_draws(uint64_t seed, uint64_t stream_id, uint64_t i0, int64_t n, uint64_t* j_dev,
                            void* hip_stream) {
    if (n < 0) return fail(RSV_E_ILLEGAL_ARGUMENT, "negative n");
    if (n && !j_dev) return fail(RSV_E_NULL_POINTER, "j_dev is NULL");
    const DrawParams dp{seed, stream_id};
    RSV_HIP_TRY(launch_export_draws(dp, i0, n, j_dev, (hipStream_t)hip_stream));
    return RSV_OK;
}

}  // extern "C"
