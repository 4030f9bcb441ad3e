// rsv_pool.hip -- process-wide caching of the per-sampler resources: device buffers, pinned host
// buffers, HIP streams and events.
//
// The reference creates a sampler per stream materialisation (Sample.scala:23-24 takes it by name)
// and a fresh one per `Sampler.apply`; a HIP sampler that paid hipStreamCreate + hipMalloc +
// hipHostMalloc + memsets at every creation spent ~380 us there -- more than a whole 1e9-element
// K1 pass.  Released resources are kept per (kind, device, power-of-two size class) and handed to
// the next sampler; blocks above kMaxPooled bytes go straight to the HIP allocator.
//
// Reuse safety: a block is only released once no queued work can touch it -- rsv_destroy
// synchronizes the sampler's stream first, and in-place growth (rsv_distinct.hip) synchronizes
// before releasing the old block -- so handing it to a sampler on another stream cannot race.
// Cached blocks live until process exit (no static destructor: the HIP runtime may already be
// torn down by then).
#include <mutex>
#include <unordered_map>
#include <vector>

#include "rsv_internal.h"

namespace rsv {
namespace {

constexpr size_t kMinClass = 256;
constexpr size_t kMaxPooled = 256ull << 20;
constexpr size_t kCacheCapDevice = 2ull << 30;  // cached (idle) bytes per device
constexpr size_t kCacheCapHost = 256ull << 20;

enum Kind : uint32_t { kDevice = 0, kHost = 1 };

struct Block {
    uint32_t kind;
    unsigned flags;  // hipHostMalloc flags (host blocks)
    int device;
    size_t bytes;    // allocated size (the class size when pooled)
    bool pooled;
};

struct Pool {
    std::mutex mu;
    std::unordered_map<void*, Block> live;
    std::unordered_map<uint64_t, std::vector<void*>> idle;  // key -> blocks
    std::unordered_map<uint64_t, size_t> idle_bytes;        // (kind, device) -> bytes
    std::unordered_map<uint64_t, std::vector<hipStream_t>> streams;
    std::unordered_map<uint64_t, std::vector<hipEvent_t>> events;
};

Pool& pool() {
    static Pool* p = new Pool();  // intentionally leaked (see header)
    return *p;
}

size_t class_of(size_t bytes) {
    size_t c = kMinClass;
    while (c < bytes) c <<= 1;
    return c;
}

uint64_t key_of(uint32_t kind, unsigned flags, int device, size_t cls) {
    // hipHostMalloc flags in 8 bits: Portable / Mapped / WriteCombined (low nibble) and NumaUser /
    // Coherent / NonCoherent (bits 29-31) -- a coherent block is never handed out as a default one
    const uint64_t f8 = (flags & 0x0Fu) | ((flags >> 24) & 0xF0u);
    return ((uint64_t)kind << 62) | (f8 << 54) | ((uint64_t)(device & 0xFF) << 46) |
           (uint64_t)__builtin_ctzll(cls);
}

uint64_t owner_of(uint32_t kind, int device) { return ((uint64_t)kind << 32) | (uint32_t)device; }

hipError_t raw_alloc(uint32_t kind, unsigned flags, size_t bytes, void** p) {
    return kind == kDevice ? hipMalloc(p, bytes) : hipHostMalloc(p, bytes, flags);
}

void raw_free(uint32_t kind, void* p) {
    if (kind == kDevice)
        (void)hipFree(p);
    else
        (void)hipHostFree(p);
}

hipError_t alloc(uint32_t kind, unsigned flags, size_t bytes, void** out) {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) device = 0;
    if (bytes == 0) bytes = 1;
    Pool& P = pool();
    const bool pooled = bytes <= kMaxPooled;
    const size_t sz = pooled ? class_of(bytes) : bytes;
    if (pooled) {
        std::lock_guard<std::mutex> lk(P.mu);
        auto it = P.idle.find(key_of(kind, flags, device, sz));
        if (it != P.idle.end() && !it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            P.idle_bytes[owner_of(kind, device)] -= sz;
            P.live[p] = Block{kind, flags, device, sz, true};
            *out = p;
            return hipSuccess;
        }
    }
    void* p = nullptr;
    hipError_t e = raw_alloc(kind, flags, sz, &p);
    if (e != hipSuccess) {
        // idle blocks of other classes may be what stands in the way: drop them and retry once
        pool_trim();
        e = raw_alloc(kind, flags, sz, &p);
        if (e != hipSuccess) return e;
    }
    std::lock_guard<std::mutex> lk(P.mu);
    P.live[p] = Block{kind, flags, device, sz, pooled};
    *out = p;
    return hipSuccess;
}

void release(void* p) {
    if (!p) return;
    Pool& P = pool();
    Block b;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto it = P.live.find(p);
        if (it == P.live.end()) return;  // not ours: ignore rather than corrupt the heap
        b = it->second;
        P.live.erase(it);
        if (b.pooled) {
            size_t& idle = P.idle_bytes[owner_of(b.kind, b.device)];
            const size_t cap = b.kind == kDevice ? kCacheCapDevice : kCacheCapHost;
            if (idle + b.bytes <= cap) {
                idle += b.bytes;
                P.idle[key_of(b.kind, b.flags, b.device, b.bytes)].push_back(p);
                return;
            }
        }
    }
    raw_free(b.kind, p);
}

}  // namespace

hipError_t pool_device_alloc(void** p, size_t bytes) { return alloc(kDevice, 0, bytes, p); }
void pool_device_free(void* p) { release(p); }
hipError_t pool_host_alloc(void** p, size_t bytes, unsigned flags) { return alloc(kHost, flags, bytes, p); }
void pool_host_free(void* p) { release(p); }

void pool_trim() {
    Pool& P = pool();
    std::vector<std::pair<uint32_t, void*>> drop;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        for (auto& kv : P.idle) {
            const uint32_t kind = (uint32_t)(kv.first >> 62);
            for (void* p : kv.second) drop.emplace_back(kind, p);
            kv.second.clear();
        }
        P.idle_bytes.clear();
    }
    for (auto& d : drop) raw_free(d.first, d.second);
}

hipError_t pool_stream(hipStream_t* out) {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) device = 0;
    Pool& P = pool();
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto& v = P.streams[(uint64_t)device];
        if (!v.empty()) {
            *out = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
}

void pool_release_stream(int device, hipStream_t st) {  // st must be idle
    if (!st) return;
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    auto& v = P.streams[(uint64_t)device];
    if (v.size() < 64) {
        v.push_back(st);
        return;
    }
    (void)hipStreamDestroy(st);
}

hipError_t pool_event(hipEvent_t* out, unsigned flags) {
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) device = 0;
    Pool& P = pool();
    const uint64_t key = ((uint64_t)flags << 32) | (uint32_t)device;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        auto& v = P.events[key];
        if (!v.empty()) {
            *out = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipEventCreateWithFlags(out, flags);
}

void pool_release_event(int device, hipEvent_t e, unsigned flags) {
    if (!e) return;
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    auto& v = P.events[((uint64_t)flags << 32) | (uint32_t)device];
    if (v.size() < 1024) {
        v.push_back(e);
        return;
    }
    (void)hipEventDestroy(e);
}

}  // namespace rsv
