// rsv_distinct.hip -- Sampler.distinct (RandomValues, Sampler.scala:383-412) on gfx950.
//
// The reference keeps, for a stream of elements, the k distinct elements with the smallest signed
// h = byteswap64(r1 ^ byteswap64(r0 ^ hash(elem))) (its max-heap evicts the current maximum
// whenever a smaller unseen element arrives, Sampler.scala:403-407).  With an injective `hash`
// the result is the bottom-k of h over the distinct elements, independent of arrival order, so
// it is computed here as
//   K3  filter:  one streaming pass over the keys (HBM-bound, 8 B/elem for Long keys): compute h,
//                keep (h, key) with h <= T in a candidate buffer (wave-aggregated append)
//   merge:       candidates + current set -> radix sort by (h, key) -> drop exact duplicates ->
//                first k = new set
// T is the current maximum (minus one) once the set is full, otherwise a quantile estimated from
// a strided sample of the batch; a threshold that proves too tight (fewer than k distinct
// candidates) or too loose (candidate buffer overflow) is corrected and the pass re-run, so the
// result is exact regardless of the estimate.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <vector>

#include "../../include/reservoir_hip.h"
#include "rsv_device.h"
#include "rsv_internal.h"

namespace rsv {

namespace {

constexpr int kBlock = 256;
constexpr int64_t kSample = 65536;

__device__ __forceinline__ unsigned long long lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Candidate output: staged per wave in LDS and written 64 at a time, so the global reservation
// counter sees one atomic per 64 candidates (a single contended word sustains ~88 atomics/us:
// one atomic per candidate cost 1.5 ms at 132k candidates).
template <typename KeyT>
struct CandOut {
    int64_t* qh;  // LDS: 128 hashes of this wave
    KeyT* qk;     // LDS: 128 keys
    uint32_t qn;  // wave-uniform fill
    int64_t* cand_h;
    KeyT* cand_k;
    unsigned long long* counter;
    int64_t cap;

    __device__ __forceinline__ void write64(uint32_t from, uint32_t cnt) {
        const uint32_t lane = threadIdx.x & 63;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(counter, (unsigned long long)cnt);
        base = __shfl(base, 0);
        if (lane < cnt) {
            const unsigned long long pos = base + lane;
            if ((int64_t)pos < cap) {
                cand_h[pos] = qh[from + lane];
                cand_k[pos] = qk[from + lane];
            }
        }
    }
    __device__ __forceinline__ void push(bool c, int64_t h, KeyT key) {
        const unsigned long long bal = __ballot(c);
        if (bal == 0) return;
        if (c) {
            const uint32_t pos = qn + __popcll(bal & lanemask_lt());
            qh[pos] = h;
            qk[pos] = key;
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= 64) {
            qn -= 64;
            __builtin_amdgcn_wave_barrier();
            write64(qn, 64);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __device__ __forceinline__ void flush() {
        __builtin_amdgcn_wave_barrier();
        if (qn) write64(0, qn);
        qn = 0;
    }
};

template <typename KeyT, int HASH>
__device__ __forceinline__ int64_t elem_hash(const KeyT* keys, const int64_t* hashes, int64_t idx,
                                             KeyT key, int64_t r0, int64_t r1) {
    if constexpr (HASH == kHashPrecomputed) return scramble(r0, r1, hashes[idx]);
    else return scramble(r0, r1, hash_of<KeyT, HASH>(key));
}

template <typename KeyT>
struct Vec;
typedef long long v2i64 __attribute__((ext_vector_type(2)));
typedef int v4i32 __attribute__((ext_vector_type(4)));
template <>
struct Vec<int64_t> {
    using T = v2i64;
    static constexpr int N = 2;
    __device__ static int64_t get(const T& v, int e) { return v[e]; }
};
template <>
struct Vec<int32_t> {
    using T = v4i32;
    static constexpr int N = 4;
    __device__ static int32_t get(const T& v, int e) { return v[e]; }
};

// K3 filter: streaming pass.  The main loop covers whole grid tiles with unguarded loads (U x 16 B
// per lane issued back to back, so each wave keeps U loads in flight); per-element work is the
// scrambled hash and one compare, and the rare candidates take one wave-uniform slow path.
template <typename KeyT, int HASH, int U>
__device__ __forceinline__ void k3_tile(const typename Vec<KeyT>::T* x, int64_t v0, int64_t T,
                                        const KeyT* keys, const int64_t* hashes, int64_t r0, int64_t r1,
                                        int64_t tinc, CandOut<KeyT>& out) {
    using V = Vec<KeyT>;
    int64_t h[U][V::N];
    bool any = false;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < V::N; ++e) {
            h[u][e] = elem_hash<KeyT, HASH>(keys, hashes, (v0 + u * T) * V::N + e, V::get(x[u], e), r0, r1);
            any |= h[u][e] <= tinc;
        }
    if (__any(any)) {  // ~1e-4 of the waves at the steady-state threshold
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < V::N; ++e)
                out.push(h[u][e] <= tinc, h[u][e], V::get(x[u], e));
    }
}

template <typename KeyT, int HASH>
__global__ __launch_bounds__(kBlock) void k3_filter(const KeyT* __restrict__ keys,
                                                    const int64_t* __restrict__ hashes, int64_t n,
                                                    int64_t r0, int64_t r1, int64_t tinc,
                                                    int64_t* __restrict__ cand_h,
                                                    KeyT* __restrict__ cand_k,
                                                    unsigned long long* __restrict__ counter,
                                                    int64_t cap) {
    using V = Vec<KeyT>;
    constexpr int U = 4;
    __shared__ int64_t sh_h[kBlock / 64][128];
    __shared__ KeyT sh_k[kBlock / 64][128];
    CandOut<KeyT> out{sh_h[threadIdx.x >> 6], sh_k[threadIdx.x >> 6], 0u, cand_h, cand_k, counter, cap};
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_vec = n / V::N;
    const typename V::T* kv = reinterpret_cast<const typename V::T*>(keys);
    const int64_t full = n_vec / (T * U);  // whole tiles: every lane has U vectors
    for (int64_t it = 0; it < full; ++it) {
        const int64_t v0 = it * T * U + tid;
        typename V::T x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(kv + v0 + u * T);
        k3_tile<KeyT, HASH, U>(x, v0, T, keys, hashes, r0, r1, tinc, out);
    }
    // remaining vectors, one per lane per step, then the n % V::N tail elements
    for (int64_t v = full * T * U + tid; v - tid < n_vec; v += T) {
        const bool ok = v < n_vec;
        typename V::T x[1];
        x[0] = ok ? kv[v] : typename V::T{};
        int64_t h[V::N];
#pragma unroll
        for (int e = 0; e < V::N; ++e) {
            h[e] = ok ? elem_hash<KeyT, HASH>(keys, hashes, v * V::N + e, V::get(x[0], e), r0, r1) : 0;
            out.push(ok && h[e] <= tinc, h[e], V::get(x[0], e));
        }
    }
    for (int64_t idx = n_vec * V::N + tid; idx - tid < n; idx += T) {
        const bool ok = idx < n;
        const KeyT key = ok ? keys[idx] : (KeyT)0;
        const int64_t h = ok ? elem_hash<KeyT, HASH>(keys, hashes, idx, key, r0, r1) : 0;
        out.push(ok && h <= tinc, h, key);
    }
    out.flush();
}

template <typename KeyT, int HASH>
__global__ __launch_bounds__(kBlock) void sample_hash_kernel(const KeyT* __restrict__ keys,
                                                             const int64_t* __restrict__ hashes,
                                                             int64_t n, int64_t ns, int64_t r0,
                                                             int64_t r1, int64_t* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ns) return;
    const int64_t idx = (int64_t)(((unsigned __int128)t * (uint64_t)n) / (uint64_t)ns);
    out[t] = elem_hash<KeyT, HASH>(keys, hashes, idx, keys[idx], r0, r1);
}

// after sorting by (h, key): flag = first of each run of identical (h, key)
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void dedup_flags(const int64_t* __restrict__ h,
                                                      const KeyT* __restrict__ key, int64_t n,
                                                      uint32_t* __restrict__ flags) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    flags[p] = (p == 0 || h[p] != h[p - 1] || key[p] != key[p - 1]) ? 1u : 0u;
}

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void compact_first_k(const int64_t* __restrict__ h,
                                                          const KeyT* __restrict__ key,
                                                          const uint32_t* __restrict__ flags,
                                                          const uint32_t* __restrict__ pos, int64_t n,
                                                          int64_t k, int64_t* __restrict__ out_h,
                                                          KeyT* __restrict__ out_k,
                                                          int64_t* __restrict__ out_count) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    if (flags[p] && (int64_t)pos[p] < k) {
        out_h[pos[p]] = h[p];
        out_k[pos[p]] = key[p];
        if ((int64_t)pos[p] == k - 1) out_count[1] = h[p];  // the new maximum (set full)
    }
    if (p == n - 1) out_count[0] = (int64_t)pos[p] + (int64_t)flags[p];
}

inline unsigned grid_1d(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

struct DistinctState {
    int32_t k = 0;
    int kw = 8;
    int hash_kind = kHashIdentity;
    int64_t r0 = 0, r1 = 0;
    int64_t m = 0;                // current set size
    int64_t max_h = INT64_MIN;    // valid when m == k
    int64_t* set_h = nullptr;     // [set_cap <= k], ascending (h, key)
    void* set_k = nullptr;
    int64_t set_cap = 0;
    int64_t cand_limit = 0;       // 4k + 4096: the most candidates one filter pass may keep
    int64_t cand_cap = 0;         // allocated (grows on demand up to cand_limit)
    int64_t* cand_h = nullptr;
    void* cand_k = nullptr;
    unsigned long long* counter = nullptr;
    int64_t merge_cap = 0;        // set + candidates of one merge (grows on demand)
    int64_t *mh0 = nullptr, *mh1 = nullptr;
    void *mk0 = nullptr, *mk1 = nullptr;
    uint32_t *flags = nullptr, *pos = nullptr;
    int64_t* d_count = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    int64_t* samp = nullptr;      // [2 * kSample]
    int64_t* h_pinned = nullptr;  // host scalars
    std::vector<int64_t> samp_host;
    KernelTimer* timer = nullptr;
};

void distinct_set_timer(DistinctState* d, KernelTimer* t) { d->timer = t; }

template <typename KeyT>
static hipError_t temp_bytes_for(int64_t cap, size_t* bytes) {
    size_t a = 0, b = 0, c = 0, d = 0;
    hipError_t e;
    e = rocprim::radix_sort_pairs(nullptr, a, (KeyT*)nullptr, (KeyT*)nullptr, (int64_t*)nullptr,
                                  (int64_t*)nullptr, (size_t)cap);
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_pairs(nullptr, b, (int64_t*)nullptr, (int64_t*)nullptr, (KeyT*)nullptr,
                                  (KeyT*)nullptr, (size_t)cap);
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(nullptr, c, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)cap,
                                rocprim::plus<uint32_t>());
    if (e != hipSuccess) return e;
    e = rocprim::radix_sort_keys(nullptr, d, (int64_t*)nullptr, (int64_t*)nullptr, (size_t)kSample);
    if (e != hipSuccess) return e;
    *bytes = std::max(std::max(a, b), std::max(c, d));
    return hipSuccess;
}

// Device buffers grow on demand (geometric, capped): a sampler with a huge k that sees few
// elements (k may be up to Int.MaxValue - 2, Sampler.scala:71) allocates for what it holds.
static hipError_t grow(void** p, size_t old_bytes, size_t new_bytes, bool keep, hipStream_t st) {
    void* q = nullptr;
    hipError_t e = pool_device_alloc(&q, new_bytes ? new_bytes : 16);
    if (e != hipSuccess) return e;
    if (keep && *p && old_bytes) e = hipMemcpyAsync(q, *p, old_bytes, hipMemcpyDeviceToDevice, st);
    // queued work may still read the old block: wait before it goes back to the pool
    if (e == hipSuccess && *p) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        pool_device_free(q);
        return e;
    }
    pool_device_free(*p);
    *p = q;
    return hipSuccess;
}

static int64_t grown(int64_t cur, int64_t need, int64_t cap) {
    int64_t c = std::max<int64_t>(cur, 1024);
    while (c < need) c *= 2;
    return std::min(c, cap);
}

static hipError_t ensure_caps(DistinctState* d, int64_t cand_need, int64_t merge_need, hipStream_t st) {
    const size_t kw = (size_t)d->kw;
    hipError_t e = hipSuccess;
    cand_need = std::min(cand_need, d->cand_limit);
    if (cand_need > d->cand_cap) {
        const int64_t c = grown(d->cand_cap, cand_need, d->cand_limit);
        if ((e = grow((void**)&d->cand_h, 0, (size_t)c * 8, false, st))) return e;
        if ((e = grow(&d->cand_k, 0, (size_t)c * kw, false, st))) return e;
        d->cand_cap = c;
    }
    const int64_t set_need = std::min<int64_t>(merge_need, d->k);
    if (set_need > d->set_cap) {
        const int64_t c = grown(d->set_cap, set_need, d->k);
        if ((e = grow((void**)&d->set_h, (size_t)d->m * 8, (size_t)c * 8, true, st))) return e;
        if ((e = grow(&d->set_k, (size_t)d->m * kw, (size_t)c * kw, true, st))) return e;
        d->set_cap = c;
    }
    if (merge_need > d->merge_cap) {
        const int64_t c = grown(d->merge_cap, merge_need, (int64_t)d->k + d->cand_limit);
        if ((e = grow((void**)&d->mh0, 0, (size_t)c * 8, false, st))) return e;
        if ((e = grow((void**)&d->mh1, 0, (size_t)c * 8, false, st))) return e;
        if ((e = grow(&d->mk0, 0, (size_t)c * kw, false, st))) return e;
        if ((e = grow(&d->mk1, 0, (size_t)c * kw, false, st))) return e;
        if ((e = grow((void**)&d->flags, 0, (size_t)c * 4, false, st))) return e;
        if ((e = grow((void**)&d->pos, 0, (size_t)c * 4, false, st))) return e;
        size_t tb = 0;
        e = d->kw == 8 ? temp_bytes_for<int64_t>(c, &tb) : temp_bytes_for<int32_t>(c, &tb);
        if (e != hipSuccess) return e;
        if (tb > d->temp_bytes) {
            if ((e = grow(&d->temp, 0, tb, false, st))) return e;
            d->temp_bytes = tb;
        }
        d->merge_cap = c;
    }
    return hipSuccess;
}

DistinctState* distinct_create(int32_t k, int key_width, int hash_kind, int64_t r0, int64_t r1,
                               int* status) {
    DistinctState* d = new DistinctState();
    d->k = k;
    d->kw = key_width;
    d->hash_kind = hash_kind;
    d->r0 = r0;
    d->r1 = r1;
    d->cand_limit = 4 * (int64_t)k + 4096;
    hipError_t e = hipSuccess;
    auto A = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = pool_device_alloc(p, bytes ? bytes : 16);
    };
    A((void**)&d->counter, 16);
    A((void**)&d->d_count, 16);
    A((void**)&d->samp, 2 * kSample * 8);
    if (e == hipSuccess) {
        size_t tb = 0;  // the threshold sample's sort
        e = rocprim::radix_sort_keys(nullptr, tb, (int64_t*)nullptr, (int64_t*)nullptr, (size_t)kSample);
        d->temp_bytes = tb;
    }
    A(&d->temp, d->temp_bytes);
    if (e == hipSuccess) e = pool_host_alloc((void**)&d->h_pinned, 64, hipHostMallocDefault);
    // Typical k: allocate the whole working set now (nothing is allocated on the sampling path).
    // Huge k (up to Int.MaxValue - 2): grow with what the sampler holds.
    const int64_t full_merge = (int64_t)k + d->cand_limit;
    const double eager_bytes = (double)full_merge * (2 * 8 + 2 * key_width + 8) + (double)d->cand_limit * (8 + key_width);
    if (e == hipSuccess && eager_bytes < 512.0 * 1024 * 1024) e = ensure_caps(d, d->cand_limit, full_merge, 0);
    if (e != hipSuccess) {
        set_error(std::string("distinct_create: ") + hipGetErrorString(e));
        *status = e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;
        distinct_destroy(d);
        return nullptr;
    }
    *status = RSV_OK;
    return d;
}

void distinct_destroy(DistinctState* d) {
    if (!d) return;
    void* ps[] = {d->set_h, d->set_k, d->cand_h, d->cand_k, d->counter, d->mh0, d->mh1, d->mk0,
                  d->mk1, d->flags, d->pos, d->d_count, d->samp, d->temp};
    for (void* p : ps) pool_device_free(p);  // the owner's stream is idle (rsv_destroy)
    pool_host_free(d->h_pinned);
    delete d;
}

int64_t distinct_size(const DistinctState* d) { return d->m; }

template <typename KeyT>
static hipError_t launch_filter(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n,
                                int64_t tinc, hipStream_t st) {
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(n / 16 + 1), 1), 256 * 8);
    KeyT* ck = (KeyT*)d->cand_k;
    switch (d->hash_kind) {
    case kHashJavaLong:
        hipLaunchKernelGGL((k3_filter<KeyT, kHashJavaLong>), dim3(grid), dim3(kBlock), 0, st, keys, hashes,
                           n, d->r0, d->r1, tinc, d->cand_h, ck, d->counter, d->cand_cap);
        break;
    case kHashJavaInt:
        hipLaunchKernelGGL((k3_filter<KeyT, kHashJavaInt>), dim3(grid), dim3(kBlock), 0, st, keys, hashes,
                           n, d->r0, d->r1, tinc, d->cand_h, ck, d->counter, d->cand_cap);
        break;
    case kHashPrecomputed:
        hipLaunchKernelGGL((k3_filter<KeyT, kHashPrecomputed>), dim3(grid), dim3(kBlock), 0, st, keys,
                           hashes, n, d->r0, d->r1, tinc, d->cand_h, ck, d->counter, d->cand_cap);
        break;
    default:
        hipLaunchKernelGGL((k3_filter<KeyT, kHashIdentity>), dim3(grid), dim3(kBlock), 0, st, keys, hashes,
                           n, d->r0, d->r1, tinc, d->cand_h, ck, d->counter, d->cand_cap);
    }
    return hipGetLastError();
}

template <typename KeyT>
static hipError_t launch_sample(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n,
                                int64_t ns, hipStream_t st) {
    const unsigned grid = grid_1d(ns);
    switch (d->hash_kind) {
    case kHashJavaLong:
        hipLaunchKernelGGL((sample_hash_kernel<KeyT, kHashJavaLong>), dim3(grid), dim3(kBlock), 0, st,
                           keys, hashes, n, ns, d->r0, d->r1, d->samp);
        break;
    case kHashJavaInt:
        hipLaunchKernelGGL((sample_hash_kernel<KeyT, kHashJavaInt>), dim3(grid), dim3(kBlock), 0, st,
                           keys, hashes, n, ns, d->r0, d->r1, d->samp);
        break;
    case kHashPrecomputed:
        hipLaunchKernelGGL((sample_hash_kernel<KeyT, kHashPrecomputed>), dim3(grid), dim3(kBlock), 0, st,
                           keys, hashes, n, ns, d->r0, d->r1, d->samp);
        break;
    default:
        hipLaunchKernelGGL((sample_hash_kernel<KeyT, kHashIdentity>), dim3(grid), dim3(kBlock), 0, st,
                           keys, hashes, n, ns, d->r0, d->r1, d->samp);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = d->temp_bytes;
    return rocprim::radix_sort_keys(d->temp, tb, d->samp, d->samp + kSample, (size_t)ns, 0, 64, st);
}

// Merge `c` entries at (src_h, src_k) with the current set; new set = first k distinct by
// (h, key).  Returns the distinct count of the union in *n_distinct.
template <typename KeyT>
static hipError_t merge_into_set(DistinctState* d, const int64_t* src_h, const KeyT* src_k, int64_t c,
                                 int64_t* n_distinct, hipStream_t st) {
    const int64_t total = d->m + c;
    if (total == 0) {
        *n_distinct = 0;
        return hipSuccess;
    }
    if (hipError_t e0 = ensure_caps(d, 0, total, st)) return e0;
    KeyT* mk0 = (KeyT*)d->mk0;
    KeyT* mk1 = (KeyT*)d->mk1;
    hipError_t e;
    if (d->m) {
        if ((e = hipMemcpyAsync(d->mh0, d->set_h, d->m * 8, hipMemcpyDeviceToDevice, st))) return e;
        if ((e = hipMemcpyAsync(mk0, d->set_k, d->m * sizeof(KeyT), hipMemcpyDeviceToDevice, st))) return e;
    }
    if (c) {
        if ((e = hipMemcpyAsync(d->mh0 + d->m, src_h, c * 8, hipMemcpyDeviceToDevice, st))) return e;
        if ((e = hipMemcpyAsync(mk0 + d->m, src_k, c * sizeof(KeyT), hipMemcpyDeviceToDevice, st))) return e;
    }
    size_t tb = d->temp_bytes;
    if (d->hash_kind == kHashIdentity || d->hash_kind == kHashJavaInt) {
        // injective hash: equal h <=> equal element, so one sort by h orders (h, key)
        if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->mh0, d->mh1, mk0, mk1, (size_t)total, 0, 64, st)))
            return e;
        std::swap(d->mh0, d->mh1);
        std::swap(d->mk0, d->mk1);
        mk0 = (KeyT*)d->mk0;
        mk1 = (KeyT*)d->mk1;
    } else {
        // stable LSD order: by key, then by h  ->  sorted by (h, key)
        if ((e = rocprim::radix_sort_pairs(d->temp, tb, mk0, mk1, d->mh0, d->mh1, (size_t)total, 0,
                                           8 * (unsigned)sizeof(KeyT), st)))
            return e;
        tb = d->temp_bytes;
        if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->mh1, d->mh0, mk1, mk0, (size_t)total, 0, 64, st)))
            return e;
    }
    hipLaunchKernelGGL(dedup_flags<KeyT>, dim3(grid_1d(total)), dim3(kBlock), 0, st, d->mh0, mk0, total,
                       d->flags);
    if ((e = hipGetLastError())) return e;
    tb = d->temp_bytes;
    if ((e = rocprim::exclusive_scan(d->temp, tb, d->flags, d->pos, 0u, (size_t)total,
                                     rocprim::plus<uint32_t>(), st)))
        return e;
    hipLaunchKernelGGL(compact_first_k<KeyT>, dim3(grid_1d(total)), dim3(kBlock), 0, st, d->mh0, mk0,
                       d->flags, d->pos, total, (int64_t)d->k, d->set_h, (KeyT*)d->set_k, d->d_count);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync(d->h_pinned, d->d_count, 16, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipStreamSynchronize(st))) return e;
    *n_distinct = d->h_pinned[0];
    d->m = std::min<int64_t>(*n_distinct, d->k);
    if (d->m == d->k) d->max_h = d->h_pinned[1];
    return hipSuccess;
}

template <typename KeyT>
static int sample_impl(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n,
                       hipStream_t st) {
#define DTRY(x)                                                                      \
    do {                                                                             \
        hipError_t _e = (x);                                                         \
        if (_e != hipSuccess) {                                                      \
            set_error(std::string("distinct: " #x ": ") + hipGetErrorString(_e));    \
            return _e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;   \
        }                                                                            \
    } while (0)
    if (n <= 0) return RSV_OK;
    const bool full = d->m == d->k;
    if (full && d->max_h == INT64_MIN) return RSV_OK;  // nothing can be smaller than the max
    const int64_t t_allowed = full ? d->max_h - 1 : INT64_MAX;  // Sampler.scala:403 (strict <)
    int64_t q = 0, ns = 0;
    auto take_sample = [&]() -> int {
        ns = std::min<int64_t>(n, kSample);
        DTRY(launch_sample<KeyT>(d, keys, hashes, n, ns, st));
        d->samp_host.resize((size_t)ns);
        DTRY(hipMemcpyAsync(d->samp_host.data(), d->samp + kSample, ns * 8, hipMemcpyDeviceToHost, st));
        DTRY(hipStreamSynchronize(st));
        return RSV_OK;
    };
    auto quantile = [&](int64_t qq) -> int64_t {
        return qq >= ns ? t_allowed : std::min(d->samp_host[(size_t)std::max<int64_t>(qq, 0)], t_allowed);
    };
    int64_t tinc = t_allowed;
    const bool estimate = !full && n > d->cand_limit / 2;
    DTRY(ensure_caps(d, estimate ? d->cand_limit : n, 0, st));
    if (estimate) {
        // The scrambled hash of distinct elements is uniform on int64 (double byteswap64 keyed
        // by the random r0, r1), so ~2k + 1024 elements fall below INT64_MIN + f 2^64 with
        // f = (2k + 1024) / n.  Heavy duplication (fewer than half the elements distinct) or a
        // degenerate precomputed hash shows up as too few / too many candidates and is corrected
        // from a strided sample below.
        const long double f = (long double)(2 * (int64_t)d->k + 1024) / (long double)n;
        tinc = f >= 1.0L ? t_allowed : (int64_t)((long double)INT64_MIN + f * 18446744073709551616.0L);
    }
    for (int attempt = 0; attempt < 128; ++attempt) {
        DTRY(hipMemsetAsync(d->counter, 0, 8, st));
        if (d->timer) d->timer->mark(st);
        DTRY(launch_filter<KeyT>(d, keys, hashes, n, tinc, st));
        if (d->timer) d->timer->mark(st);
        DTRY(hipMemcpyAsync(d->h_pinned + 2, d->counter, 8, hipMemcpyDeviceToHost, st));
        DTRY(hipStreamSynchronize(st));
        const int64_t c = d->h_pinned[2];
        if (c > d->cand_cap) {  // threshold too loose for the candidate buffer: tighten
            if (ns == 0) {
                if (int rc = take_sample()) return rc;
                q = (int64_t)((__int128)(d->cand_limit / 4) * ns / n);
                DTRY(ensure_caps(d, d->cand_limit, 0, st));
            } else {
                q /= 2;
            }
            int64_t t = quantile(q);
            if (t >= tinc) t = tinc - (int64_t)(((uint64_t)tinc - (uint64_t)INT64_MIN) / 2) - 1;
            tinc = t;
            continue;
        }
        int64_t nd = 0;
        DTRY(merge_into_set<KeyT>(d, d->cand_h, (const KeyT*)d->cand_k, c, &nd, st));
        // exact once every batch element below the new k-th hash was a candidate
        if (tinc >= t_allowed || (d->m == d->k && d->max_h <= tinc)) return RSV_OK;
        // too tight: widen (the partial merge is harmless: bottom-k(bottom-k(S u C1) u C2) equals
        // bottom-k(S u C2) for C1 a subset of C2)
        if (ns == 0) {
            if (int rc = take_sample()) return rc;
            q = (int64_t)(std::upper_bound(d->samp_host.begin(), d->samp_host.end(), tinc) - d->samp_host.begin());
        }
        q = q < 16 ? 64 : q * 4;
        int64_t t = quantile(q);
        if (t <= tinc) {  // coarse sample: double the distance from INT64_MIN instead
            const uint64_t span = (uint64_t)tinc - (uint64_t)INT64_MIN;
            t = span >= (uint64_t)t_allowed - (uint64_t)tinc ? t_allowed : (int64_t)((uint64_t)tinc + span + 1);
        }
        tinc = std::min(t, t_allowed);
    }
    set_error("distinct: threshold search did not converge");
    return RSV_E_DEVICE;
#undef DTRY
}

int distinct_sample_device(DistinctState* d, const void* keys, const int64_t* hashes, int64_t n,
                           hipStream_t st) {
    return d->kw == 8 ? sample_impl<int64_t>(d, (const int64_t*)keys, hashes, n, st)
                      : sample_impl<int32_t>(d, (const int32_t*)keys, hashes, n, st);
}

int distinct_export(DistinctState* d, void* keys_dev, int64_t* hash_dev, hipStream_t st) {
    if (d->m == 0) return RSV_OK;
    if (keys_dev) RSV_HIP_TRY(hipMemcpyAsync(keys_dev, d->set_k, d->m * d->kw, hipMemcpyDeviceToDevice, st));
    if (hash_dev) RSV_HIP_TRY(hipMemcpyAsync(hash_dev, d->set_h, d->m * 8, hipMemcpyDeviceToDevice, st));
    return RSV_OK;
}

int distinct_merge(DistinctState* d, const void* keys_dev, const int64_t* hash_dev, int64_t n,
                   hipStream_t st) {
    int64_t off = 0;
    while (off < n) {  // chunks that fit the merge buffer
        const int64_t c = std::min<int64_t>(n - off, d->cand_limit);
        int64_t nd = 0;
        hipError_t e = d->kw == 8
                           ? merge_into_set<int64_t>(d, hash_dev + off, (const int64_t*)keys_dev + off, c, &nd, st)
                           : merge_into_set<int32_t>(d, hash_dev + off, (const int32_t*)keys_dev + off, c, &nd, st);
        if (e != hipSuccess) {
            set_error(std::string("distinct_merge: ") + hipGetErrorString(e));
            return RSV_E_DEVICE;
        }
        off += c;
    }
    return RSV_OK;
}

}  // namespace rsv
