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
#include <cstdio>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <limits>
#include <type_traits>
#include <vector>

#include "../../include/reservoir_hip.h"
#include "rsv_device.h"
#include "rsv_host_values.h"
#include "rsv_internal.h"

namespace rsv {

namespace {

constexpr int kBlock = 256;
constexpr int64_t kSample = 65536;

__device__ __forceinline__ unsigned long long lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Candidate output: staged per wave in LDS and written B at a time, so the global reservation
// counter sees one atomic per B candidates (a single contended word sustains ~88 atomics/us:
// one atomic per candidate cost 1.5 ms at 132k candidates).  IDX: each candidate also carries its
// pass-relative index (the ordered mode's arrival order); its chunks run at ~3k candidates per
// pass, so it stages B = 256 (64: ~35 us of atomics per short chunk).
// Sink (the scheduled pass): also files each written candidate into its merge bucket, so the
// bucket atomics ride under the HBM-bound stream instead of a scatter kernel after it
template <typename KeyT, bool IDX = false, typename Sink = void>
struct CandOut {
    static constexpr uint32_t B = IDX ? 256 : 64;  // batch; the LDS queue holds B + 64
    int64_t* qh;  // LDS: B + 64 hashes of this wave
    KeyT* qk;     // LDS: B + 64 keys
    uint32_t qn;  // wave-uniform fill
    int64_t* cand_h;
    KeyT* cand_k;
    unsigned long long* counter;
    int64_t cap;
    uint32_t* qi = nullptr;      // LDS: B + 64 indices (IDX)
    uint32_t* cand_i = nullptr;  // (IDX)
    Sink* sink = nullptr;

    __device__ __forceinline__ void write64(uint32_t from, uint32_t cnt) {
        const uint32_t lane = threadIdx.x & 63;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(counter, (unsigned long long)cnt);
        base = __shfl(base, 0);
        write_at(base, from, cnt);
    }
    __device__ __forceinline__ void write_at(unsigned long long base, uint32_t from, uint32_t cnt) {
        const uint32_t lane = threadIdx.x & 63;
#pragma unroll
        for (uint32_t j0 = 0; j0 < B; j0 += 64) {
            const uint32_t j = j0 + lane;
            if (j < cnt) {
                const unsigned long long pos = base + j;
                if ((int64_t)pos < cap) {
                    cand_h[pos] = qh[from + j];
                    cand_k[pos] = qk[from + j];
                    if constexpr (IDX) cand_i[pos] = qi[from + j];
                    if constexpr (!std::is_void<Sink>::value) sink->put(qh[from + j], qk[from + j], qi[from + j] + 1u);
                }
            }
        }
    }
    __device__ __forceinline__ void push(bool c, int64_t h, KeyT key, uint32_t idx) {
        const unsigned long long bal = __ballot(c);
        if (bal == 0) return;
        if (c) {
            const uint32_t pos = qn + __popcll(bal & lanemask_lt());
            qh[pos] = h;
            qk[pos] = key;
            if constexpr (IDX) qi[pos] = idx;
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= B) {
            qn -= B;
            __builtin_amdgcn_wave_barrier();
            write64(qn, B);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __device__ __forceinline__ void flush() {
        __builtin_amdgcn_wave_barrier();
        if (qn) write64(0, qn);
        qn = 0;
    }
    // the final flush of every wave of the workgroup under ONE reservation atomic: the counter is
    // a single contended word (~88 atomics/us), and a pass whose waves each end with a few staged
    // candidates (the ordered mode's short chunks) was bound by one atomic per wave
    template <int WAVES>
    __device__ __forceinline__ void flush_block(uint32_t* s_q, unsigned long long* s_base) {
        const uint32_t w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) s_q[w] = qn;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
#pragma unroll
            for (int i = 0; i < WAVES; ++i) tot += s_q[i];
            *s_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t i = 0; i < w; ++i) pre += s_q[i];
        if (qn) write_at(*s_base + pre, 0, qn);
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
// filter bounds: one inclusive bound for the pass, or (the ordered mode's scheduled pass) a bound
// per index range, looked up with a cursor -- a thread's indices only increase between resets
struct ConstBound {
    int64_t t;
    __device__ __forceinline__ int64_t operator()(int64_t) { return t; }
    __device__ __forceinline__ void reset() {}
};

struct RangeBound {
    const int64_t* b;  // LDS: range starts, b[nr] = n
    const int64_t* t;  // LDS: bound of range r
    int r;
    int64_t next, cur;
    __device__ __forceinline__ void reset() {
        r = 0;
        next = b[1];
        cur = t[0];
    }
    __device__ __forceinline__ int64_t operator()(int64_t idx) {
        while (idx >= next) {
            ++r;
            next = b[r + 1];
            cur = t[r];
        }
        return cur;
    }
};

// streaming shape of the filter passes: 16-B loads in flight per lane, workgroups per CU
// (dev builds vary them: make exp EXP="-DRSV_K3_U=16 -DRSV_K3_WGCU=64")
#ifndef RSV_K3_U
#define RSV_K3_U 8
#endif
#ifndef RSV_K3_WGCU
#define RSV_K3_WGCU 32
#endif
constexpr int kK3U = RSV_K3_U;
constexpr int64_t kK3Grid = 256 * RSV_K3_WGCU;

template <typename KeyT, int HASH, int U, bool GUARD, typename Out, typename Bound>
__device__ __forceinline__ void k3_tile(const typename Vec<KeyT>::T* x, int64_t v0, int64_t T, int64_t n_vec,
                                        const KeyT* keys, const int64_t* hashes, int64_t r0, int64_t r1,
                                        Bound& bound, Out& out, uint32_t ioff) {
    using V = Vec<KeyT>;
    int64_t h[U][V::N];
    bool c[U][V::N];
    bool any = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t v = v0 + u * T;
        const bool ok = !GUARD || v < n_vec;
        const int64_t vi = GUARD && !ok ? n_vec - 1 : v;  // the clamped (loaded) vector
#pragma unroll
        for (int e = 0; e < V::N; ++e) {
            h[u][e] = elem_hash<KeyT, HASH>(keys, hashes, vi * V::N + e, V::get(x[u], e), r0, r1);
            c[u][e] = ok & (h[u][e] <= bound((int64_t)ioff + vi * V::N + e));
            any |= c[u][e];
        }
    }
    if (__any(any)) {  // ~1e-4 of the waves at the steady-state threshold
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < V::N; ++e)
                out.push(c[u][e], h[u][e], V::get(x[u], e), ioff + (uint32_t)((v0 + u * T) * V::N + e));
    }
}

// IDX (the ordered mode's chunk pass): candidates also carry their index in [0, n < 2^32).
template <typename KeyT, int HASH, bool IDX, typename Bound, typename Sink = void>
__device__ __forceinline__ void k3_filter_body(const KeyT* __restrict__ keys, const int64_t* __restrict__ hashes,
                                               int64_t n, int64_t r0, int64_t r1, Bound bound,
                                               int64_t* __restrict__ cand_h, KeyT* __restrict__ cand_k,
                                               unsigned long long* __restrict__ counter, int64_t cap,
                                               uint32_t* __restrict__ cand_i, Sink* sink = nullptr) {
    using V = Vec<KeyT>;
    constexpr int U = kK3U;  // 8 x 16-B loads in flight per lane (tools/micro_k3: 6.0 -> 6.4 TB/s vs 4)
    constexpr uint32_t Q = CandOut<KeyT, IDX>::B + 64;
    __shared__ int64_t sh_h[kBlock / 64][Q];
    __shared__ KeyT sh_k[kBlock / 64][Q];
    __shared__ uint32_t sh_i[IDX ? kBlock / 64 : 1][IDX ? Q : 1];
    CandOut<KeyT, IDX, Sink> out{sh_h[threadIdx.x >> 6], sh_k[threadIdx.x >> 6], 0u, cand_h, cand_k, counter, cap};
    if constexpr (IDX) {
        out.qi = sh_i[threadIdx.x >> 6];
        out.cand_i = cand_i;
    }
    out.sink = sink;
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the vector loads start at the first 16-B boundary (a batch may begin anywhere in a tensor);
    // the <= 3 head elements before it go through the scalar loop at the end
    const int64_t head = std::min<int64_t>(n, (int64_t)(((16u - ((uintptr_t)keys & 15u)) & 15u) / sizeof(KeyT)));
    const KeyT* kb = keys + head;
    const int64_t* hb = HASH == kHashPrecomputed ? hashes + head : hashes;
    const int64_t nb = n - head;
    const int64_t n_vec = nb / V::N;
    const typename V::T* kv = reinterpret_cast<const typename V::T*>(kb);
    const int64_t full = n_vec / (T * U);  // whole tiles: every lane has U vectors
    bound.reset();
    for (int64_t it = 0; it < full; ++it) {
        const int64_t v0 = it * T * U + tid;
        typename V::T x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(kv + v0 + u * T);
        k3_tile<KeyT, HASH, U, false>(x, v0, T, n_vec, kb, hb, r0, r1, bound, out, (uint32_t)head);
    }
    if (full * T * U < n_vec) {  // the partial last tile, same shape: out-of-range lanes re-load the
        const int64_t v0 = full * T * U + tid;  // last vector (no guarded loads) and are masked out
        typename V::T x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t v = v0 + u * T;
            x[u] = __builtin_nontemporal_load(kv + (v < n_vec ? v : n_vec - 1));
        }
        k3_tile<KeyT, HASH, U, true>(x, v0, T, n_vec, kb, hb, r0, r1, bound, out, (uint32_t)head);
    }
    // then the head and the nb % V::N tail elements
    bound.reset();
    for (int64_t idx = tid; idx - tid < head; idx += T) {
        const bool ok = idx < head;
        const KeyT key = ok ? keys[idx] : (KeyT)0;
        const int64_t h = ok ? elem_hash<KeyT, HASH>(keys, hashes, idx, key, r0, r1) : 0;
        out.push(ok && h <= bound(ok ? idx : 0), h, key, (uint32_t)idx);
    }
    bound.reset();
    for (int64_t idx = head + n_vec * V::N + tid; idx - tid < n; idx += T) {
        const bool ok = idx < n;
        const KeyT key = ok ? keys[idx] : (KeyT)0;
        const int64_t h = ok ? elem_hash<KeyT, HASH>(keys, hashes, idx, key, r0, r1) : 0;
        out.push(ok && h <= bound(ok ? idx : n - 1), h, key, (uint32_t)idx);
    }
    __shared__ uint32_t s_q[kBlock / 64];
    __shared__ unsigned long long s_base;
    __builtin_amdgcn_wave_barrier();
    out.template flush_block<kBlock / 64>(s_q, &s_base);
}

template <typename KeyT, int HASH, bool IDX = false>
__global__ __launch_bounds__(kBlock) void k3_filter(const KeyT* __restrict__ keys,
                                                    const int64_t* __restrict__ hashes, int64_t n,
                                                    int64_t r0, int64_t r1, int64_t tinc,
                                                    int64_t* __restrict__ cand_h,
                                                    KeyT* __restrict__ cand_k,
                                                    unsigned long long* __restrict__ counter,
                                                    int64_t cap, uint32_t* __restrict__ cand_i = nullptr) {
    k3_filter_body<KeyT, HASH, IDX>(keys, hashes, n, r0, r1, ConstBound{tinc}, cand_h, cand_k, counter, cap, cand_i);
}

// A filter with no bound (the heap still filling): every element is a candidate, so element i is
// written to place i -- no staging, no reservation atomics -- and the counter set to n
// (heap-filling chunk of C4's ordered share, 132k keys: the staged k3_filter took 12.4 us)
template <typename KeyT, int HASH, bool IDX>
__global__ __launch_bounds__(kBlock) void hash_all(const KeyT* __restrict__ keys, const int64_t* __restrict__ hashes,
                                                   int64_t n, int64_t r0, int64_t r1, int64_t* __restrict__ out_h,
                                                   KeyT* __restrict__ out_k, uint32_t* __restrict__ out_i,
                                                   unsigned long long* __restrict__ counter) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const KeyT key = keys[i];
        out_h[i] = elem_hash<KeyT, HASH>(keys, hashes, i, key, r0, r1);
        out_k[i] = key;
        if constexpr (IDX) out_i[i] = (uint32_t)i;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *counter = (unsigned long long)n;  // re-armed to 0 by read_ctl
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
    // rank k ties with rank k - 1 on h: the maximum's bucket holds more distinct elements than the
    // set keeps (entry p - 1 is rank k - 1 or one of its duplicates)
    if (flags[p] && (int64_t)pos[p] == k && p > 0 && h[p - 1] == h[p]) out_count[2] = 1;
    if (p == n - 1) {
        const int64_t nd = (int64_t)pos[p] + (int64_t)flags[p];
        out_count[0] = nd;
        if (nd <= k) out_count[1] = h[p];  // the set's largest hash (its duplicates share it)
    }
}

// ---- bucketed merge (set mode, typical k) ------------------------------------------------------
// set + candidates -> buckets by h (the scrambled hash is uniform; bucket b covers the b-th of B
// equal parts of the span, B = 2^lb >= total / 128, so buckets hold ~64-128 entries) -> one wave
// per bucket sorts by (h, key) in registers (bitonic network over cross-lane shuffles, no LDS, no
// barriers) and drops duplicates -> each bucket's distinct entries land at their global rank; the
// first k are the new set.  Three dispatches sized from counts read on the device: no host round
// trip between the filter and the merge, no radix-sort passes.  A bucket above kBucketCap entries
// (a degenerate precomputed hash) sets the overflow word and the host reruns the merge on the
// radix-sort path.
//   ctl: [0] filter candidate counter  [1] overflow  [2] distinct count  [3] largest kept h
//        [4] publication ticket  [5] tie at the boundary (rank k has rank k - 1's h)  [6..7] unused
//        then (uint32, from ctl + 8) bucket_count[b] at b * 32 (one 128-B line each: the scatter's
//        atomics on neighbouring counters would serialise on a shared line), bucket_distinct[b] at
//        bmax * 32 + b.  bucket_sort re-zeroes the counts it consumed, so only ctl[0..1] are cleared
//        per pass (and the counts after an overflow).
constexpr uint32_t kBucketCap = 256;  // 4 entries per lane of the sorting wave
constexpr uint32_t kBucketAvgLog = 7;
constexpr uint32_t kCountStride = 32;
constexpr int kCtlWords = 8;

__device__ __forceinline__ uint32_t* bucket_count(int64_t* ctl) { return (uint32_t*)(ctl + kCtlWords); }
__device__ __forceinline__ uint32_t* bucket_distinct(int64_t* ctl, int32_t log_bmax) {
    return (uint32_t*)(ctl + kCtlWords) + ((size_t)kCountStride << log_bmax);
}

// per-16-bucket sums of the distinct counts (bucket_sort adds, bucket_emit reads): an emit
// workgroup's rank base is then B / 16 group sums + <= 15 bucket counts instead of every bucket
// (groups of 256 put 256 same-address atomics in line: bucket_sort 9 -> 28 us at 4096 buckets)
__device__ __forceinline__ uint32_t* bucket_group(int64_t* ctl, int32_t log_bmax) {
    return (uint32_t*)(ctl + kCtlWords) + ((size_t)(kCountStride + 1) << log_bmax);
}
__device__ __forceinline__ void zero_bucket_groups(int64_t* ctl, int32_t log_bmax) {
    uint32_t* gs = bucket_group(ctl, log_bmax);
    for (uint32_t i = threadIdx.x; i <= ((1u << log_bmax) >> 4); i += blockDim.x) gs[i] = 0;
}

__device__ __forceinline__ uint32_t bucket_log(int64_t total, int32_t log_bmax) {
    uint32_t lb = 0;
    while ((int32_t)lb < log_bmax && ((int64_t)1 << (lb + kBucketAvgLog)) < total) ++lb;
    return lb;
}

// Bucket of u = h - INT64_MIN in [0, span]: floor(u * B / (span + 1)) as umulhi(u, q * B) with
// q = floor((2^64 - 1) / (span + 1)) (host), monotone in u; a span below B buckets directly.
struct BucketMap {
    uint64_t mult;  // 0: b = u
    uint32_t last;
    __device__ __forceinline__ BucketMap(uint64_t q, uint32_t lb) {
        last = (1u << lb) - 1u;
        mult = (lb == 0) ? 0ull : ((q >> (64 - lb)) ? 0ull : q << lb);
        if (lb == 0) last = 0;
    }
    __device__ __forceinline__ uint32_t operator()(int64_t h) const {
        const uint64_t u = (uint64_t)h ^ 0x8000000000000000ull;
        const uint64_t b = mult ? __umul64hi(u, mult) : (last ? u : 0ull);
        return (uint32_t)(b < last ? b : last);  // an entry above the span sorts after every bucket
    }
};

template <typename KeyT>
__device__ __forceinline__ bool ent_less(int64_t ha, KeyT ka, int64_t hb, KeyT kb) {
    return ha < hb || (ha == hb && ka < kb);
}

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void bucket_scatter(const int64_t* __restrict__ set_h,
                                                         const KeyT* __restrict__ set_k, int64_t m,
                                                         const int64_t* __restrict__ cand_h,
                                                         const KeyT* __restrict__ cand_k, int64_t cand_cap,
                                                         int64_t* __restrict__ ctl, uint64_t q,
                                                         int32_t log_bmax, int64_t* __restrict__ bh,
                                                         KeyT* __restrict__ bk) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) ctl[5] = 0;  // bucket_emit sets it
        zero_bucket_groups(ctl, log_bmax);
    }
    const int64_t c = ctl[0];
    if (c > cand_cap) return;  // the filter overflowed its buffer: the host tightens and reruns
    const int64_t total = m + c;
    const BucketMap map(q, bucket_log(total, log_bmax));
    uint32_t* bcnt = bucket_count(ctl);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        int64_t h;
        KeyT key;
        if (i < m) {
            h = set_h[i];
            key = set_k[i];
        } else {
            h = cand_h[i - m];
            key = cand_k[i - m];
        }
        const uint32_t b = map(h);
        const uint32_t p = atomicAdd(&bcnt[(size_t)b * kCountStride], 1u);
        if (p < kBucketCap) {
            bh[(size_t)b * kBucketCap + p] = h;
            bk[(size_t)b * kBucketCap + p] = key;
        } else {
            ctl[1] = 1;
        }
    }
}

template <typename T>
__device__ __forceinline__ T shfl_xor_any(T v, int mask) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t x = (uint64_t)v;
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, mask);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), mask);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__shfl_xor((int)v, mask);
    }
}

template <typename T>
__device__ __forceinline__ T shfl_any(T v, int src) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t x = (uint64_t)v;
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, src);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), src);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__shfl((int)v, src);
    }
}

// One wave per bucket: entry i = r * 64 + lane lives in register slot r of `lane` (R slots).
// Bitonic network: strides >= 64 swap between a lane's own slots, smaller ones exchange with lane
// ^ stride; then the first of each run of equal entries is kept and written back compacted;
// bucket_distinct[b] = their number.
// The one-register bucket (n <= 64) sorted on ONE 64-bit word per lane: (h - min h) << 6 | lane,
// when the bucket's hashes span < 2^58 (a merge bucket covers a narrow slice of the hash range:
// always, in practice; else the caller runs the full network).  The 21 compare-exchange stages then
// move 2 words instead of 5 (h, key, tag) and compare once; the entries are re-read by their slot
// after it, and runs of equal h (duplicates, colliding hashes) are put in (key, tag) order by an
// odd-even transposition restricted to the run.  In: this lane's entry (lane < n; others MAX).
template <typename KeyT, bool TAGGED, typename Load>
__device__ __forceinline__ bool wave_packed_sort(const Load& load, uint32_t n, int64_t& h, KeyT& k, uint32_t& g) {
    const uint32_t lane = threadIdx.x & 63;
    const bool valid = lane < n;
    const uint64_t u = (uint64_t)h ^ 0x8000000000000000ull;
    uint64_t lo = valid ? u : ~0ull;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = xor_any(lo, d);
        lo = o < lo ? o : lo;
    }
    if (__ballot(valid && ((u - lo) >> 58) != 0)) return false;
    uint64_t key = valid ? ((u - lo) << 6) | lane : ~0ull;
#pragma unroll
    for (uint32_t size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            const uint64_t o = xor_any(key, (int)stride);
            const bool lower = (lane & stride) == 0;
            const bool up = (lane & size) == 0;
            const bool take = (lower == up) ? (o < key) : (key < o);
            key = take ? o : key;
        }
    }
    if (valid) load((uint32_t)key & 63u, h, k, g);
    for (;;) {
        bool any = false;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            int partner = p == 0 ? (int)(lane ^ 1u) : ((lane & 1u) ? (int)lane + 1 : (int)lane - 1);
            if (partner < 0 || partner > 63) partner = (int)lane;
            const int64_t oh = shfl_any(h, partner);
            const KeyT ok = shfl_any(k, partner);
            const uint32_t og = TAGGED ? (uint32_t)__shfl((int)g, partner) : 0u;
            bool sw = false;
            if (valid && (uint32_t)partner < n && partner != (int)lane && oh == h) {
                const bool other_less = ok < k || (TAGGED && ok == k && og < g);
                const bool mine_less = k < ok || (TAGGED && k == ok && g < og);
                sw = (int)lane < partner ? other_less : mine_less;
            }
            if (sw) {
                k = ok;
                g = og;
            }
            any |= sw;
        }
        if (!__ballot(any)) break;
    }
    return true;
}

// entries (h, key) read in place (bucket_sort, rows_sort)
template <typename KeyT>
struct PairSrc {
    const int64_t* h;
    const KeyT* k;
    __device__ __forceinline__ void load(uint32_t i, int64_t& hh, KeyT& kk) const {
        hh = h[i];
        kk = k[i];
    }
};

template <typename KeyT, int R, typename Src>
__device__ __forceinline__ uint32_t wave_sort_bucket(const Src src, int64_t* gh, KeyT* gk, uint32_t n,
                                                     uint32_t* out_cnt) {
    const uint32_t lane = threadIdx.x & 63;
    constexpr uint32_t N = 64u * R;
    int64_t h[R];
    KeyT k[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * 64u + lane;
        if (i < n) {
            src.load(i, h[r], k[r]);
        } else {
            h[r] = INT64_MAX;
            k[r] = std::numeric_limits<KeyT>::max();
        }
    }
    bool packed = false;
    if constexpr (R == 1) {
        uint32_t g0 = 0;
        packed = wave_packed_sort<KeyT, false>(
            [&](uint32_t i, int64_t& hh, KeyT& kk, uint32_t&) { src.load(i, hh, kk); }, n, h[0], k[0], g0);
    }
    if (!packed) {
#pragma unroll
    for (uint32_t size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {
                const uint32_t rs = stride / 64;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if ((r & rs) == 0) {
                        const uint32_t i = r * 64u + lane;
                        const bool up = (i & size) == 0;
                        const int r2 = r + rs;
                        if (ent_less<KeyT>(h[r2], k[r2], h[r], k[r]) == up) {
                            const int64_t th = h[r];
                            const KeyT tk = k[r];
                            h[r] = h[r2];
                            k[r] = k[r2];
                            h[r2] = th;
                            k[r2] = tk;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t i = r * 64u + lane;
                    const int64_t oh = xor_any(h[r], (int)stride);
                    const KeyT ok = xor_any(k[r], (int)stride);
                    const bool lower = (lane & stride) == 0;
                    const bool up = (i & size) == 0;
                    // the lower lane keeps the smaller entry in an ascending run, the larger otherwise
                    const bool other_less = ent_less<KeyT>(oh, ok, h[r], k[r]);
                    const bool mine_less = ent_less<KeyT>(h[r], k[r], oh, ok);
                    const bool take = (lower == up) ? other_less : mine_less;
                    if (take) {
                        h[r] = oh;
                        k[r] = ok;
                    }
                }
            }
        }
    }
    }  // !packed
    // distinct: entry i differs from entry i - 1
    uint32_t base = 0;
    int64_t prev_h_last = 0;
    KeyT prev_k_last = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * 64u + lane;
        int64_t ph = shfl_any(h[r], (int)((lane + 63) & 63));
        KeyT pk = shfl_any(k[r], (int)((lane + 63) & 63));
        if (lane == 0) {
            ph = prev_h_last;
            pk = prev_k_last;
        }
        const bool first = i < n && (i == 0 || ph != h[r] || pk != k[r]);
        const unsigned long long bal = __ballot(first);
        if (first) {
            const uint32_t o = base + (uint32_t)__popcll(bal & lanemask_lt());
            gh[o] = h[r];
            gk[o] = k[r];
        }
        base += (uint32_t)__popcll(bal);
        prev_h_last = shfl_any(h[r], 63);
        prev_k_last = shfl_any(k[r], 63);
    }
    if (lane == 0) *out_cnt = base;
    return base;
}

template <typename KeyT, int R>
__device__ __forceinline__ uint32_t wave_sort_bucket(int64_t* gh, KeyT* gk, uint32_t n, uint32_t* out_cnt) {
    return wave_sort_bucket<KeyT, R>(PairSrc<KeyT>{gh, gk}, gh, gk, n, out_cnt);
}

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void bucket_sort(int64_t m, int64_t cand_cap, int64_t* __restrict__ ctl,
                                                      int32_t log_bmax, int64_t* __restrict__ bh,
                                                      KeyT* __restrict__ bk) {
    const int64_t c = ctl[0];
    if (c > cand_cap || ctl[1]) return;
    const uint32_t lb = bucket_log(m + c, log_bmax);
    const uint32_t b = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (b >= (1u << lb)) return;
    uint32_t* bcnt = bucket_count(ctl) + (size_t)b * kCountStride;
    uint32_t* bdist = bucket_distinct(ctl, log_bmax) + b;
    const uint32_t n = *bcnt;
    int64_t* gh = bh + (size_t)b * kBucketCap;
    KeyT* gk = bk + (size_t)b * kBucketCap;
    if (n == 0) {
        if ((threadIdx.x & 63) == 0) *bdist = 0;
        return;
    }
    const uint32_t nd = n <= 64    ? wave_sort_bucket<KeyT, 1>(gh, gk, n, bdist)
                        : n <= 128 ? wave_sort_bucket<KeyT, 2>(gh, gk, n, bdist)
                                   : wave_sort_bucket<KeyT, 4>(gh, gk, n, bdist);
    if ((threadIdx.x & 63) == 0) atomicAdd(bucket_group(ctl, log_bmax) + (b >> 4), nd);
    if ((threadIdx.x & 63) == 0) *bcnt = 0;  // consumed (n was read before the sort's loads); re-armed
}

// each bucket's distinct entries to their global rank (ranks < k) in the set arrays.  A workgroup
// covers kEmitBuckets consecutive buckets: their rank base is the sum of the distinct counts before
// them (one strided pass over bucket_distinct per workgroup), then one wave per 4 buckets copies.
constexpr uint32_t kEmitBuckets = 16;

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void bucket_emit(int64_t m, int64_t cand_cap, int64_t* __restrict__ ctl,
                                                      int32_t log_bmax, const int64_t* __restrict__ bh,
                                                      const KeyT* __restrict__ bk, int64_t k,
                                                      int64_t* __restrict__ set_h, KeyT* __restrict__ set_k,
                                                      int32_t lb_fixed = -1) {
    __shared__ uint64_t s_pre[kBlock / 64], s_tot[kBlock / 64];
    __shared__ uint64_t s_base[kEmitBuckets + 1];
    const int64_t c = ctl[0];
    if (c > cand_cap || ctl[1]) return;
    const uint32_t lb = lb_fixed >= 0 ? (uint32_t)lb_fixed : bucket_log(m + c, log_bmax);
    const uint32_t B = 1u << lb;
    const uint32_t b0 = blockIdx.x * kEmitBuckets;
    if (b0 >= B) return;
    const uint32_t* bdist = bucket_distinct(ctl, log_bmax);
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t* gsum = bucket_group(ctl, log_bmax);
    const uint32_t G = (B + 15) >> 4, g0 = b0 >> 4;
    uint64_t pre = 0, tot = 0;
    for (uint32_t i = t; i < G; i += kBlock) {
        const uint64_t v = gsum[i];
        tot += v;
        if (i < g0) pre += v;
    }
    for (uint32_t i = (g0 << 4) + t; i < b0; i += kBlock) pre += bdist[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        pre += shfl_xor_any(pre, off);
        tot += shfl_xor_any(tot, off);
    }
    if (lane == 0) {
        s_pre[w] = pre;
        s_tot[w] = tot;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t p = 0, q = 0;
        for (int i = 0; i < kBlock / 64; ++i) {
            p += s_pre[i];
            q += s_tot[i];
        }
        const uint32_t nb = std::min<uint32_t>(kEmitBuckets, B - b0);
        for (uint32_t i = 0; i < nb; ++i) {
            s_base[i] = p;
            p += bdist[b0 + i];
        }
        s_base[kEmitBuckets] = q;
        if (b0 == 0) ctl[2] = (int64_t)q;
    }
    __syncthreads();
    tot = s_base[kEmitBuckets];
    const uint64_t mk = std::min<uint64_t>(tot, (uint64_t)k);
    for (uint32_t j = 0; j < kEmitBuckets / (kBlock / 64); ++j) {
        const uint32_t bi = w * (kEmitBuckets / (kBlock / 64)) + j;
        const uint32_t b = b0 + bi;
        if (b >= B) break;
        const uint64_t base = s_base[bi];
        if (base >= (uint64_t)k) break;  // later buckets rank higher still
        const uint32_t cnt = bdist[b];
        const int64_t* gh = bh + (size_t)b * kBucketCap;
        const KeyT* gk = bk + (size_t)b * kBucketCap;
        for (uint32_t r = lane; r < cnt; r += 64) {
            const uint64_t rank = base + r;
            if (rank < (uint64_t)k) {
                set_h[rank] = gh[r];
                set_k[rank] = gk[r];
                if (rank + 1 == mk) ctl[3] = gh[r];
            } else if (rank == (uint64_t)k && r > 0 && gh[r - 1] == gh[r]) {
                ctl[5] = 1;  // equal h share a bucket (the map is monotone): rank k - 1 is entry r - 1
            }
        }
    }
}

// ---- ordered mode: the scheduled pass ---------------------------------------------------------
// Once the heap is full, the rest of a long batch is filtered in ONE pass whose bound is fixed ahead
// per index range: range r = [b[r], b[r+1]) keeps h <= t[r], t[0] = the current bound (exact) and
// t[r] for r >= 1 predicted from the hash's uniformity (SchedPlan, host).  The pass keeps a
// superset of what the reference admits iff every predicted bound is at least the true one at its
// range's start, i.e. iff at least k distinct elements that arrived before b[r] have h <= t[r].
// The merge verifies exactly that: it dedups the candidates by (h, key), keeps each element's
// first arrival, and counts, per range, the distinct elements that arrived before it with h under
// its bound (an element counts for the ranges r_a(arrival) .. r_h(h): a difference array).  A
// failed range (or a full buffer) leaves the batch to the chunk loop with the set restored.
constexpr int kMaxRanges = 64;
constexpr int kVerifyCopies = 64;  // verification accumulators (spread the sort kernel's atomics)

struct SchedDev {
    int64_t b[kMaxRanges + 1];  // range starts (batch-relative), b[nr] = n
    int64_t t[kMaxRanges];      // inclusive bound per range, non-increasing
    int32_t nr;                 // ranges
    uint32_t B, B_lo;           // merge buckets; the first B_lo map h <= t[nr - 1] linearly
    uint32_t lb;                // log2 B
    uint64_t lo_mult;           // low region: bucket = umulhi(h - MIN, lo_mult * B_lo)
    float hi_a[kMaxRanges];     // high region, piece p (t[p + 1] < h <= t[p]): pos = a u + c, u = (h - MIN) / 2^64
    float hi_c[kMaxRanges];
    int64_t off;                // the pass's log entries start `off` past the base it is given
};

// bucket of h for the scheduled merge: B_lo buckets map [MIN, t_lo] linearly (monotone: the
// final set and its tie lie there), the rest map (t_lo, t[0]] by the entries' expected cumulative
// count (piecewise linear in h; only balance matters there)
struct SchedMap {
    const SchedDev* sd;
    const int64_t* st;  // LDS copy of sd->t
    uint32_t B, B_lo, nr;
    int64_t t_lo;
    uint64_t lo_mult;
    __device__ __forceinline__ uint32_t operator()(int64_t h) const {
        const uint64_t u = (uint64_t)h ^ 0x8000000000000000ull;
        if (h <= t_lo) return std::min<uint32_t>(B_lo - 1, (uint32_t)__umul64hi(u, lo_mult));
        // piece p = the last range with t[p] >= h (t non-increasing; the set's top sits at t[0] + 1),
        // by a fixed six-step search (nr <= 64; h > t[nr - 1] here, so p < nr - 1)
        int lo = 0;
#pragma unroll
        for (int step = 32; step; step >>= 1) {
            const int q = lo + step;
            lo = (q < (int)nr - 1 && st[q < kMaxRanges ? q : kMaxRanges - 1] >= h) ? q : lo;
        }
        const float pos = sd->hi_a[lo] * (float)((double)u * 5.421010862427522e-20) + sd->hi_c[lo];
        const uint32_t bh = (uint32_t)std::max(0.0f, pos * (float)(B - B_lo));
        return B_lo + std::min(B - B_lo - 1, bh);
    }
};

template <typename KeyT>
struct SchedSink {
    SchedMap map;
    uint32_t* bcnt;
    int64_t* bh;
    KeyT* bk;
    uint32_t* bi;
    int64_t* ovf;
    __device__ __forceinline__ void put(int64_t h, KeyT key, uint32_t tag) {
        const uint32_t b = map(h);
        const uint32_t at = atomicAdd(&bcnt[(size_t)b * kCountStride], 1u);
        if (at < kBucketCap) {
            bh[(size_t)b * kBucketCap + at] = h;
            bk[(size_t)b * kBucketCap + at] = key;
            bi[(size_t)b * kBucketCap + at] = tag;
        } else {
            *ovf = 1;
        }
    }
};

// the scheduled pass: logs the candidates (with their batch index) for the merge and the replica.
// The merge buckets are filled by sched_file after it: filed inside the pass, every candidate batch
// held its wave on the bucket atomics between streaming loads (C4 share: 790 us with the filing,
// 696 us without, rocprof kernel stats; sched_file takes the filing off the streaming path).
template <typename KeyT, int HASH>
__global__ __launch_bounds__(kBlock) void sched_filter(const KeyT* __restrict__ keys, const int64_t* __restrict__ hashes,
                                                       int64_t n, int64_t r0, int64_t r1, const SchedDev* __restrict__ sd,
                                                       int64_t* __restrict__ cand_h, KeyT* __restrict__ cand_k,
                                                       uint32_t* __restrict__ cand_i, int64_t* __restrict__ ctl,
                                                       int64_t cap, int32_t log_bmax, int* __restrict__ vacc_zero) {
    __shared__ int64_t sb[kMaxRanges + 1], stt[kMaxRanges];
    if (vacc_zero) {  // freshly allocated merge area (the fused pass; ctl_plan zeroed the ctl words)
        const size_t words = (size_t)kCountStride << log_bmax, stride = (size_t)gridDim.x * blockDim.x;
        uint32_t* cnt = bucket_count(ctl);
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) cnt[i] = 0;
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)kVerifyCopies * (kMaxRanges + 1);
             i += stride)
            vacc_zero[i] = 0;
    }
    const int nr = sd->nr;
    if (nr < 2) return;  // no pass (ctl_plan found none)
    // (the plan is NOT a kernel argument: 8192 workgroups reading ~1.6 KB of kernarg memory each
    // made the pass 709 -> 769 us; a device copy, read through L2, costs one small copy dispatch)
    if (blockIdx.x == 0) {  // the merge's tie word and group sums (bucket_sort adds, bucket_emit sets)
        if (threadIdx.x == 0) ctl[5] = 0;
        zero_bucket_groups(ctl, log_bmax);
    }
    for (int i = threadIdx.x; i <= nr; i += blockDim.x) {
        sb[i] = sd->b[i];
        if (i < nr) stt[i] = sd->t[i];
    }
    __syncthreads();
    RangeBound rb{sb, stt, 0, 0, 0};
    const int64_t off = sd->off;
    k3_filter_body<KeyT, HASH, true>(keys, hashes, n, r0, r1, rb, cand_h + off, cand_k + off, (unsigned long long*)ctl,
                                     cap, cand_i + off);
}

// the scheduled merge's bucket filing, after the pass: the set's members (tag 0; backed up first,
// restored if a bound fails verification) and the pass's logged candidates (tag 1 + batch index,
// their count from the pass's counter ctl[0], at most cap).  Grid-stride over all of them.
// ---- the plan (host: sched_sample; device: ctl_plan, the fused first chunk + pass) ------------
__host__ __device__ inline double sched_ufrac(int64_t t) {  // fraction of the hash range at or below t
    return ((double)((uint64_t)t - (uint64_t)INT64_MIN) + 1.0) / 18446744073709551616.0;
}
__host__ __device__ inline int64_t sched_bound_at(double frac) {  // largest t with ufrac(t) <= frac
    if (frac >= 1.0) return INT64_MAX;
    const double x = floor(frac * 18446744073709551616.0) - 1.0;
    return x < 0 ? INT64_MIN : (int64_t)((uint64_t)x ^ 0x8000000000000000ull);
}

// Range starts and bounds of a pass over n elements after S0 seen, current bound t0 (see
// sched_sample); returns the expected candidate count, or -1 for fewer than two ranges.
__host__ __device__ inline double sched_plan_ranges(SchedDev* sp, double S0, int64_t t0, int64_t n, int64_t k,
                                                    double beta) {
    S0 = S0 > 1.0 ? S0 : 1.0;
    const double D0 = fmax((double)k, (double)k / sched_ufrac(t0));
    const double dfr = fmin(1.0, fmax(0.5, D0 / S0));
    const double g = fmax(1.08, pow((S0 + (double)n) / S0, 1.0 / (kMaxRanges - 2)));
    int nr = 0;
    sp->b[0] = 0;
    sp->t[0] = t0;
    for (double P = S0 * g;; P *= g) {
        ++nr;
        int64_t bn = ((int64_t)(P - S0) + 15) & ~(int64_t)15;
        if (bn >= n - 16 || nr == kMaxRanges) {
            sp->b[nr] = n;
            break;
        }
        bn = bn > sp->b[nr - 1] + 16 ? bn : sp->b[nr - 1] + 16;
        sp->b[nr] = bn;
        const double D = D0 + dfr * (double)bn;
        const int64_t tb = sched_bound_at(beta * (double)k / D);
        sp->t[nr] = tb < sp->t[nr - 1] ? tb : sp->t[nr - 1];
    }
    sp->nr = nr;
    if (nr < 2) return -1.0;
    double c_pred = 0;
    for (int r = 0; r < nr; ++r) c_pred += (double)(sp->b[r + 1] - sp->b[r]) * fmin(1.0, sched_ufrac(sp->t[r]));
    return c_pred;
}

// The merge's bucket map for 2^lb buckets.  Its entries are uniform in h below their range's
// bound: F(h) = sum_r len_r min(u, u_r) (u = fraction of the hash range below h); the set's k
// members count as range 0 elements (uniform below t[0]: k / u_0 of them per unit of u)
__host__ __device__ inline void sched_plan_map(SchedDev* sp, int64_t k, int32_t lb) {
    const int nr = sp->nr;
    auto flen = [&](int r) {
        return (double)(sp->b[r + 1] - sp->b[r]) + (r == 0 ? (double)k / sched_ufrac(sp->t[0]) : 0.0);
    };
    double F_top = 0, L_all = 0;
    for (int r = 0; r < nr; ++r) {
        F_top += flen(r) * sched_ufrac(sp->t[r]);
        L_all += flen(r);
    }
    sp->lb = (uint32_t)lb;
    sp->B = 1u << lb;
    const int64_t t_lo = sp->t[nr - 1];
    const double F_lo = L_all * sched_ufrac(t_lo);
    const double lo_frac = fmin(0.9, fmax(0.02, F_lo / F_top));
    const uint32_t blo = (uint32_t)(lo_frac * sp->B);
    sp->B_lo = blo < 1 ? 1u : (blo > sp->B - 1 ? sp->B - 1 : blo);
    const uint64_t span_lo = (uint64_t)t_lo - (uint64_t)INT64_MIN;
    sp->lo_mult = span_lo == UINT64_MAX ? 1ull : UINT64_MAX / (span_lo + 1);
    const double inv = 1.0 / fmax(F_top - F_lo, 1e-30);
    double A = 0, FU = 0;  // piece p: A = sum_{r <= p} len_r, and the ranges above it at their bounds
    for (int p = 0; p + 1 < nr; ++p) {
        A += flen(p);
        FU += flen(p) * sched_ufrac(sp->t[p]);
        sp->hi_a[p] = (float)(A * inv);
        sp->hi_c[p] = (float)((F_top - FU - F_lo) * inv);
    }
}

// wave-wide inclusive scans / reductions (one wave; every lane takes part)
template <typename T, typename F>
__device__ __forceinline__ T wave_scan(T v, F op) {
    const int lane = threadIdx.x & 63;
    for (int d = 1; d < 64; d <<= 1) {
        const T o = __shfl_up(v, d);
        if (lane >= d) v = op(v, o);
    }
    return v;
}

// The fused first chunk's control words to the host (as ctl_publish) AND, from them, the plan of the
// scheduled pass over the rest of the batch into `out`.  The first chunk is the heap-filling one; the
// host would otherwise read these words back, plan on the host and only then launch the pass (~18 us
// of idle GPU, rocprof timeline r03).  The plan is sched_plan_ranges + sched_plan_map with lane r
// computing range r: its start is 16 r + the prefix max of (bn_j - 16 j) (= the host's running
// max(bn, b[r - 1] + 16)), its bound a prefix min, the map's sums prefix sums (one thread doing the
// host loops took 352 us).  No pass (out->nr = 0, and the pass's overflow word set so that its sort
// and emit skip) unless the chunk merged on the device with the heap full and the plan fits the
// buffers prepared for it (cap entries, 2^lb buckets).
__global__ __launch_bounds__(64) void ctl_plan(int64_t* __restrict__ ctl, int64_t* dst, uint32_t* flag, uint32_t gen,
                                               int64_t cand_cap, int64_t k, double S0, int64_t n, double beta,
                                               int64_t cap, int32_t lb, SchedDev* __restrict__ out,
                                               int64_t* __restrict__ sctl, int zero) {
    const int r = threadIdx.x;  // 64 lanes = kMaxRanges
    if (zero && r < kCtlWords) sctl[r] = 0;  // a fresh merge area (sched_filter zeroes its counts)
    int64_t v[6];
    for (int i = 0; i < 6; ++i) v[i] = ctl[i];
    if (r < 6) dst[r] = v[r];
    __syncthreads();
    if (r < 2) ctl[r] = 0;
    int nr = 0;
    int64_t br = 0, tr = 0;
    bool ok = v[0] <= cand_cap && v[1] == 0 && v[2] >= k && v[3] != INT64_MIN;
    double fl = 0, ur = 0;
    if (ok) {
        S0 = fmax(S0, 1.0);
        const int64_t t0 = v[3] - 1;
        const double D0 = fmax((double)k, (double)k / sched_ufrac(t0));
        const double dfr = fmin(1.0, fmax(0.5, D0 / S0));
        const double g = fmax(1.08, pow((S0 + (double)n) / S0, 1.0 / (kMaxRanges - 2)));
        const int64_t bn = r == 0 ? 0 : (((int64_t)(S0 * pow(g, (double)r) - S0) + 15) & ~(int64_t)15);
        const uint64_t ends = __ballot(r >= 1 && bn >= n - 16);
        nr = ends ? __ffsll((unsigned long long)ends) - 1 : kMaxRanges;
        br = wave_scan<long long>(bn - 16 * r, [](long long a, long long b) { return a > b ? a : b; }) + 16 * r;
        if (r >= nr) br = n;
        const int64_t tb = r == 0 ? t0 : sched_bound_at(beta * (double)k / (D0 + dfr * (double)br));
        tr = wave_scan<long long>(r < nr ? tb : INT64_MAX, [](long long a, long long b) { return a < b ? a : b; });
        const int64_t bnext = __shfl_down((long long)br, 1);  // read only where r + 1 < nr
        ur = sched_ufrac(tr);
        const double len = r < nr ? (double)((r + 1 == nr ? n : bnext) - br) : 0.0;
        double cp = len * fmin(1.0, ur);
        for (int d = 32; d; d >>= 1) cp += __shfl_xor(cp, d);
        ok = nr >= 2 && 1.5 * cp + 4 * 4096 <= (double)cap;
        fl = len + (r == 0 ? (double)k / sched_ufrac(t0) : 0.0);  // the set's members count as range 0
    }
    if (__ballot(ok) != ~0ull) ok = false;
    if (!ok) {
        if (r == 0) out->nr = 0;
        if (r == 1) sctl[1] = 1;  // the pass's sort and emit skip too (sched_publish re-arms it)
        publish_flag(flag, gen);
        return;
    }
    // the bucket map (sched_plan_map)
    double fu = fl * ur, F_top = fu, L_all = fl;
    for (int d = 32; d; d >>= 1) {
        F_top += __shfl_xor(F_top, d);
        L_all += __shfl_xor(L_all, d);
    }
    const int64_t t_lo = __shfl(tr, nr - 1);
    const double F_lo = L_all * sched_ufrac(t_lo);
    const double inv = 1.0 / fmax(F_top - F_lo, 1e-30);
    const double A = wave_scan<double>(fl, [](double a, double b) { return a + b; });
    const double FU = wave_scan<double>(fu, [](double a, double b) { return a + b; });
    if (r + 1 < nr) {
        out->hi_a[r] = (float)(A * inv);
        out->hi_c[r] = (float)((F_top - FU - F_lo) * inv);
    }
    if (r <= nr) out->b[r] = br;
    if (r == 63 && nr == kMaxRanges) out->b[kMaxRanges] = n;
    if (r < nr) out->t[r] = tr;
    if (r == 0) {
        out->nr = nr;
        const uint32_t B = 1u << lb;
        out->lb = (uint32_t)lb;
        out->B = B;
        const double lo_frac = fmin(0.9, fmax(0.02, F_lo / F_top));
        const uint32_t blo = (uint32_t)(lo_frac * B);
        out->B_lo = blo < 1 ? 1u : (blo > B - 1 ? B - 1 : blo);
        const uint64_t span_lo = (uint64_t)t_lo - (uint64_t)INT64_MIN;
        out->lo_mult = span_lo == UINT64_MAX ? 1ull : UINT64_MAX / (span_lo + 1);
        out->off = v[0];  // behind the chunk's own candidates in the log
    }
    publish_flag(flag, gen);
}

// the plan into device memory: one workgroup copies its by-value argument (the first, so it starts
// the kernarg segment; &plan would copy it to scratch).  Cheaper than hipMemcpyAsync from pinned
// memory, whose host call held the pass back by ~20 us (rocprof timeline, C4 ordered)
__global__ __launch_bounds__(256) void sched_plan_store(const SchedDev plan, SchedDev* __restrict__ out) {
    (void)plan;
    static_assert(sizeof(SchedDev) % 4 == 0, "SchedDev copied as words");
    const uint32_t* src = (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
    for (uint32_t i = threadIdx.x; i < sizeof(SchedDev) / 4; i += blockDim.x) ((uint32_t*)out)[i] = src[i];
}

template <typename KeyT>
__device__ __forceinline__ bool ent_less3(int64_t ha, KeyT ka, uint32_t ia, int64_t hb, KeyT kb, uint32_t ib) {
    return ha < hb || (ha == hb && (ka < kb || (ka == kb && ia < ib)));
}

// one wave per bucket: sort by (h, key, tag), keep the first of each (h, key) run (its earliest
// arrival), write them back compacted; each kept element adds +1 / -1 at ranges r_a / r_h + 1 of
// the block's difference array (sdiff, LDS)
// a bucket's entries in place in global memory (sched_sort)
template <typename KeyT>
struct BucketSrc {
    const int64_t* h;
    const KeyT* k;
    const uint32_t* g;
    __device__ __forceinline__ void load(uint32_t i, int64_t& hh, KeyT& kk, uint32_t& gg) const {
        hh = h[i];
        kk = k[i];
        gg = g[i];
    }
};

// a fine bucket of a coarse bin staged in LDS, through the bin's permutation (sched_bin_sort)
template <typename KeyT>
struct LdsBinSrc {
    const int64_t* h;
    const KeyT* k;
    const uint32_t* g;
    const uint16_t* perm;
    __device__ __forceinline__ void load(uint32_t i, int64_t& hh, KeyT& kk, uint32_t& gg) const {
        const uint32_t p = perm[i];
        hh = h[p];
        kk = k[p];
        gg = g[p];
    }
};

template <typename KeyT, int R, typename Src>
__device__ __forceinline__ uint32_t wave_sort_bucket_tagged(const Src src, int64_t* gh, KeyT* gk, uint32_t n,
                                                            const int64_t* sb, const int64_t* stt, int nr,
                                                            int* sdiff) {
    const uint32_t lane = threadIdx.x & 63;
    constexpr uint32_t N = 64u * R;
    int64_t h[R];
    KeyT k[R];
    uint32_t g[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * 64u + lane;
        if (i < n) {
            src.load(i, h[r], k[r], g[r]);
        } else {
            h[r] = INT64_MAX;
            k[r] = std::numeric_limits<KeyT>::max();
            g[r] = 0xFFFFFFFFu;
        }
    }
    bool packed = false;
    if constexpr (R == 1)
        packed = wave_packed_sort<KeyT, true>(
            [&](uint32_t i, int64_t& hh, KeyT& kk, uint32_t& gg) { src.load(i, hh, kk, gg); }, n, h[0], k[0], g[0]);
    if (!packed) {
#pragma unroll
    for (uint32_t size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {
                const uint32_t rs = stride / 64;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if ((r & rs) == 0) {
                        const uint32_t i = r * 64u + lane;
                        const bool up = (i & size) == 0;
                        const int r2 = r + rs;
                        if (ent_less3<KeyT>(h[r2], k[r2], g[r2], h[r], k[r], g[r]) == up) {
                            const int64_t th = h[r];
                            const KeyT tk = k[r];
                            const uint32_t tg = g[r];
                            h[r] = h[r2];
                            k[r] = k[r2];
                            g[r] = g[r2];
                            h[r2] = th;
                            k[r2] = tk;
                            g[r2] = tg;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t i = r * 64u + lane;
                    const int64_t oh = xor_any(h[r], (int)stride);
                    const KeyT ok = xor_any(k[r], (int)stride);
                    const uint32_t og = xor_lane32(g[r], (int)stride);
                    const bool lower = (lane & stride) == 0;
                    const bool up = (i & size) == 0;
                    const bool other_less = ent_less3<KeyT>(oh, ok, og, h[r], k[r], g[r]);
                    const bool mine_less = ent_less3<KeyT>(h[r], k[r], g[r], oh, ok, og);
                    if ((lower == up) ? other_less : mine_less) {
                        h[r] = oh;
                        k[r] = ok;
                        g[r] = og;
                    }
                }
            }
        }
    }
    }  // !packed
    uint32_t base = 0;
    int64_t prev_h_last = 0;
    KeyT prev_k_last = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * 64u + lane;
        int64_t ph = shfl_any(h[r], (int)((lane + 63) & 63));
        KeyT pk = shfl_any(k[r], (int)((lane + 63) & 63));
        if (lane == 0) {
            ph = prev_h_last;
            pk = prev_k_last;
        }
        const bool first = i < n && (i == 0 || ph != h[r] || pk != k[r]);
        const unsigned long long bal = __ballot(first);
        int ra = 1, rh = -1;
        if (first) {
            const uint32_t o = base + (uint32_t)__popcll(bal & lanemask_lt());
            gh[o] = h[r];
            gk[o] = k[r];
            // ranges this element verifies: r_a = first r >= 1 with b[r] >= tag (arrived before b[r]),
            // r_h = last r with t[r] >= h.  Both as fixed six-step searches (nr <= 64) run side by
            // side, so their dependent LDS reads overlap: pa = last index with b[pa] < tag (b[0] = 0,
            // b[nr] = n >= every tag; a set member, tag 0, stays at 0), pt = last with t[pt] >= h
            const int64_t tag = (int64_t)g[r];
            int pa = 0, pt = 0;
#pragma unroll
            for (int step = 32; step; step >>= 1) {
                const int qa = pa + step, qt = pt + step;
                const bool ma = qa <= nr && sb[qa < kMaxRanges ? qa : kMaxRanges] < tag;
                const bool mt = qt < nr && stt[qt < kMaxRanges ? qt : kMaxRanges - 1] >= h[r];
                pa = ma ? qa : pa;
                pt = mt ? qt : pt;
            }
            ra = pa + 1;
            rh = stt[0] >= h[r] ? pt : -1;
        }
        // +1 at r_a, -1 at r_h + 1 of the difference array.  The bucket map is monotone in h, so a
        // bucket's elements share r_h almost always: one atomic for the wave's -1s then, instead of
        // up to 64 on one LDS word
        const bool part = ra <= rh;
        const unsigned long long pm = __ballot(part);
        if (pm) {
            const int lead = __builtin_ctzll(pm);
            const int rh0 = __shfl(rh, lead);
            if (__ballot(part && rh != rh0) == 0) {
                if ((int)(threadIdx.x & 63) == lead) atomicAdd(&sdiff[rh0 + 1], -(int)__popcll(pm));
            } else if (part) {
                atomicAdd(&sdiff[rh + 1], -1);
            }
            // (the +1s stay one atomic each: aggregating them per distinct r_a was slower, 69 vs
            // 60 us, DESIGN.md 5 decision 6)
            if (part) atomicAdd(&sdiff[ra], 1);
        }
        base += (uint32_t)__popcll(bal);
        prev_h_last = shfl_any(h[r], 63);
        prev_k_last = shfl_any(k[r], 63);
    }
    return base;
}

// ---- the scheduled merge by coarse bins (sched_bin_file -> sched_bin_sort) -------------------
// The merge's 2^lb fine buckets grouped 2^kBinLog to a coarse bin.  sched_bin_file files every
// entry into its bin: a workgroup's 4096 entries are counted per bin in LDS, ONE global atomic per
// (workgroup, bin) reserves their places (~4 entries per atomic at 1024 bins, where sched_file paid
// one returning atomic per entry on 128-B count lines), and they are stored in runs.  sched_bin_sort
// then stages one bin in LDS (one workgroup per bin), splits it into its fine buckets by a counting
// sort there, and sorts / dedups / verifies each fine bucket with the same wave network as
// sched_sort, reading LDS instead of global memory; the bin's group sums are plain stores and its
// verification columns one set of atomics per bin.  Bin capacity kBinCap (LDS): ~2.3x the plan's
// expected fill; more (like a fine bucket over kBucketCap) is the overflow the host falls back on.
constexpr int kBinLog = 5;
constexpr uint32_t kBinCap = 3072;
constexpr int kBinTile = 4;          // entries per thread of sched_bin_file
#ifndef RSV_BIN_FILE_THREADS
#define RSV_BIN_FILE_THREADS 1024
#endif
constexpr int kBinFileThreads = RSV_BIN_FILE_THREADS;  // (dev builds vary it)
constexpr int kBinSortThreads = 512;

__host__ __device__ inline uint32_t bin_log(uint32_t lb, uint32_t fl = kBinLog) { return lb > fl ? lb - fl : 0u; }



template <typename KeyT>
__global__ __launch_bounds__(kBinFileThreads) void sched_bin_file(const SchedDev* __restrict__ sd, const int64_t* __restrict__ cand_h,
                                                       const KeyT* __restrict__ cand_k, const uint32_t* __restrict__ cand_i,
                                                       int64_t* __restrict__ ctl, int64_t cap,
                                                       const int64_t* __restrict__ set_h, const KeyT* __restrict__ set_k,
                                                       int64_t m, int64_t* __restrict__ bh, KeyT* __restrict__ bk,
                                                       uint32_t* __restrict__ bi, int64_t* __restrict__ bak_h,
                                                       KeyT* __restrict__ bak_k) {
    extern __shared__ uint32_t hist[];  // [2^lbin]
    __shared__ int64_t stt[kMaxRanges];
    const int nr = sd->nr;
    if (nr < 2) return;
    const uint32_t lb = sd->lb, lbin = bin_log(lb), C = 1u << lbin;
    const int64_t total = m + std::min<int64_t>((int64_t)__hip_atomic_load((const unsigned long long*)ctl,
                                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                                cap);
    const int64_t base = (int64_t)blockIdx.x * (kBinFileThreads * kBinTile);
    if (base >= total) return;  // whole workgroup
    const int64_t off = sd->off;
    cand_h += off;
    cand_k += off;
    cand_i += off;
    for (int i = threadIdx.x; i < nr; i += blockDim.x) stt[i] = sd->t[i];
    for (uint32_t i = threadIdx.x; i < C; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    const uint32_t B_lo = sd->B_lo;
    const uint64_t q = sd->lo_mult;
    const SchedMap map{sd, stt, sd->B, B_lo, (uint32_t)nr, stt[nr - 1], q > UINT64_MAX / B_lo ? UINT64_MAX : q * B_lo};
    int64_t eh[kBinTile];
    KeyT ek[kBinTile];
    uint32_t eg[kBinTile], ebin[kBinTile], eloc[kBinTile];
#pragma unroll
    for (int j = 0; j < kBinTile; ++j) {
        const int64_t t = base + (int64_t)j * kBinFileThreads + threadIdx.x;
        ebin[j] = 0xFFFFFFFFu;
        if (t < total) {
            if (t < m) {
                eh[j] = set_h[t];
                ek[j] = set_k[t];
                eg[j] = 0u;
                bak_h[t] = eh[j];
                bak_k[t] = ek[j];
            } else {
                eh[j] = cand_h[t - m];
                ek[j] = cand_k[t - m];
                eg[j] = cand_i[t - m] + 1u;
            }
            ebin[j] = map(eh[j]) >> (lb - lbin);
            eloc[j] = atomicAdd(&hist[ebin[j]], 1u);
        }
    }
    __syncthreads();
    uint32_t* bcnt = bucket_count(ctl);
    for (uint32_t i = threadIdx.x; i < C; i += blockDim.x) {
        const uint32_t n = hist[i];
        if (n) hist[i] = atomicAdd(&bcnt[(size_t)i * kCountStride], n);
    }
    __syncthreads();
    const uint32_t cap_bin = std::min<uint32_t>(kBinCap, (uint32_t)kBucketCap << (lb - lbin));
    bool over = false;
#pragma unroll
    for (int j = 0; j < kBinTile; ++j) {
        if (ebin[j] == 0xFFFFFFFFu) continue;
        const uint32_t pos = hist[ebin[j]] + eloc[j];
        if (pos < cap_bin) {
            const size_t slot = ((size_t)ebin[j] << (lb - lbin)) * kBucketCap + pos;
            bh[slot] = eh[j];
            bk[slot] = ek[j];
            bi[slot] = eg[j];
        } else {
            over = true;
        }
    }
    if (over) ctl[1] = 1;
}

template <typename KeyT>
__global__ __launch_bounds__(kBinSortThreads) void sched_bin_sort(int64_t cand_cap, int64_t* __restrict__ ctl,
                                                                  int32_t log_bmax, int64_t* __restrict__ bh,
                                                                  KeyT* __restrict__ bk, uint32_t* __restrict__ bi,
                                                                  const SchedDev* __restrict__ sd,
                                                                  int* __restrict__ vacc) {
    constexpr uint32_t kF = 1u << kBinLog;
    __shared__ int64_t lh[kBinCap];
    __shared__ KeyT lk[kBinCap];
    __shared__ uint32_t lg[kBinCap];
    __shared__ uint16_t perm[kBinCap];
    __shared__ int64_t sb[kMaxRanges + 1], stt[kMaxRanges];
    __shared__ int sdiff[kMaxRanges + 1];
    __shared__ uint32_t fcnt[kF], foff[kF], fnd[kF];
    const int64_t c = ctl[0];
    const int nr = sd->nr;
    if (c > cand_cap || ctl[1] || nr < 2) return;  // uniform over the grid (set before this kernel)
    const uint32_t lb = sd->lb, lbin = bin_log(lb), F = 1u << (lb - lbin);
    const uint32_t bin = blockIdx.x, fb0 = bin * F;
    for (int i = threadIdx.x; i <= nr; i += blockDim.x) {
        sb[i] = sd->b[i];
        sdiff[i] = 0;
        if (i < nr) stt[i] = sd->t[i];
    }
    if (threadIdx.x < kF) fcnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t B_lo = sd->B_lo;
    const uint64_t q = sd->lo_mult;
    const SchedMap map{sd, stt, sd->B, B_lo, (uint32_t)nr, stt[nr - 1], q > UINT64_MAX / B_lo ? UINT64_MAX : q * B_lo};
    uint32_t* bcnt = bucket_count(ctl) + (size_t)bin * kCountStride;
    const uint32_t nb = std::min<uint32_t>(*bcnt, kBinCap);  // more: sched_bin_file flagged the overflow
    const size_t slab = (size_t)fb0 * kBucketCap;
    constexpr int kPer = kBinCap / kBinSortThreads;
    uint32_t fj[kPer], fr[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t i = j * kBinSortThreads + threadIdx.x;
        if (i < nb) {
            const int64_t h = bh[slab + i];
            lh[i] = h;
            lk[i] = bk[slab + i];
            lg[i] = bi[slab + i];
            fj[j] = map(h) - fb0;
            fr[j] = atomicAdd(&fcnt[fj[j]], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the fine counts (F <= 64)
        const uint32_t lane = threadIdx.x;
        const uint32_t v = lane < F ? fcnt[lane] : 0u;
        uint32_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(x, d);
            if ((int)lane >= d) x += o;
        }
        if (lane < F) foff[lane] = x - v;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t i = j * kBinSortThreads + threadIdx.x;
        if (i < nb) perm[foff[fj[j]] + fr[j]] = (uint16_t)i;
    }
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* bdist = bucket_distinct(ctl, log_bmax);
    for (uint32_t f = wave; f < F; f += kBinSortThreads / 64) {
        const uint32_t n = fcnt[f], b = fb0 + f;
        uint32_t nd = 0;
        if (n > kBucketCap) {
            if (lane == 0) ctl[1] = 1;  // the verdict reports the overflow; emit skips
        } else if (n > 0) {
            const LdsBinSrc<KeyT> src{lh, lk, lg, perm + foff[f]};
            int64_t* gh = bh + (size_t)b * kBucketCap;
            KeyT* gk = bk + (size_t)b * kBucketCap;
            nd = n <= 64    ? wave_sort_bucket_tagged<KeyT, 1>(src, gh, gk, n, sb, stt, nr, sdiff)
                 : n <= 128 ? wave_sort_bucket_tagged<KeyT, 2>(src, gh, gk, n, sb, stt, nr, sdiff)
                            : wave_sort_bucket_tagged<KeyT, 4>(src, gh, gk, n, sb, stt, nr, sdiff);
        }
        if (lane == 0) {
            bdist[b] = nd;
            fnd[f] = nd;
        }
    }
    __syncthreads();
    uint32_t* gsum = bucket_group(ctl, log_bmax);
    for (uint32_t g = threadIdx.x; g < (F + 15) / 16; g += blockDim.x) {
        uint32_t v = 0;
        for (uint32_t f = g * 16; f < std::min(F, g * 16 + 16); ++f) v += fnd[f];
        gsum[(fb0 >> 4) + g] = v;
    }
    int* acc = vacc + (size_t)(bin % kVerifyCopies) * (kMaxRanges + 1);
    for (int i = threadIdx.x; i <= nr; i += blockDim.x)
        if (sdiff[i]) atomicAdd(&acc[i], sdiff[i]);
    if (threadIdx.x == 0) *bcnt = 0;
}

// ctl[0..5], the verification verdict (first range r >= 1 short of k elements, or -1) and the
// plan's range count (< 2: no pass ran) to coherent host memory, then the flag
// (then re-arms the candidate counter, the overflow word and the accumulators for the next pass)
__device__ __forceinline__ void sched_verdict(int64_t* __restrict__ ctl, int* __restrict__ vacc,
                                              const SchedDev* __restrict__ sd, int64_t k, int64_t* dst, uint32_t* flag,
                                              uint32_t gen) {
    __shared__ int col[kMaxRanges + 1];
    const int nr = sd->nr;
    for (int i = threadIdx.x; i <= nr; i += blockDim.x) {
        int v = 0;
        for (int j = 0; j < kVerifyCopies; ++j) {
            v += vacc[(size_t)j * (kMaxRanges + 1) + i];
            vacc[(size_t)j * (kMaxRanges + 1) + i] = 0;
        }
        col[i] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = 0, fail = -1, minc = INT64_MAX;
        for (int r = 0; r < nr; ++r) {
            run += col[r];
            if (r >= 1) {
                minc = std::min(minc, run);
                if (run < k && fail < 0) fail = r;
            }
        }
        for (int i = 0; i < 6; ++i) dst[i] = ctl[i];
        dst[6] = fail;
        dst[7] = minc;
        dst[8] = nr;
        ctl[0] = 0;
        ctl[1] = 0;
    }
    publish_flag(flag, gen);
}

// the set's first min(ctl[2], k) keys into coherent host memory by every workgroup; each releases at
// system scope and takes a ticket, the last stores the flag
__device__ __forceinline__ void publish_set_body(const uint32_t* __restrict__ src, uint32_t* dst,
                                                 const int64_t* __restrict__ ctl, int64_t k, int32_t key_words,
                                                 uint32_t* flag, uint32_t gen, uint32_t* ticket) {
    const int64_t words = std::min<int64_t>(ctl[2], k) * key_words;
    const int64_t vecs = words >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < vecs; i += stride) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (int64_t i = (vecs << 2) + t0; i < words; i += stride) dst[i] = src[i];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        const uint32_t prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __hip_atomic_store(flag, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The scheduled pass's verdict (workgroup 0) and, when a target is given, the merged set's
// speculative publication (every workgroup) in one dispatch: the set copy (~13 us for 512 KB) no
// longer waits for a second kernel behind the verdict
__global__ __launch_bounds__(1024) void sched_publish(int64_t* __restrict__ ctl, int* __restrict__ vacc,
                                                     const SchedDev* __restrict__ sd, int64_t k, int64_t* dst,
                                                     uint32_t* flag, uint32_t gen, const uint32_t* __restrict__ set_src,
                                                     uint32_t* set_dst, int32_t key_words, uint32_t* set_flag,
                                                     uint32_t set_gen, uint32_t* ticket) {
    if (blockIdx.x == 0) sched_verdict(ctl, vacc, sd, k, dst, flag, gen);
    if (set_dst) publish_set_body(set_src, set_dst, ctl, k, key_words, set_flag, set_gen, ticket);
}

// ctl[0..5] -> coherent host memory + flag (one wave; the host spins instead of a stream sync);
// then the candidate counter and overflow word are re-armed for the next filter pass (each lane
// clears only the word it read itself, so the copy sees the old value)
__global__ __launch_bounds__(64) void ctl_publish(int64_t* __restrict__ ctl, int64_t* dst, uint32_t* flag,
                                                  uint32_t gen) {
    if (threadIdx.x < 6) {
        const int64_t v = ctl[threadIdx.x];
        dst[threadIdx.x] = v;
        if (threadIdx.x < 2) ctl[threadIdx.x] = 0;
    }
    publish_flag(flag, gen);
}

// Speculative publication of a set-mode merge (large batches): as publish_multi_kernel, but the
// set's size is read on the device (ctl[2], the merged distinct count, capped at k), so the host
// enqueues it right behind ctl_publish and it runs while the host turns the ctl read around.  The
// host uses it only if that merge turns out to be the batch's last (distinct_spec_take).
__global__ __launch_bounds__(1024) void publish_set_kernel(const uint32_t* __restrict__ src, uint32_t* dst,
                                                           const int64_t* __restrict__ ctl, int64_t k,
                                                           int32_t key_words, uint32_t* flag, uint32_t gen,
                                                           uint32_t* ticket) {
    publish_set_body(src, dst, ctl, k, key_words, flag, gen, ticket);
}

// First-occurrence flags of one segment for the host replay (rsv_host_values.h: only the first
// occurrence of a key can be admitted): the replica's members at the segment's start followed by the
// segment's keys in arrival order, stably sorted by key with their positions as values; entry t
// keeps its flag when it heads its key's run (no member and no earlier entry carries the key).
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void mark_first(const KeyT* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                     int64_t total, uint32_t nm, uint8_t* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += stride) {
        const uint32_t v = sv[p];
        if (v >= nm) flag[v - nm] = (p == 0 || sk[p] != sk[p - 1]) ? 1 : 0;
    }
}

// one logged segment gathered into arrival order (perm from the radix sort of its arrival indices)
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void permute_log(const uint32_t* __restrict__ perm, const int64_t* __restrict__ h,
                                                      const KeyT* __restrict__ k, int64_t c, int64_t* __restrict__ oh,
                                                      KeyT* __restrict__ ok) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < c; t += stride) {
        const uint32_t p = perm[t];
        oh[t] = h[p];
        ok[t] = k[p];
    }
}

// ---- device combine of packed rows (rsv_export_packed / rsv_merge_packed on DISTINCT samplers) ---
// A row is one sampler's set: [keys widened to int64 (k) | hashes (k) | meta], ascending (h, key),
// meta = n, count, tied, max_hash, log_retained, ordered (reservoir_amd/distributed.py reads it).
// The merge of `parts` rows with the sampler's own set (run 0) is the bottom-k by (h, key) of the
// union -- the bucketed merge of the filter path, fed from the runs directly: every run is already
// sorted, so a bucket's entries are one contiguous range per run.  rows_bounds finds the ranges in
// one streaming pass (no atomics), rows_sort gathers each bucket (one wave) from the runs into LDS,
// sorts and dedups it, bucket_emit places the distinct entries by rank, merge_publish hands the
// control words to the host (coherent memory + flag) -- four dispatches and no host wait.
// Entries above `top` are dropped first: top = the smallest maximum of a FULL run (k entries: the
// bottom-k of the union lies at or below it) and at most the largest hash present.
constexpr int kRowMeta = 6;

template <typename KeyT>
struct Runs {
    const int64_t* rows;
    int64_t stride, k;
    const int64_t* set_h;
    const KeyT* set_k;
    int64_t m;
    __device__ __forceinline__ int64_t n(int r) const {
        if (r == 0) return m;
        const int64_t v = rows[(int64_t)(r - 1) * stride + 2 * k];
        return v < 0 ? 0 : (v > k ? k : v);
    }
    __device__ __forceinline__ int64_t h(int r, int64_t i) const {
        return r == 0 ? set_h[i] : rows[(int64_t)(r - 1) * stride + k + i];
    }
    __device__ __forceinline__ KeyT key(int r, int64_t i) const {
        return r == 0 ? set_k[i] : (KeyT)rows[(int64_t)(r - 1) * stride + i];
    }
    __device__ __forceinline__ int64_t max_h(int r) const { return rows[(int64_t)(r - 1) * stride + 2 * k + 3]; }
    __device__ __forceinline__ bool tied(int r) const { return rows[(int64_t)(r - 1) * stride + 2 * k + 2] != 0; }
    __device__ __forceinline__ bool ordered(int r) const { return rows[(int64_t)(r - 1) * stride + 2 * k + 5] != 0; }
};

// the cut and its tie flag, computed by one wave (every workgroup of rows_bounds does: <= 64 rows,
// lane r - 1 reads row r's meta -- one load latency instead of a chain of 4 per row, which made the
// pass 111 us at 8 rows).  T = the smallest maximum of a full run; tiedT: a full run whose own
// boundary bucket was oversubscribed sits at T (its export holds only part of that bucket -- with
// the merged maximum at T the union's tie word cannot see it).  Wave-uniform results.
template <typename KeyT>
__device__ __forceinline__ void runs_top(const Runs<KeyT>& R, int parts, int64_t set_max, bool set_over,
                                         int64_t* top, int64_t* T_out, bool* tiedT, bool* all_ordered) {
    const int lane = (int)(threadIdx.x & 63);
    const bool on = lane < parts;
    const int64_t n = on ? R.n(lane + 1) : 0;
    const int64_t mh = on ? R.max_h(lane + 1) : INT64_MIN;
    const bool t = on && R.tied(lane + 1), ord = !on || R.ordered(lane + 1);
    const bool full = n == R.k;
    int64_t T = full ? mh : INT64_MAX, mx = n > 0 ? mh : INT64_MIN;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T = std::min(T, shfl_xor_any(T, off));
        mx = std::max(mx, shfl_xor_any(mx, off));
    }
    if (R.m == R.k) T = std::min(T, set_max);
    if (R.m > 0) mx = std::max(mx, set_max);
    const bool tt = (R.m == R.k && set_over && set_max == T) || __ballot(full && t && mh == T) != 0;
    *top = std::min(T, mx);
    *T_out = T;
    *tiedT = tt;
    *all_ordered = __ballot(!ord) == 0;
}

// start[r * (B + 1) + b] = first index of run r whose bucket is >= b (entries above top: bucket B).
// One thread per index i in [0, n_r] (i = n_r closes the run); grid (x, parts + 1), y = run.  Each
// bucket's first entry stores its index (one store per non-empty bucket); the buckets a run skips
// keep the all-ones fill and rows_fill gives them the next bucket's start (a run sparse in the
// buckets -- an empty one, or a shard with few elements under the cut -- would otherwise leave one
// thread storing every skipped bucket in turn: 128 us at 8 rows with an empty target).
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void rows_bounds(Runs<KeyT> R, int32_t parts, int64_t set_max, int32_t set_over,
                                                      uint32_t lb, int64_t* __restrict__ ctl, int32_t log_bmax,
                                                      uint32_t* __restrict__ start) {
    __shared__ int64_t s_top;
    __shared__ uint64_t s_q;
    const int r = (int)blockIdx.y;
    if (threadIdx.x < 64) {
        int64_t top, T;
        bool tiedT, ord;
        runs_top(R, parts, set_max, set_over != 0, &top, &T, &tiedT, &ord);
        if (threadIdx.x == 0) {
            const uint64_t span = (uint64_t)top - (uint64_t)INT64_MIN;
            s_top = top;
            s_q = span == UINT64_MAX ? 1ull : UINT64_MAX / (span + 1);
            if (blockIdx.x == 0 && r == 0) {
                ctl[5] = 0;  // bucket_emit's tie word
                ctl[6] = (tiedT ? 2 : 0) | (ord ? 1 : 0);
                ctl[7] = T;
            }
        }
    }
    if (blockIdx.x == 0 && r == 0) zero_bucket_groups(ctl, log_bmax);
    __syncthreads();
    const int64_t top = s_top;
    const BucketMap map(s_q, lb);
    const uint32_t B = 1u << lb;
    const int64_t n = R.n(r);
    uint32_t* st = start + (size_t)r * (B + 1);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
        uint32_t bi = B;
        if (i < n) {
            const int64_t h = R.h(r, i);
            if (h <= top) bi = map(h);
        }
        int64_t bp = -1;
        if (i > 0) {
            const int64_t h = R.h(r, i - 1);
            bp = h <= top ? (int64_t)map(h) : (int64_t)B;
        }
        if ((int64_t)bi != bp) st[bi] = (uint32_t)i;
    }
}

// the skipped buckets of every run: start[b] = min(start[b], start[b + 1]) from the top bucket down
// (a suffix minimum; unwritten entries are all ones).  One workgroup per run, each thread a
// contiguous piece, a workgroup scan of the pieces' minima for the carries.
__global__ __launch_bounds__(1024) void rows_fill(uint32_t lb, uint32_t* __restrict__ start) {
    __shared__ uint32_t s_min[1024 / 64];
    const uint32_t B1 = (1u << lb) + 1;
    uint32_t* st = start + (size_t)blockIdx.x * B1;
    const uint32_t per = (B1 + blockDim.x - 1) / blockDim.x;
    const uint32_t a = threadIdx.x * per, e = std::min(B1, a + per);
    uint32_t m = 0xFFFFFFFFu;
    for (uint32_t b = e; b-- > a;) m = std::min(m, st[b]);  // this piece's minimum
    // exclusive suffix minimum over the pieces after this one: within the wave, then across waves
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = m;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_down((int)incl, off);
        if (lane + off < 64) incl = std::min(incl, v);
    }
    if (lane == 0) s_min[w] = incl;
    __syncthreads();
    uint32_t carry = (uint32_t)__shfl_down((int)incl, 1);
    if (lane == 63) carry = 0xFFFFFFFFu;
    for (uint32_t x = w + 1; x < blockDim.x / 64; ++x) carry = std::min(carry, s_min[x]);
    for (uint32_t b = e; b-- > a;) {
        carry = std::min(carry, st[b]);
        st[b] = carry;
    }
}

// one wave per bucket: its entries from every run (contiguous ranges by rows_bounds) into LDS,
// sorted by (h, key), duplicates dropped (wave_sort_bucket), the distinct ones written compacted to
// the bucket area; bucket_distinct / group sums as bucket_sort leaves them.  > kBucketCap entries (a
// degenerate hash): the overflow word, and the host redoes the merge on the radix-sort path.
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void rows_sort(Runs<KeyT> R, int32_t parts, uint32_t lb,
                                                    const uint32_t* __restrict__ start, int64_t* __restrict__ ctl,
                                                    int32_t log_bmax, int64_t* __restrict__ bh, KeyT* __restrict__ bk) {
    constexpr int kMaxRuns = 65;
    __shared__ int64_t s_h[kBlock / 64][kBucketCap];
    __shared__ KeyT s_k[kBlock / 64][kBucketCap];
    __shared__ int64_t s_lo[kBlock / 64][kMaxRuns], s_ex[kBlock / 64][kMaxRuns + 1];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t B = 1u << lb;
    const uint32_t b = blockIdx.x * (kBlock / 64) + w;
    if (b >= B) return;
    const int nr = parts + 1;
    // per run: [lo, hi) of this bucket; exclusive prefix of the counts (runs > 64: a second round)
    int64_t base = 0;
    for (int r0 = 0; r0 < nr; r0 += 64) {
        const int r = r0 + (int)lane;
        int64_t lo = 0, cnt = 0;
        if (r < nr) {
            lo = start[(size_t)r * (B + 1) + b];
            cnt = (int64_t)start[(size_t)r * (B + 1) + b + 1] - lo;
        }
        int64_t incl = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t v = shfl_any(incl, (int)(lane >= (uint32_t)off ? lane - off : lane));
            if (lane >= (uint32_t)off) incl += v;
        }
        if (r < nr) {
            s_lo[w][r] = lo;
            s_ex[w][r] = base + incl - cnt;
        }
        base += shfl_any(incl, 63);
    }
    if (lane == 0) s_ex[w][nr] = base;
    __builtin_amdgcn_wave_barrier();
    uint32_t* bdist = bucket_distinct(ctl, log_bmax) + b;
    if (base > (int64_t)kBucketCap) {
        if (lane == 0) {
            ctl[1] = 1;
            *bdist = 0;
        }
        return;
    }
    const uint32_t n = (uint32_t)base;
    if (n == 0) {
        if (lane == 0) *bdist = 0;
        return;
    }
    for (uint32_t j = lane; j < n; j += 64) {
        int r = 0;
        while (s_ex[w][r + 1] <= (int64_t)j) ++r;
        const int64_t i = s_lo[w][r] + ((int64_t)j - s_ex[w][r]);
        s_h[w][j] = R.h(r, i);
        s_k[w][j] = R.key(r, i);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t nd = n <= 64    ? wave_sort_bucket<KeyT, 1>(s_h[w], s_k[w], n, bdist)
                        : n <= 128 ? wave_sort_bucket<KeyT, 2>(s_h[w], s_k[w], n, bdist)
                                   : wave_sort_bucket<KeyT, 4>(s_h[w], s_k[w], n, bdist);
    __builtin_amdgcn_wave_barrier();
    int64_t* gh = bh + (size_t)b * kBucketCap;
    KeyT* gk = bk + (size_t)b * kBucketCap;
    for (uint32_t j = lane; j < nd; j += 64) {
        gh[j] = s_h[w][j];
        gk[j] = s_k[w][j];
    }
    if (lane == 0 && nd) atomicAdd(bucket_group(ctl, log_bmax) + (b >> 4), nd);
}

// the merge's control words (ctl[0..7]) to coherent host memory + flag; re-arms ctl[0..1]
__global__ __launch_bounds__(64) void merge_publish(int64_t* __restrict__ ctl, int64_t* dst, uint32_t* flag,
                                                    uint32_t gen) {
    if (threadIdx.x < 8) {
        const int64_t v = ctl[threadIdx.x];
        dst[threadIdx.x] = v;
        if (threadIdx.x < 2) ctl[threadIdx.x] = 0;
    }
    publish_flag(flag, gen);
}

// one sampler's set as a packed row
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void export_row_kernel(const int64_t* __restrict__ set_h,
                                                            const KeyT* __restrict__ set_k, int64_t m, int64_t k,
                                                            int64_t* __restrict__ row, int64_t count, int64_t tied,
                                                            int64_t max_hash, int64_t retained, int64_t ordered) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += stride) {
        row[i] = i < m ? (int64_t)set_k[i] : 0;
        row[k + i] = i < m ? set_h[i] : INT64_MAX;
    }
    if (blockIdx.x == 0 && threadIdx.x < kRowMeta) {
        const int64_t meta[kRowMeta] = {m, count, tied, max_hash, retained, ordered};
        row[2 * k + threadIdx.x] = meta[threadIdx.x];
    }
}

// int64-widened row keys -> KeyT (the overflow fallback's merge_into_set input)
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void narrow_keys(const int64_t* __restrict__ src, int64_t n, KeyT* __restrict__ dst) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = (KeyT)src[i];
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
    int64_t set_top = INT64_MIN;  // the set's largest hash, valid when m > 0
    int64_t* set_h = nullptr;     // [set_cap <= k], ascending (h, key)
    void* set_k = nullptr;
    int64_t set_cap = 0;
    // speculative set publication (set mode, batches >= kSpecMinBatch): target from the runtime
    void* spec_dst = nullptr;     // coherent host buffer (device alias)
    uint32_t* spec_flag = nullptr;
    uint32_t* spec_gen_ctr = nullptr;  // the handle's publication generation counter
    bool spec_arm = false;        // read_ctl enqueues publish_set_kernel behind ctl_publish
    bool spec_ok = false;         // the last enqueued publication holds the batch's final set
    uint32_t spec_gen = 0;
    int64_t spec_min = 1ll << 27;  // smallest batch that publishes speculatively (~180 us of filter)
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
    // bucketed merge (bucket_scatter/sort/emit); log_bmax < 0: radix-sort merge only
    int32_t log_bmax = -1;
    int64_t* ctl = nullptr;       // control block (see bucket_scatter); `counter` points at ctl[0]
    int64_t* hc = nullptr;        // coherent host: ctl[0..3] copies + flag at hc[8]
    int64_t* hc_dev = nullptr;
    uint32_t hc_gen = 0;
    int64_t* bh = nullptr;        // [bmax * kBucketCap] bucket entries
    void* bk = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    int64_t* samp = nullptr;      // [2 * kSample]
    int64_t* h_pinned = nullptr;  // host scalars
    std::vector<int64_t> samp_host;
    KernelTimer* timer = nullptr;
    bool last_tie = false;        // merge_into_set: rank k tied with rank k - 1 on h
    // RSV_DISTINCT_ORDERED (see ordered_sample_impl): the set arrays track the bottom-k by (h, key)
    // of what the reference could admit; the exact replica of RandomValues runs on the host over a
    // device log of the admitted candidates, only when the tie bucket makes it necessary
    bool ordered = false;
    bool over = false;              // more admitted distinct elements have h <= max_h than k
    bool exact = true;              // the set arrays hold the reference's set
    HostValues rep;                 // the replica, current up to the first logged segment
    int64_t seen = 0;               // elements sampled so far (chunk sizing)
    int64_t rate_c = 0, rate_m = 0; // the last full-heap chunk: candidates, length,
    double rate_span = 0;           // and its threshold's distance above Long.MinValue
    struct Seg {
        int64_t off, c, m;          // log offset, candidates, chunk length
    };
    std::vector<Seg> segs;
    int64_t* log_h = nullptr;       // [log_cap] candidates of every chunk since the last replay
    void* log_k = nullptr;
    uint32_t* log_i = nullptr;      // chunk-relative arrival index
    int64_t log_n = 0, log_cap = 0, log_limit = 0;
    // the scheduled pass (sched_sample): range bounds, its own merge area, the set's backup
    SchedDev* sdev = nullptr;
    int64_t* sctl = nullptr;        // ctl words + bucket counts of the scheduled merge
    int32_t log_bmax_s = -1;
    int64_t* sbh = nullptr;
    void* sbk = nullptr;
    uint32_t* sbi = nullptr;
    int* vacc = nullptr;            // [kVerifyCopies][kMaxRanges + 1]
    int64_t* bak_h = nullptr;       // [k] the set before the pass
    void* bak_k = nullptr;
    int64_t* shc = nullptr;         // coherent host: published words + flag at [12]
    int64_t* shc_dev = nullptr;
    uint32_t sgen = 0;
    bool sdirty = false;            // sctl / vacc allocated, not yet zeroed (the fused pass zeroes them)
    bool sched = true;              // RSV_ORDERED_SCHED=0: the chunk loop only
    double sched_beta = 1.6;        // RSV_SCHED_BETA (test hook: a small beta forces the fallback)
    uint32_t* perm = nullptr;       // [ord_cap] one segment's candidates in arrival order
    uint32_t* sorted_i = nullptr;   // [ord_cap] radix-sort key output
    int64_t* ord_h = nullptr;       // [ord_cap] one segment's hashes and keys permuted into arrival order
    void* ord_k = nullptr;
    int64_t ord_cap = 0;            // capacity of the two buffers above and of the pinned copies
    int64_t* ph = nullptr;          // pinned: hashes, keys (as KeyT) of one segment in arrival order
    void* pk = nullptr;
    // first-occurrence flags (segment_to_host with `first`): members + segment keys, sorted copies,
    // their positions, the flags on the device and pinned, the members' pinned staging
    void* fk_in = nullptr;
    void* fk_out = nullptr;
    uint32_t* fv = nullptr;
    uint8_t* fflag = nullptr;
    uint8_t* pflag = nullptr;
    void* pmem = nullptr;
    int64_t fcap = 0;               // capacity (entries) of fk_in / fk_out / fv; fflag / pflag hold ord_cap
    int64_t pmem_cap = 0;
    int64_t first_min = 4096;       // segments at least this long replay through the flags (no host set)
    // the next segment staged while the host runs this one (replay_log): its pinned copies
    int64_t* ph2 = nullptr;
    void* pk2 = nullptr;
    uint8_t* pflag2 = nullptr;
    int64_t ord2_cap = 0;
    bool overlap = true;            // RSV_REPLAY_OVERLAP=0 (test hook): stage no segment ahead
    hipEvent_t seg_ev = nullptr;    // a segment's own copies done (the next one's staging may still run)
    // Exact multi-rank merge of ordered samplers (rsv_export_log / rsv_merge_log): the candidates
    // the replica consumed (arrival order, host) + the segments still in the log, and the segments
    // logged before the last merge -- together every candidate logged since creation (`arch_ok`).
    // Sampling again after a merge drops them (the merged state has no single arrival order).
    // Opt-in (rsv_retain_log, before the first sample): the archive holds 12-16 B per consumed
    // candidate on the host, up to kArchMax of them.
    bool retain = false;
    std::vector<int64_t> arch_h, arch_k;  // keys: arch_k (8-byte keys) or arch_k4 (4-byte keys)
    std::vector<int32_t> arch_k4;
    bool arch_ok = true;
    std::vector<Seg> pre_segs;
    bool merged = false;
    int64_t sched_passes = 0, sched_fallbacks = 0;  // rsv_distinct_info counters
    // the replica lags the set arrays (a merge replaced the set): rebuilt from them before the
    // next replay, which is the only reader (a merge without a later tie never pays for it)
    bool rep_stale = false;
    // device combine of packed rows (distinct_merge_rows): enqueued without a host wait; the host
    // fields (m, max_h, set_top, over) are settled from its published words at the next call
    bool pend = false;
    uint32_t pend_gen = 0;
    uint32_t pend_lb = 0;
    const int64_t* pend_rows = nullptr;  // the rows' snapshot (rows_copy) a bucket overflow redoes the merge from
    int64_t* rows_copy = nullptr;        // engine-owned copy of the last merged rows (the caller may reuse theirs)
    int64_t rows_copy_cap = 0;           // words
    int32_t pend_parts = 0;
    int64_t pend_stride = 0;
    uint32_t* mstart = nullptr;  // [(parts + 1) x (B + 1)] bucket starts of every run
    int64_t mstart_cap = 0;
    // key_width > 8 (fixed-width byte keys): the whole sampler is rsv_wide.hip's; every entry point
    // below forwards to it
    WideDistinct* wide = nullptr;
};

// <= 2 GB of host archive (12-16 B per candidate): beyond it rsv_export_log reports the log as not
// retained
constexpr int64_t kArchMax = (int64_t)1 << 27;

void distinct_set_timer(DistinctState* d, KernelTimer* t) {
    d->timer = t;
    if (d->wide) wide_set_timer(d->wide, t);
}

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

DistinctState* distinct_create(int32_t k, int key_width, int hash_kind, int64_t r0, int64_t r1, bool ordered,
                               int* status) {
    DistinctState* d = new DistinctState();
    d->ordered = ordered;
    if (key_width > 8) {  // fixed-width byte keys: rsv_wide.hip
        d->k = k;
        d->kw = key_width;
        d->hash_kind = hash_kind;
        // set mode's one-pass batches publish speculatively (rsv_wide.hip wide_spec_target)
        d->wide = wide_create(k, key_width, hash_kind == kHashUuid ? kWideSrcUuid : kWideSrcHashes, r0, r1, ordered,
                              status);
        if (!d->wide) {
            delete d;
            return nullptr;
        }
        return d;
    }
    if (ordered) d->rep.reset(k);
    d->k = k;
    d->kw = key_width;
    d->hash_kind = hash_kind;
    d->r0 = r0;
    d->r1 = r1;
    d->cand_limit = 4 * (int64_t)k + 4096;
    d->log_limit = std::max<int64_t>(d->cand_limit, std::min<int64_t>(std::max<int64_t>(32 * d->cand_limit, 1 << 22), 1 << 27));
    if (const char* v = std::getenv("RSV_ORDERED_LOG_LIMIT"))  // test hook: force eager replays
        d->log_limit = std::max<int64_t>(d->cand_limit, std::atoll(v));
    if (const char* v = std::getenv("RSV_ORDERED_SCHED")) d->sched = v[0] != '0';
    if (const char* v = std::getenv("RSV_SCHED_BETA")) d->sched_beta = std::atof(v);
    if (const char* v = std::getenv("RSV_FIRST_MIN"))  // test hook: which replay form serves small segments
        d->first_min = std::max<int64_t>(1, std::atoll(v));
    if (const char* v = std::getenv("RSV_REPLAY_OVERLAP")) d->overlap = v[0] != '0';  // test hook
    if (const char* v = std::getenv("RSV_SPEC_MIN_BATCH"))  // test hook: speculative publication
        d->spec_min = std::max<int64_t>(1, std::atoll(v));
    hipError_t e = hipSuccess;
    auto A = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = pool_device_alloc(p, bytes ? bytes : 16);
    };
    // bucketed merge for typical k: bmax buckets of kBucketCap entries, mean occupancy <= 128 at
    // the largest merge (k + cand_limit entries)
    int32_t log_bmax = 0;
    while (((int64_t)1 << (log_bmax + kBucketAvgLog)) < (int64_t)k + d->cand_limit) ++log_bmax;
    const double bucket_bytes = (double)((int64_t)1 << log_bmax) * kBucketCap * (8 + key_width);
    const bool bucketed = bucket_bytes <= 256.0 * 1024 * 1024;
    const size_t ctl_bytes =
        kCtlWords * 8 + (bucketed ? ((size_t)(kCountStride + 1) * 4 << log_bmax) + 4 * (((size_t)1 << log_bmax >> 4) + 1) : 0);
    A((void**)&d->ctl, ctl_bytes);
    if (e == hipSuccess) e = hipMemset(d->ctl, 0, ctl_bytes);  // once: bucket_sort keeps the counts zeroed
    d->counter = (unsigned long long*)d->ctl;
    if (e == hipSuccess) e = pool_host_alloc((void**)&d->hc, 128, hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&d->hc_dev, d->hc, 0);
    if (e == hipSuccess) ((uint32_t*)(d->hc + 8))[0] = 0;
    if (bucketed) {
        A((void**)&d->bh, ((size_t)1 << log_bmax) * kBucketCap * 8);
        A(&d->bk, ((size_t)1 << log_bmax) * kBucketCap * key_width);
        if (e == hipSuccess) d->log_bmax = log_bmax;
    }
    A((void**)&d->d_count, 32);

    A((void**)&d->samp, 2 * kSample * 8);
    if (e == hipSuccess) {
        size_t tb = 0;  // the threshold sample's sort
        e = rocprim::radix_sort_keys(nullptr, tb, (int64_t*)nullptr, (int64_t*)nullptr, (size_t)kSample);
        d->temp_bytes = tb;
    }
    A(&d->temp, d->temp_bytes);
    if (e == hipSuccess) e = pool_host_alloc((void**)&d->h_pinned, 128, hipHostMallocDefault);
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
    if (d->wide) {
        wide_destroy(d->wide);
        delete d;
        return;
    }
    void* ps[] = {d->set_h, d->set_k, d->cand_h, d->cand_k, d->ctl, d->bh, d->bk, d->mh0, d->mh1, d->mk0,
                  d->mk1, d->flags, d->pos, d->d_count, d->samp, d->temp, d->log_h, d->log_k, d->log_i,
                  d->perm, d->sorted_i, d->ord_h, d->ord_k, d->sdev, d->sctl, d->sbh, d->sbk, d->sbi, d->vacc,
                  d->bak_h, d->bak_k, d->mstart, d->fk_in, d->fk_out, d->fv, d->fflag, d->rows_copy};
    for (void* p : ps) pool_device_free(p);  // the owner's stream is idle (rsv_destroy)
    pool_host_free(d->h_pinned);
    pool_host_free(d->hc);
    pool_host_free(d->ph);
    pool_host_free(d->pk);
    pool_host_free(d->pflag);
    pool_host_free(d->ph2);
    pool_host_free(d->pk2);
    pool_host_free(d->pflag2);
    if (d->seg_ev) (void)hipEventDestroy(d->seg_ev);
    pool_host_free(d->pmem);
    pool_host_free(d->shc);
    delete d;
}

int64_t distinct_size(const DistinctState* d) { return d->wide ? wide_size(d->wide) : d->m; }
const void* distinct_keys_dev(const DistinctState* d) { return d->wide ? wide_keys_dev(d->wide) : d->set_k; }

void distinct_spec_target(DistinctState* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t* gen_counter) {
    // the bucketed merge only: set mode behind ctl_publish, ordered mode behind the scheduled pass
    if (d->wide) {
        wide_spec_target(d->wide, dst_host_dev, flag_dev, gen_counter);
        return;
    }
    if (d->log_bmax < 0) return;
    d->spec_dst = dst_host_dev;
    d->spec_flag = flag_dev;
    d->spec_gen_ctr = gen_counter;
    d->spec_ok = false;
}

bool distinct_is_ordered(const DistinctState* d) { return d->ordered; }
int64_t distinct_spec_min(const DistinctState* d) { return d->spec_min; }

bool distinct_spec_take(DistinctState* d, uint32_t* gen) {
    if (d->wide) return wide_spec_take(d->wide, gen);
    const bool ok = d->spec_ok && d->spec_dst;
    if (ok) *gen = d->spec_gen;
    d->spec_dst = nullptr;
    d->spec_arm = d->spec_ok = false;
    return ok;
}

int distinct_publish(DistinctState* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st) {
    if (d->wide) return wide_publish(d->wide, dst_host_dev, flag_dev, gen, st);
    RSV_HIP_TRY(launch_publish_multi(d->set_k, d->m * d->kw, dst_host_dev, flag_dev, gen, (uint32_t*)(d->ctl + 4), st));
    return RSV_OK;
}

template <typename KeyT>
static hipError_t launch_filter(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n,
                                int64_t tinc, hipStream_t st) {
    KeyT* ck = (KeyT*)d->cand_k;
    if (tinc == INT64_MAX && n <= d->cand_cap) {  // no bound: every element a candidate, in place
        const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(n), 1), 4096);
#define RSV_HASH_ALL(H)                                                                                       \
    hipLaunchKernelGGL((hash_all<KeyT, H, false>), dim3(g), dim3(kBlock), 0, st, keys, hashes, n, d->r0, d->r1, \
                       d->cand_h, ck, (uint32_t*)nullptr, d->counter)
        switch (d->hash_kind) {
        case kHashJavaLong: RSV_HASH_ALL(kHashJavaLong); break;
        case kHashJavaInt: RSV_HASH_ALL(kHashJavaInt); break;
        case kHashPrecomputed: RSV_HASH_ALL(kHashPrecomputed); break;
        default: RSV_HASH_ALL(kHashIdentity);
        }
#undef RSV_HASH_ALL
        return hipGetLastError();
    }
    // 32 workgroups per CU over the pass (tools/micro_k3: 2048 -> 8192 workgroups, 5.9 -> 6.4 TB/s)
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(n / 32 + 1), 1), kK3Grid);
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

// span bits of every hash in a merge whose entries are all <= top (rocPRIM and the buckets both
// work on h - INT64_MIN)
static unsigned span_bits(int64_t top) {
    const uint64_t span = (uint64_t)top - (uint64_t)INT64_MIN;
    return span ? 64u - (unsigned)__builtin_clzll(span) : 1u;
}

// ctl[0..5] to the host: published by one wave into coherent memory and spun on (a stream
// synchronize costs ~15-20 us more); falls back to a blocking synchronize after ~2 ms
static hipError_t read_ctl(DistinctState* d, int64_t* out, hipStream_t st) {
    const uint32_t gen = ++d->hc_gen;
    uint32_t* flag = (uint32_t*)(d->hc + 8);
    hipLaunchKernelGGL(ctl_publish, dim3(1), dim3(64), 0, st, d->ctl, d->hc_dev,
                       (uint32_t*)(d->hc_dev + 8), gen);
    if (hipError_t e = hipGetLastError()) return e;
    if (d->spec_arm) {  // behind ctl_publish (which re-arms ctl[0..1]; the kernel reads ctl[2])
        d->spec_arm = false;
        const uint32_t g = ++*d->spec_gen_ctr;
        const int64_t per = 32 * 1024;  // bytes per workgroup, as launch_publish_multi
        const unsigned grid =
            (unsigned)std::min<int64_t>(32, std::max<int64_t>(1, ((int64_t)d->k * d->kw + per - 1) / per));
        hipLaunchKernelGGL(publish_set_kernel, dim3(grid), dim3(1024), 0, st, (const uint32_t*)d->set_k,
                           (uint32_t*)d->spec_dst, (const int64_t*)d->ctl, (int64_t)d->k, d->kw / 4, d->spec_flag,
                           g, (uint32_t*)(d->ctl + 4));
        if (hipError_t e = hipGetLastError()) return e;
        d->spec_gen = g;
    }
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == gen) {
            seen = true;
            break;
        }
        __builtin_ia32_pause();
        if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
    }
    if (!seen) {
        if (hipError_t e = hipStreamSynchronize(st)) return e;
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen) return hipErrorUnknown;
    }
    for (int i = 0; i < 6; ++i) out[i] = __atomic_load_n(d->hc + i, __ATOMIC_RELAXED);
    return hipSuccess;
}

// the filter's candidates (count read on the device) + the current set -> new set, on the
// bucketed path; results land in ctl[1..3] (overflow, distinct count, largest kept h)
template <typename KeyT>
static hipError_t launch_bucket_merge(DistinctState* d, int64_t tinc, hipStream_t st, const int64_t* cand_h = nullptr,
                                      const KeyT* cand_k = nullptr, int64_t cand_cap = 0) {
    if (!cand_h) {  // the set-mode filter's buffer
        cand_h = d->cand_h;
        cand_k = (const KeyT*)d->cand_k;
        cand_cap = d->cand_cap;
    }
    const int64_t top = d->m ? std::max(tinc, d->set_top) : tinc;
    const uint64_t span = (uint64_t)top - (uint64_t)INT64_MIN;
    const uint64_t q = span == UINT64_MAX ? 1ull : UINT64_MAX / (span + 1);
    const unsigned waves = 1u << d->log_bmax;  // one per bucket
    const unsigned wgrid = (waves + kBlock / 64 - 1) / (kBlock / 64);
    const unsigned sgrid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(d->m + cand_cap), 1), 1024);
    KeyT* bk = (KeyT*)d->bk;
    hipLaunchKernelGGL(bucket_scatter<KeyT>, dim3(sgrid), dim3(kBlock), 0, st, d->set_h, (const KeyT*)d->set_k, d->m,
                       cand_h, cand_k, cand_cap, d->ctl, q, d->log_bmax, d->bh, bk);
    hipLaunchKernelGGL(bucket_sort<KeyT>, dim3(wgrid), dim3(kBlock), 0, st, d->m, cand_cap, d->ctl, d->log_bmax,
                       d->bh, bk);
    const unsigned egrid = (waves + kEmitBuckets - 1) / kEmitBuckets;
    hipLaunchKernelGGL(bucket_emit<KeyT>, dim3(egrid), dim3(kBlock), 0, st, d->m, cand_cap, d->ctl, d->log_bmax,
                       (const int64_t*)d->bh, (const KeyT*)bk, (int64_t)d->k, d->set_h, (KeyT*)d->set_k);
    return hipGetLastError();
}

// Merge `c` entries at (src_h, src_k) with the current set; new set = first k distinct by
// (h, key).  Returns the distinct count of the union in *n_distinct.
template <typename KeyT>
static hipError_t merge_into_set(DistinctState* d, const int64_t* src_h, const KeyT* src_k, int64_t c,
                                 int64_t* n_distinct, hipStream_t st, int64_t h_max = INT64_MAX) {
    // every hash in the merge is <= h_max (the filter threshold; the set lies below it too): the
    // keys share their top bits, so the radix passes stop at the highest bit that varies
    // (rocPRIM sorts signed keys as h ^ sign bit = h - INT64_MIN: those are all < 2^hbits)
    unsigned hbits = 64;
    if (h_max != INT64_MAX && (d->m == 0 || d->m == d->k)) {  // else the set's maximum is unknown here
        const int64_t top = d->m == d->k ? std::max(h_max, d->max_h) : h_max;
        hbits = span_bits(top);
    }
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
        if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->mh0, d->mh1, mk0, mk1, (size_t)total, 0, hbits, st)))
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
        if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->mh1, d->mh0, mk1, mk0, (size_t)total, 0, hbits, st)))
            return e;
    }
    hipLaunchKernelGGL(dedup_flags<KeyT>, dim3(grid_1d(total)), dim3(kBlock), 0, st, d->mh0, mk0, total,
                       d->flags);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemsetAsync(d->d_count + 2, 0, 8, st))) return e;
    tb = d->temp_bytes;
    if ((e = rocprim::exclusive_scan(d->temp, tb, d->flags, d->pos, 0u, (size_t)total,
                                     rocprim::plus<uint32_t>(), st)))
        return e;
    hipLaunchKernelGGL(compact_first_k<KeyT>, dim3(grid_1d(total)), dim3(kBlock), 0, st, d->mh0, mk0,
                       d->flags, d->pos, total, (int64_t)d->k, d->set_h, (KeyT*)d->set_k, d->d_count);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync(d->h_pinned, d->d_count, 24, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipStreamSynchronize(st))) return e;
    *n_distinct = d->h_pinned[0];
    d->last_tie = d->h_pinned[2] != 0;
    d->m = std::min<int64_t>(*n_distinct, d->k);
    if (d->m) d->set_top = d->h_pinned[1];
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
    d->spec_ok = false;
    if (n <= 0) return RSV_OK;
    const bool full = d->m == d->k;
    // Set mode keeps the bottom-k by (h, key): an element tied with the current maximum hash can
    // still displace the set's largest key, so the bound is inclusive.  (The reference's strict
    // `h < maxHash`, Sampler.scala:403, makes the tie bucket depend on arrival order; that is
    // RSV_DISTINCT_ORDERED's job.  With an injective hash both agree: no two elements tie.)
    const int64_t t_allowed = full ? d->max_h : INT64_MAX;
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
        if (attempt == 8 && n > d->cand_limit / 2) {
            // A hash with few distinct values near the boundary (e.g. a constant precomputed hash)
            // defeats the threshold search: no threshold keeps between k and cand_cap candidates.
            // Take the batch in slices whose every element fits the candidate buffer (each slice
            // merges in one pass); what the attempts above merged is a subset of the batch.
            const int64_t step = d->cand_limit / 2;
            for (int64_t off = 0; off < n; off += step)
                if (int rc = sample_impl<KeyT>(d, keys + off, hashes ? hashes + off : nullptr, std::min(step, n - off), st))
                    return rc;
            return RSV_OK;
        }
        // the merge needs the set arrays at their full size (set_h/set_k are written by rank)
        const bool bucketed = d->log_bmax >= 0 && d->set_cap >= d->k;
        // candidate counter and overflow word: zeroed at creation and re-armed by every read_ctl
        // (ctl_publish), so no memset dispatch ahead of the filter
        if (d->timer) d->timer->mark(st);
        DTRY(launch_filter<KeyT>(d, keys, hashes, n, tinc, st));
        if (d->timer) d->timer->mark(st);
        if (bucketed) DTRY(launch_bucket_merge<KeyT>(d, tinc, st));
        // large batches: publish the merged set speculatively (used if this pass is the last) --
        // armed only on a pass expected to be final: the analytic first pass, or one whose
        // threshold admits everything; a retry that tightens or widens publishes at result()
        const bool spec = bucketed && d->spec_dst && n >= d->spec_min && (attempt == 0 || tinc >= t_allowed);
        d->spec_arm = spec;
        DTRY(read_ctl(d, d->h_pinned + 4, st));
        const int64_t c = d->h_pinned[4];
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
        if (bucketed && d->h_pinned[5] == 0) {  // merged on the device already
            nd = d->h_pinned[6];
            d->m = std::min<int64_t>(nd, d->k);
            if (d->m) d->set_top = d->h_pinned[7];
            if (d->m == d->k) d->max_h = d->set_top;
        } else {
            if (bucketed)  // bucket overflow: the scatter's counts were not consumed
                DTRY(hipMemsetAsync(d->ctl + kCtlWords, 0, (size_t)kCountStride * 4 << d->log_bmax, st));
            DTRY(merge_into_set<KeyT>(d, d->cand_h, (const KeyT*)d->cand_k, c, &nd, st, tinc));
        }
        // exact once every batch element below the new k-th hash was a candidate
        if (tinc >= t_allowed || (d->m == d->k && d->max_h <= tinc)) {
            d->spec_ok = spec && d->h_pinned[5] == 0;  // merged on the device: the publication holds it
            return RSV_OK;
        }
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

template <typename KeyT>
static hipError_t launch_filter_idx(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n,
                                    int64_t tinc, int64_t* out_h, KeyT* out_k, uint32_t* out_i, int64_t cap,
                                    hipStream_t st) {
    if (tinc == INT64_MAX && n <= cap) {  // no bound (the heap filling): every element in place
        const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(n), 1), 4096);
#define RSV_HASH_ALL(H)                                                                                        \
    hipLaunchKernelGGL((hash_all<KeyT, H, true>), dim3(g), dim3(kBlock), 0, st, keys, hashes, n, d->r0, d->r1, out_h, \
                       out_k, out_i, d->counter)
        switch (d->hash_kind) {
        case kHashJavaLong: RSV_HASH_ALL(kHashJavaLong); break;
        case kHashJavaInt: RSV_HASH_ALL(kHashJavaInt); break;
        case kHashPrecomputed: RSV_HASH_ALL(kHashPrecomputed); break;
        default: RSV_HASH_ALL(kHashIdentity);
        }
#undef RSV_HASH_ALL
        return hipGetLastError();
    }
    // ~8 keys per thread (one 1024-key tile per two waves) up to 8192 workgroups: a short chunk
    // where every key is a candidate (the heap filling) would otherwise run on a few waves
    // (132k keys: 17 workgroups, 18 us)
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(n / 8 + 1), 1), 256 * 32);
#define RSV_FILTER_IDX(H)                                                                                       \
    hipLaunchKernelGGL((k3_filter<KeyT, H, true>), dim3(grid), dim3(kBlock), 0, st, keys, hashes, n, d->r0,     \
                       d->r1, tinc, out_h, out_k, d->counter, cap, out_i)
    switch (d->hash_kind) {
    case kHashJavaLong: RSV_FILTER_IDX(kHashJavaLong); break;
    case kHashJavaInt: RSV_FILTER_IDX(kHashJavaInt); break;
    case kHashPrecomputed: RSV_FILTER_IDX(kHashPrecomputed); break;
    default: RSV_FILTER_IDX(kHashIdentity);
    }
#undef RSV_FILTER_IDX
    return hipGetLastError();
}

// ordered-mode replay buffers: device permutation / sort output and pinned host copies of one
// logged segment
static hipError_t ensure_ordered(DistinctState* d, int64_t cap, hipStream_t st) {
    if (cap <= d->ord_cap) return hipSuccess;
    hipError_t e;
    if ((e = grow((void**)&d->perm, 0, (size_t)cap * 4, false, st))) return e;
    if ((e = grow((void**)&d->sorted_i, 0, (size_t)cap * 4, false, st))) return e;
    if ((e = grow((void**)&d->ord_h, 0, (size_t)cap * 8, false, st))) return e;
    if ((e = grow(&d->ord_k, 0, (size_t)cap * d->kw, false, st))) return e;
    pool_host_free(d->ph);
    pool_host_free(d->pk);
    d->ph = nullptr;
    d->pk = nullptr;
    if ((e = pool_host_alloc((void**)&d->ph, (size_t)cap * 8, hipHostMallocDefault))) return e;
    if ((e = pool_host_alloc(&d->pk, (size_t)cap * d->kw, hipHostMallocDefault))) return e;
    if ((e = grow((void**)&d->fflag, 0, (size_t)cap, false, st))) return e;
    pool_host_free(d->pflag);
    d->pflag = nullptr;
    if ((e = pool_host_alloc((void**)&d->pflag, (size_t)cap, hipHostMallocDefault))) return e;
    size_t tb = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                       rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (size_t)cap)))
        return e;
    if (tb > d->temp_bytes) {
        if ((e = grow(&d->temp, 0, tb, false, st))) return e;
        d->temp_bytes = tb;
    }
    d->ord_cap = cap;
    return hipSuccess;
}

// room for `need` log entries (kept contents).  The first allocation takes ~8 full chunks (at most
// 256 MB): a growth copies the log and waits for the stream (~100 us each, measured).
static hipError_t ensure_log(DistinctState* d, int64_t need, hipStream_t st) {
    if (need <= d->log_cap) return hipSuccess;
    const int64_t first = std::min<int64_t>(8 * d->cand_limit, (256ll << 20) / (12 + d->kw));
    const int64_t want = std::max(need, std::min(d->log_limit, d->log_cap ? need : first));
    const int64_t c = grown(d->log_cap, want, std::max(want, d->log_limit));
    hipError_t e;
    if ((e = grow((void**)&d->log_h, (size_t)d->log_n * 8, (size_t)c * 8, true, st))) return e;
    if ((e = grow(&d->log_k, (size_t)d->log_n * d->kw, (size_t)c * d->kw, true, st))) return e;
    if ((e = grow((void**)&d->log_i, (size_t)d->log_n * 4, (size_t)c * 4, true, st))) return e;
    d->log_cap = c;
    return hipSuccess;
}

// The replica's set -> the device set arrays (ascending (h, key), as the SET mode keeps them), so
// result / export / merge read the same place in both modes.
template <typename KeyT>
static hipError_t upload_replica(DistinctState* d, hipStream_t st) {
    // the heap's entries go up in heap order and are put in ascending (h, key) order on the device by
    // two stable radix sorts, key then h (a host std::sort of k = 65536 entries took ~3 ms)
    const int64_t m = d->rep.size();
    hipError_t e = ensure_caps(d, 0, m, st);
    if (e != hipSuccess || m == 0) {
        d->m = 0;
        return e;
    }
    std::vector<KeyT> kk((size_t)m);
    for (int64_t i = 0; i < m; ++i) kk[(size_t)i] = (KeyT)d->rep.he[(size_t)i + 1];
    if ((e = hipMemcpyAsync(d->mh0, d->rep.hh.data() + 1, (size_t)m * 8, hipMemcpyHostToDevice, st))) return e;
    if ((e = hipMemcpyAsync(d->mk0, kk.data(), (size_t)m * sizeof(KeyT), hipMemcpyHostToDevice, st))) return e;
    size_t tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, (KeyT*)d->mk0, (KeyT*)d->mk1, d->mh0, d->mh1, (size_t)m, 0,
                                       8 * (unsigned)sizeof(KeyT), st)))
        return e;
    tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->mh1, d->set_h, (KeyT*)d->mk1, (KeyT*)d->set_k, (size_t)m, 0,
                                       64, st)))
        return e;
    if ((e = hipStreamSynchronize(st))) return e;  // kk goes out of scope
    d->m = m;
    d->max_h = d->rep.max_hash;
    d->set_top = d->rep.hh[1];  // the heap's root: the set's largest hash
    return hipSuccess;
}

// the first-occurrence sort's buffers for `total` entries (members + one segment)
template <typename KeyT>
static hipError_t ensure_first(DistinctState* d, int64_t nm, int64_t total, hipStream_t st) {
    hipError_t e;
    if (nm > d->pmem_cap) {
        const int64_t c = std::min<int64_t>(d->k, std::max<int64_t>(nm, 2 * d->pmem_cap));
        pool_host_free(d->pmem);
        d->pmem = nullptr;
        d->pmem_cap = 0;
        if ((e = pool_host_alloc(&d->pmem, (size_t)c * sizeof(KeyT), hipHostMallocDefault))) return e;
        d->pmem_cap = c;
    }
    if (total <= d->fcap) return hipSuccess;
    if ((e = grow(&d->fk_in, 0, (size_t)total * sizeof(KeyT), false, st))) return e;
    if ((e = grow(&d->fk_out, 0, (size_t)total * sizeof(KeyT), false, st))) return e;
    if ((e = grow((void**)&d->fv, 0, (size_t)total * 4, false, st))) return e;
    size_t tb = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, tb, (KeyT*)nullptr, (KeyT*)nullptr,
                                       rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (size_t)total)))
        return e;
    if (tb > d->temp_bytes) {
        if ((e = grow(&d->temp, 0, tb, false, st))) return e;
        d->temp_bytes = tb;
    }
    d->fcap = total;
    return hipSuccess;
}

// One logged segment in arrival order into the pinned host copies d->ph / d->pk: a radix sort by
// the chunk-relative index restores the order, and the permutation is applied on the device, so
// the host reads the segment sequentially (two random reads per element from a ~20 MB log cost
// more than the replica's heap).  With `first`, also its first-occurrence flags into d->pflag.
template <typename KeyT>
static hipError_t segment_to_host(DistinctState* d, const DistinctState::Seg& g, hipStream_t st, bool first,
                                  bool sync = true) {
    hipError_t e;
    if ((e = ensure_ordered(d, g.c, st))) return e;
    unsigned bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < (uint64_t)g.m) ++bits;
    size_t tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->log_i + g.off, d->sorted_i,
                                       rocprim::counting_iterator<uint32_t>(0), d->perm, (size_t)g.c, 0, bits, st)))
        return e;
    hipLaunchKernelGGL(permute_log<KeyT>, dim3((unsigned)std::min<int64_t>((g.c + kBlock - 1) / kBlock, 8192)),
                       dim3(kBlock), 0, st, d->perm, d->log_h + g.off, (const KeyT*)d->log_k + g.off, g.c, d->ord_h,
                       (KeyT*)d->ord_k);
    if ((e = hipGetLastError())) return e;
    if (first) {
        const int64_t nm = d->rep.size(), total = nm + g.c;
        if ((e = ensure_first<KeyT>(d, nm, total, st))) return e;
        KeyT* pm = (KeyT*)d->pmem;
        for (int64_t i = 0; i < nm; ++i) pm[i] = (KeyT)d->rep.he[(size_t)i + 1];
        if (nm && (e = hipMemcpyAsync(d->fk_in, pm, (size_t)nm * sizeof(KeyT), hipMemcpyHostToDevice, st))) return e;
        if ((e = hipMemcpyAsync((KeyT*)d->fk_in + nm, d->ord_k, (size_t)g.c * sizeof(KeyT), hipMemcpyDeviceToDevice, st)))
            return e;
        size_t fb = d->temp_bytes;
        if ((e = rocprim::radix_sort_pairs(d->temp, fb, (KeyT*)d->fk_in, (KeyT*)d->fk_out,
                                           rocprim::counting_iterator<uint32_t>(0), d->fv, (size_t)total, 0,
                                           8 * (unsigned)sizeof(KeyT), st)))
            return e;
        hipLaunchKernelGGL(mark_first<KeyT>, dim3((unsigned)std::min<int64_t>((total + kBlock - 1) / kBlock, 8192)),
                           dim3(kBlock), 0, st, (const KeyT*)d->fk_out, (const uint32_t*)d->fv, total, (uint32_t)nm,
                           d->fflag);
        if ((e = hipGetLastError())) return e;
        if ((e = hipMemcpyAsync(d->pflag, d->fflag, (size_t)g.c, hipMemcpyDeviceToHost, st))) return e;
    }
    if ((e = hipMemcpyAsync(d->ph, d->ord_h, (size_t)g.c * 8, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipMemcpyAsync(d->pk, d->ord_k, (size_t)g.c * sizeof(KeyT), hipMemcpyDeviceToHost, st))) return e;
    if (sync) return hipStreamSynchronize(st);
    // the caller enqueues more (the next segment's staging), then waits for this event only
    if (!d->seg_ev && (e = hipEventCreateWithFlags(&d->seg_ev, hipEventDisableTiming))) return e;
    return hipEventRecord(d->seg_ev, st);
}

static void archive_drop(DistinctState* d) {
    d->arch_ok = false;
    std::vector<int64_t>().swap(d->arch_h);
    std::vector<int64_t>().swap(d->arch_k);
    std::vector<int32_t>().swap(d->arch_k4);
}

// The replica from the set arrays, in (h, key) order, after a merge replaced the set (a merged set
// has no single arrival order; rsv_merge_log is the exact form).
template <typename KeyT>
static hipError_t rebuild_replica(DistinctState* d, hipStream_t st) {
    std::vector<int64_t> hh((size_t)d->m);
    std::vector<KeyT> kk((size_t)d->m);
    hipError_t e = hipSuccess;
    if (d->m) {
        if ((e = hipMemcpyAsync(hh.data(), d->set_h, (size_t)d->m * 8, hipMemcpyDeviceToHost, st))) return e;
        if ((e = hipMemcpyAsync(kk.data(), d->set_k, (size_t)d->m * sizeof(KeyT), hipMemcpyDeviceToHost, st))) return e;
        if ((e = hipStreamSynchronize(st))) return e;
    }
    d->rep.reset(d->k);
    for (int64_t i = 0; i < d->m; ++i) d->rep.sample((int64_t)kk[(size_t)i], hh[(size_t)i]);
    if (d->m == d->k) d->max_h = d->rep.max_hash;
    d->rep_stale = false;
    return hipSuccess;
}

// The next segment's host copies staged while the host replays this one (replay_log): segment gn in
// arrival order into the pinned buffers the current run does not read, with first-occurrence flags
// taken against the members at the START of the current segment gs plus all of gs's keys -- the
// replica's members at gn's start are a subset of those, and a key of gs that is no member there
// cannot be admitted at gn either (rejected at its first arrival, or evicted as the heap's maximum:
// maxHash has not risen since, Sampler.scala:403), so the flags are exactly as exact as gn's own
// would be.  gs's keys are still in ord_k (put there in arrival order for gs's own copies).  Enqueued
// only: the caller synchronizes the stream before it reads the copies.
template <typename KeyT>
static hipError_t segment_stage_next(DistinctState* d, const DistinctState::Seg& gs, const DistinctState::Seg& gn,
                                     int64_t* dph, void* dpk, uint8_t* dpflag, hipStream_t st) {
    hipError_t e;
    const int64_t nm = d->rep.size();  // the members at gs's start (gs has not been replayed yet)
    const int64_t total = nm + gs.c + gn.c;
    KeyT* pm = (KeyT*)d->pmem;  // free: the stream was synchronized since its last upload
    for (int64_t i = 0; i < nm; ++i) pm[i] = (KeyT)d->rep.he[(size_t)i + 1];
    if (nm && (e = hipMemcpyAsync(d->fk_in, pm, (size_t)nm * sizeof(KeyT), hipMemcpyHostToDevice, st))) return e;
    if ((e = hipMemcpyAsync((KeyT*)d->fk_in + nm, d->ord_k, (size_t)gs.c * sizeof(KeyT), hipMemcpyDeviceToDevice, st)))
        return e;
    unsigned bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < (uint64_t)gn.m) ++bits;
    size_t tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->log_i + gn.off, d->sorted_i,
                                       rocprim::counting_iterator<uint32_t>(0), d->perm, (size_t)gn.c, 0, bits, st)))
        return e;
    hipLaunchKernelGGL(permute_log<KeyT>, dim3((unsigned)std::min<int64_t>((gn.c + kBlock - 1) / kBlock, 8192)),
                       dim3(kBlock), 0, st, d->perm, d->log_h + gn.off, (const KeyT*)d->log_k + gn.off, gn.c, d->ord_h,
                       (KeyT*)d->ord_k);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync((KeyT*)d->fk_in + nm + gs.c, d->ord_k, (size_t)gn.c * sizeof(KeyT), hipMemcpyDeviceToDevice,
                            st)))
        return e;
    size_t fb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, fb, (KeyT*)d->fk_in, (KeyT*)d->fk_out,
                                       rocprim::counting_iterator<uint32_t>(0), d->fv, (size_t)total, 0,
                                       8 * (unsigned)sizeof(KeyT), st)))
        return e;
    hipLaunchKernelGGL(mark_first<KeyT>, dim3((unsigned)std::min<int64_t>((total + kBlock - 1) / kBlock, 8192)),
                       dim3(kBlock), 0, st, (const KeyT*)d->fk_out, (const uint32_t*)d->fv, total,
                       (uint32_t)(nm + gs.c), d->fflag);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync(dpflag, d->fflag, (size_t)gn.c, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipMemcpyAsync(dph, d->ord_h, (size_t)gn.c * 8, hipMemcpyDeviceToHost, st))) return e;
    return hipMemcpyAsync(dpk, d->ord_k, (size_t)gn.c * sizeof(KeyT), hipMemcpyDeviceToHost, st);
}

// the alternate pinned copies for segments of up to `cap` candidates
static hipError_t ensure_ordered2(DistinctState* d, int64_t cap) {
    if (cap <= d->ord2_cap) return hipSuccess;
    hipError_t e;
    pool_host_free(d->ph2);
    pool_host_free(d->pk2);
    pool_host_free(d->pflag2);
    if (d->seg_ev) (void)hipEventDestroy(d->seg_ev);
    d->ph2 = nullptr;
    d->pk2 = nullptr;
    d->pflag2 = nullptr;
    d->ord2_cap = 0;
    if ((e = pool_host_alloc((void**)&d->ph2, (size_t)cap * 8, hipHostMallocDefault))) return e;
    if ((e = pool_host_alloc(&d->pk2, (size_t)cap * d->kw, hipHostMallocDefault))) return e;
    if ((e = pool_host_alloc((void**)&d->pflag2, (size_t)cap, hipHostMallocDefault))) return e;
    d->ord2_cap = cap;
    return hipSuccess;
}

// Every logged segment, in order, through the host replica (RandomValues.sample on each candidate,
// Sampler.scala:394-409); the consumed candidates are kept in the host archive for rsv_export_log
// when the sampler retains its log (rsv_retain_log).  When two consecutive segments both replay
// through the first-occurrence flags, the next one's sort, flags and copies run on the device while
// the host replays the current one (segment_stage_next; C4's hash-twin share: the second segment's
// 0.76 ms to the host hidden under the first one's 2.4 ms heap run).
template <typename KeyT>
static hipError_t replay_log(DistinctState* d, hipStream_t st) {
    hipError_t e;
    if (d->rep_stale && (e = rebuild_replica<KeyT>(d, st))) return e;
    // (the flags' sort holds the members too: ~20 B per entry on the device, so a huge replica
    // keeps the set-based form)
    auto first_ok = [&](int64_t c, int64_t extra) {
        return c >= d->first_min && d->rep.size() + extra + c <= ((int64_t)1 << 28);
    };
    const size_t ns = d->segs.size();
    if (d->overlap && ns >= 2) {  // every buffer at its final size first: a growth would drop ord_k
        int64_t cmax = 0, pair = 0;
        for (size_t s = 0; s < ns; ++s) {
            cmax = std::max(cmax, d->segs[s].c);
            if (s + 1 < ns) pair = std::max(pair, d->segs[s].c + d->segs[s + 1].c);
        }
        if ((e = ensure_ordered(d, cmax, st))) return e;
        if ((e = ensure_first<KeyT>(d, d->k, d->k + pair, st))) return e;
        if ((e = ensure_ordered2(d, cmax))) return e;
    }
    // the pinned copies of a segment: set 0 (ph / pk / pflag, segment_to_host's, which may grow them)
    // or set 1 (ph2 / pk2 / pflag2)
    auto set_h = [&](int c) { return c ? d->ph2 : d->ph; };
    auto set_k = [&](int c) { return c ? d->pk2 : d->pk; };
    auto set_f = [&](int c) { return c ? d->pflag2 : d->pflag; };
    bool staged = false;  // segment s's copies (and flags) were staged behind the previous run
    int cur = 0;          // the set segment s's copies are in
    for (size_t s = 0; s < ns; ++s) {
        const DistinctState::Seg& g = d->segs[s];
        if (g.c == 0) {
            staged = false;
            continue;
        }
        static const bool debug = std::getenv("RSV_REPLAY_DEBUG") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        bool first = true;
        if (staged) {  // staged behind the previous segment's run: wait for its copies
            if ((e = hipStreamSynchronize(st))) return e;
            cur ^= 1;
        }
        // the next segment is staged behind this one when both replay through the flags
        const DistinctState::Seg* gn = s + 1 < ns ? &d->segs[s + 1] : nullptr;
        const int64_t nm = d->rep.size();
        const bool stage_next = d->overlap && d->ph2 && gn && gn->c > 0 && first_ok(gn->c, g.c) &&
                                nm + g.c + gn->c <= d->fcap && gn->c <= d->ord2_cap && gn->c <= d->ord_cap &&
                                d->pmem_cap >= nm;
        if (!staged) {
            first = first_ok(g.c, 0);
            // (when staging follows, wait only for this segment's own copies, after enqueueing it)
            if ((e = segment_to_host<KeyT>(d, g, st, first, !(stage_next && first)))) return e;
            cur = 0;
        }
        const bool was_staged = staged;
        staged = false;
        if (stage_next && first) {
            if ((e = segment_stage_next<KeyT>(d, g, *gn, set_h(cur ^ 1), set_k(cur ^ 1), set_f(cur ^ 1), st))) return e;
            staged = true;
            if (!was_staged && (e = hipEventSynchronize(d->seg_ev))) return e;
        }
        const auto t1 = std::chrono::steady_clock::now();
        const KeyT* pk = (const KeyT*)set_k(cur);
        const int64_t* ph = set_h(cur);
        const uint8_t* pflag = set_f(cur);
        if (d->retain && d->arch_ok) {
            if ((int64_t)d->arch_h.size() + g.c > kArchMax) {
                archive_drop(d);
            } else {
                d->arch_h.insert(d->arch_h.end(), ph, ph + g.c);
                if constexpr (sizeof(KeyT) == 8) d->arch_k.insert(d->arch_k.end(), pk, pk + g.c);
                else d->arch_k4.insert(d->arch_k4.end(), pk, pk + g.c);
            }
        }
        if (first)
            d->rep.sample_run_unique(g.c, pflag, [&](int64_t t) { return (int64_t)pk[t]; },
                                     [&](int64_t t) { return ph[t]; });
        else
            d->rep.sample_run(g.c, [&](int64_t t) { return (int64_t)pk[t]; }, [&](int64_t t) { return ph[t]; });
        if (debug) {
            const auto t2 = std::chrono::steady_clock::now();
            int64_t kept = 0;
            if (first)
                for (int64_t t = 0; t < g.c; ++t) kept += pflag[t];
            std::fprintf(stderr, "[rsv replay] candidates=%lld first=%d kept=%lld staged_next=%d to_host_us=%.1f run_us=%.1f\n",
                         (long long)g.c, (int)first, (long long)kept, (int)staged,
                         std::chrono::duration<double, std::micro>(t1 - t0).count(),
                         std::chrono::duration<double, std::micro>(t2 - t1).count());
        }
    }
    if (staged && (e = hipStreamSynchronize(st))) return e;  // (never: the last segment stages nothing)
    d->segs.clear();
    if (d->pre_segs.empty()) d->log_n = 0;  // else the log still holds the pre-merge segments
    return hipSuccess;
}

// the scheduled pass's buffers for merges of up to `entries` (set + candidates); allocated on first use
template <typename KeyT>
static hipError_t sched_ensure(DistinctState* d, int32_t lb, hipStream_t st, bool defer_zero = false) {
    hipError_t e = hipSuccess;
    if (!d->sdev) {
        if ((e = pool_device_alloc((void**)&d->sdev, sizeof(SchedDev)))) return e;
        if ((e = pool_host_alloc((void**)&d->shc, 128, hipHostMallocCoherent | hipHostMallocMapped))) return e;
        if ((e = hipHostGetDevicePointer((void**)&d->shc_dev, d->shc, 0))) return e;
        ((uint32_t*)(d->shc + 12))[0] = 0;
        if ((e = pool_device_alloc((void**)&d->vacc, (size_t)kVerifyCopies * (kMaxRanges + 1) * 4))) return e;
        d->sdirty = true;  // re-armed by sched_publish after every pass
        if ((e = pool_device_alloc((void**)&d->bak_h, (size_t)d->k * 8))) return e;
        if ((e = pool_device_alloc(&d->bak_k, (size_t)d->k * d->kw))) return e;
    }
    if (lb > d->log_bmax_s) {
        // the old area may still be read by queued work: wait before it goes back to the pool
        if (d->sctl && (e = hipStreamSynchronize(st))) return e;
        for (void* p : {(void*)d->sctl, (void*)d->sbh, d->sbk, (void*)d->sbi}) pool_device_free(p);
        d->sctl = nullptr;
        d->sbh = nullptr;
        d->sbk = nullptr;
        d->sbi = nullptr;
        d->log_bmax_s = -1;
        const size_t B = (size_t)1 << lb;
        // rounded to 256 B: one aligned fill dispatch (an unaligned tail costs a second one)
        const size_t ctl_bytes = (kCtlWords * 8 + (kCountStride + 1) * 4 * B + 4 * ((B >> 4) + 1) + 255) & ~(size_t)255;
        if ((e = pool_device_alloc((void**)&d->sctl, ctl_bytes))) return e;
        d->sdirty = true;  // counts, counter: re-armed after each pass
        if ((e = pool_device_alloc((void**)&d->sbh, B * kBucketCap * 8))) return e;
        if ((e = pool_device_alloc(&d->sbk, B * kBucketCap * sizeof(KeyT)))) return e;
        if ((e = pool_device_alloc((void**)&d->sbi, B * kBucketCap * 4))) return e;
        d->log_bmax_s = lb;
    }
    // zeroed here unless the caller's next pass is the fused one (ctl_plan + sched_filter zero
    // them: two fills and their host calls fewer ahead of a fresh sampler's first kernel)
    if (d->sdirty && !defer_zero) {
        const size_t B = (size_t)1 << d->log_bmax_s;
        if ((e = hipMemsetAsync(d->vacc, 0, (size_t)kVerifyCopies * (kMaxRanges + 1) * 4, st))) return e;
        if ((e = hipMemsetAsync(d->sctl, 0, kCtlWords * 8 + kCountStride * 4 * B, st))) return e;
        d->sdirty = false;
    }
    return hipSuccess;
}

// Buffer sizes of a scheduled pass expecting c_pred candidates: its log entries (cap) and merge
// buckets (2^lb, ~<= 64 entries per bucket: most sort in a single 64-lane pass); false: > 1 GiB of
// buckets (the chunk loop instead)
static bool sched_sizes(int64_t k, double c_pred, int64_t* cap, int32_t* lb) {
    *cap = std::min<int64_t>((int64_t)(1.5 * c_pred) + 4 * 4096, ((int64_t)1 << 31) - 1);
    int32_t l = 1;
    while (((int64_t)1 << (l + 6)) < k + *cap) ++l;
    *lb = l;
    return (((int64_t)kBucketCap * 8 + 20) << l) <= ((int64_t)1 << 30);
}

// a pass over n keys at the heap's first fill: its expected candidates (sched_plan_ranges' c_pred
// with D0 = k and distinct elements arriving at >= 3/4 of the positions)
static double sched_estimate(const DistinctState* d, int64_t n) {
    const double k = (double)d->k;
    return d->sched_beta * k / 0.75 * std::log1p(0.75 * (double)n / k);
}

// The scheduled pass's buffers (and their zeroing) for a batch of n keys, queued ahead of the batch's
// first chunk so that the pass itself starts without a host round trip for them; a pass that needs
// more reallocates in sched_ensure.
template <typename KeyT>
static hipError_t sched_prepare(DistinctState* d, int64_t n, hipStream_t st, bool defer_zero) {
    int64_t cap;
    int32_t lb;
    if (!sched_sizes(d->k, sched_estimate(d, n), &cap, &lb)) return hipSuccess;
    return sched_ensure<KeyT>(d, lb, st, defer_zero);
}

#define STRY(x)                                                                                        \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess) {                                                                        \
            set_error(std::string("distinct (scheduled pass): " #x ": ") + hipGetErrorString(_e));    \
            return _e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;                     \
        }                                                                                              \
    } while (0)

// The pass's kernels over keys[0, n), the plan already in d->sdev (or being written there by a
// kernel ahead of them): candidates into the log from lbase (+ the plan's `off`), the set's
// backup, the bucket merge, the verdict to d->shc; then the speculative publication of the set.
template <typename KeyT>
static int sched_launch(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n, int64_t lbase,
                        int64_t cap, uint32_t B, int32_t lb, hipStream_t st, uint32_t* gen, bool* spec,
                        bool zero = false) {
    const int64_t k = d->k;
    const size_t kw = sizeof(KeyT);
    KeyT* bk = (KeyT*)d->sbk;
    if (d->timer) d->timer->mark(st);
    {
        const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(n / 32 + 1), 1), kK3Grid);
        KeyT* lk = (KeyT*)d->log_k + lbase;
#define RSV_SCHED_FILTER(H)                                                                                        \
    hipLaunchKernelGGL((sched_filter<KeyT, H>), dim3(grid), dim3(kBlock), 0, st, keys, hashes, n, d->r0, d->r1,      \
                       (const SchedDev*)d->sdev, d->log_h + lbase, lk, d->log_i + lbase, d->sctl, cap, d->log_bmax_s,     \
                       zero ? d->vacc : nullptr)
        switch (d->hash_kind) {
        case kHashJavaLong: RSV_SCHED_FILTER(kHashJavaLong); break;
        case kHashJavaInt: RSV_SCHED_FILTER(kHashJavaInt); break;
        case kHashPrecomputed: RSV_SCHED_FILTER(kHashPrecomputed); break;
        default: RSV_SCHED_FILTER(kHashIdentity);
        }
#undef RSV_SCHED_FILTER
        STRY(hipGetLastError());
        // one entry per thread (the count is on the device: sized for the buffer's capacity, idle
        // threads exit): every bucket atomic in flight at once -- a 1024-workgroup grid-stride over
        // ~1.1 M entries waited on ~4 atomics per thread in sequence (61 us)
        const uint32_t C = 1u << bin_log((uint32_t)lb);
        const unsigned fgrid = (unsigned)((k + cap + kBinFileThreads * kBinTile - 1) / (kBinFileThreads * kBinTile));
        hipLaunchKernelGGL(sched_bin_file<KeyT>, dim3(fgrid), dim3(kBinFileThreads), C * 4, st, (const SchedDev*)d->sdev,
                           (const int64_t*)(d->log_h + lbase), (const KeyT*)lk, (const uint32_t*)(d->log_i + lbase),
                           d->sctl, cap, (const int64_t*)d->set_h, (const KeyT*)d->set_k, k, d->sbh, bk, d->sbi,
                           d->bak_h, (KeyT*)d->bak_k);
        STRY(hipGetLastError());
    }
    if (d->timer) d->timer->mark(st);
    hipLaunchKernelGGL(sched_bin_sort<KeyT>, dim3(1u << bin_log((uint32_t)lb)), dim3(kBinSortThreads), 0, st, cap, d->sctl, d->log_bmax_s,
                       d->sbh, bk, d->sbi, (const SchedDev*)d->sdev, d->vacc);
    hipLaunchKernelGGL(bucket_emit<KeyT>, dim3((B + kEmitBuckets - 1) / kEmitBuckets), dim3(kBlock), 0, st, k, cap,
                       d->sctl, d->log_bmax_s, (const int64_t*)d->sbh, (const KeyT*)bk, k, d->set_h, (KeyT*)d->set_k, lb);
    *gen = ++d->sgen;
    // the merged set published speculatively with the verdict (size from sctl[2] on the device):
    // result() takes it if the pass verified and left no tie for the replica to settle
    *spec = d->spec_dst && n >= d->spec_min;
    const int64_t per = 32 * 1024;  // bytes per workgroup, as launch_publish_multi
    const unsigned pgrid =
        *spec ? (unsigned)std::min<int64_t>(32, std::max<int64_t>(1, (k * (int64_t)kw + per - 1) / per)) : 1u;
    const uint32_t g = *spec ? ++*d->spec_gen_ctr : 0u;
    hipLaunchKernelGGL(sched_publish, dim3(pgrid), dim3(1024), 0, st, d->sctl, d->vacc, (const SchedDev*)d->sdev, k,
                       d->shc_dev, (uint32_t*)(d->shc_dev + 12), *gen, (const uint32_t*)d->set_k,
                       *spec ? (uint32_t*)d->spec_dst : nullptr, (int32_t)(kw / 4), d->spec_flag, g,
                       (uint32_t*)(d->ctl + 4));
    STRY(hipGetLastError());
    if (*spec) d->spec_gen = g;
    return RSV_OK;
}

// the host side of a pass's verdict: spin on the flag (a stream synchronize after 50 ms)
static int sched_wait(DistinctState* d, uint32_t gen, hipStream_t st, int64_t* hv) {
    uint32_t* flag = (uint32_t*)(d->shc + 12);
    const auto t0w = std::chrono::steady_clock::now();
    bool seen = false;
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == gen) {
            seen = true;
            break;
        }
        __builtin_ia32_pause();
        if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0w > std::chrono::milliseconds(50)) break;
    }
    if (!seen) {
        STRY(hipStreamSynchronize(st));
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen) STRY(hipErrorUnknown);
    }
    for (int i = 0; i < 9; ++i) hv[i] = __atomic_load_n(d->shc + i, __ATOMIC_RELAXED);
    return RSV_OK;
}

// The verdict of a pass over n elements from bound t0 whose log starts at log_n: the host fields,
// or (false *done) the batch left to the chunk loop with the set restored
template <typename KeyT>
static int sched_finish(DistinctState* d, const int64_t* hv, int64_t n, int64_t t0, int64_t cap, uint32_t B,
                        bool spec, hipStream_t st, bool* done) {
    *done = false;
    const int64_t k = d->k;
    const int64_t c = hv[0];
    static const bool debug = std::getenv("RSV_SCHED_DEBUG") != nullptr;
    if (debug)
        std::fprintf(stderr, "[rsv sched] n=%lld ranges=%lld cand=%lld cap=%lld bucket_overflow=%lld "
                             "failed_range=%lld min_count=%lld k=%lld\n",
                     (long long)n, (long long)hv[8], (long long)c, (long long)cap, (long long)hv[1], (long long)hv[6],
                     (long long)hv[7], (long long)k);
    if (c > cap || hv[1]) {  // buffer or bucket overflow: nothing was merged; the counts were not consumed
        STRY(hipMemsetAsync(d->sctl + kCtlWords, 0, (size_t)kCountStride * 4 * B, st));
        ++d->sched_fallbacks;
        return RSV_OK;
    }
    if (hv[6] >= 0) {  // a predicted bound was too tight: put the set back, the chunk loop redoes the batch
        STRY(hipMemcpyAsync(d->set_h, d->bak_h, (size_t)k * 8, hipMemcpyDeviceToDevice, st));
        STRY(hipMemcpyAsync(d->set_k, d->bak_k, (size_t)k * sizeof(KeyT), hipMemcpyDeviceToDevice, st));
        ++d->sched_fallbacks;
        return RSV_OK;
    }
    ++d->sched_passes;
    const int64_t old_max = d->max_h;
    d->m = std::min<int64_t>(hv[2], k);
    d->set_top = hv[3];
    if (d->m == k) d->max_h = d->set_top;
    if (d->m == k) d->over = hv[5] != 0 || (d->over && d->max_h == old_max);
    d->rate_c = c;
    d->rate_m = n;
    d->rate_span = (double)((uint64_t)t0 - (uint64_t)INT64_MIN) + 1.0;
    d->segs.push_back(DistinctState::Seg{d->log_n, c, n});
    d->log_n += c;
    d->seen += n;
    d->spec_ok = spec && d->m == k && !d->over;  // verified, and no replay will change the set
    *done = true;
    return RSV_OK;
}

// The scheduled pass over keys[0, n) of a batch, heap full (see SchedDev).  Bounds: with D
// distinct elements seen, the k-th smallest hash sits near fraction k / D of the range; D at
// position P is predicted as D0 + dfr (P - S0) (D0 from the current bound, dfr the history's
// distinct fraction, clamped to [0.5, 1]), and range r's bound keeps fraction beta k / D(start)
// (beta = 1.6: a stream whose new-distinct rate falls to ~60% of its history's still verifies).
// Ranges grow geometrically (<= kMaxRanges).  *done = false: nothing changed, run the chunk loop.
template <typename KeyT>
static int sched_sample(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n, hipStream_t st,
                        bool* done) {
    *done = false;
    const int64_t k = d->k;
    if (d->m != k || d->max_h == INT64_MIN || n >= ((int64_t)1 << 31) || d->set_cap < k) return RSV_OK;
    SchedDev plan;
    const int64_t t0 = d->max_h - 1;
    const double c_pred = sched_plan_ranges(&plan, (double)d->seen, t0, n, k, d->sched_beta);
    if (c_pred < 0) return RSV_OK;  // one range: the plain chunk loop does the same work
    int64_t cap;
    int32_t lb;
    if (!sched_sizes(k, c_pred, &cap, &lb)) return RSV_OK;
    sched_plan_map(&plan, k, lb);
    plan.off = 0;
    // the log holds this batch's candidates as one segment
    if (d->log_n + cap > d->log_limit) {
        if (cap > d->log_limit) return RSV_OK;
        if (!d->segs.empty()) STRY(replay_log<KeyT>(d, st));
        if (d->log_n + cap > d->log_limit) return RSV_OK;
    }
    STRY(ensure_log(d, d->log_n + cap, st));
    STRY(sched_ensure<KeyT>(d, lb, st));
    hipLaunchKernelGGL(sched_plan_store, dim3(1), dim3(256), 0, st, plan, d->sdev);
    uint32_t gen;
    bool spec;
    if (int rc = sched_launch<KeyT>(d, keys, hashes, n, d->log_n, cap, plan.B, lb, st, &gen, &spec)) return rc;
    int64_t hv[9];
    if (int rc = sched_wait(d, gen, st, hv)) return rc;
    return sched_finish<KeyT>(d, hv, n, t0, cap, plan.B, spec, st, done);
}

// The heap-filling chunk with the scheduled pass over the rest of the batch behind it, on the
// device without a host turnaround between them (ctl_plan plans the pass from the chunk's merge).
// Launches keys[0, m) as a chunk (candidates at log_n, <= ccap of them) and keys[m, n) as a pass
// (its log right behind the chunk's candidates); waits once, for the pass's verdict; leaves the
// chunk's control words in hp.  *pass: the plan was valid (the pass ran; its verdict in hv).
template <typename KeyT>
static int fused_fill_and_pass(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t m, int64_t n,
                               int64_t ccap, int64_t cap, int32_t lb, hipStream_t st, int64_t* hp, int64_t* hv,
                               bool* pass, bool* spec) {
    int64_t* lh = d->log_h + d->log_n;
    KeyT* lk = (KeyT*)d->log_k + d->log_n;
    if (d->timer) d->timer->mark(st);
    STRY(launch_filter_idx<KeyT>(d, keys, hashes, m, INT64_MAX, lh, lk, d->log_i + d->log_n, ccap, st));
    if (d->timer) d->timer->mark(st);
    STRY(launch_bucket_merge<KeyT>(d, INT64_MAX, st, lh, lk, ccap));
    const uint32_t cgen = ++d->hc_gen;
    const bool zero = d->sdirty;
    hipLaunchKernelGGL(ctl_plan, dim3(1), dim3(64), 0, st, d->ctl, d->hc_dev, (uint32_t*)(d->hc_dev + 8), cgen, ccap,
                       (int64_t)d->k, std::max(1.0, (double)(d->seen + m)), n - m, d->sched_beta, cap, lb, d->sdev,
                       d->sctl, (int)zero);
    STRY(hipGetLastError());
    uint32_t gen;
    if (int rc = sched_launch<KeyT>(d, keys + m, hashes ? hashes + m : nullptr, n - m, d->log_n, cap, 1u << lb, lb, st,
                                    &gen, spec, zero))
        return rc;
    d->sdirty = false;
    if (int rc = sched_wait(d, gen, st, hv)) return rc;
    if (__atomic_load_n((uint32_t*)(d->hc + 8), __ATOMIC_ACQUIRE) != cgen) STRY(hipErrorUnknown);  // stream order
    for (int i = 0; i < 6; ++i) hp[i] = __atomic_load_n(d->hc + i, __ATOMIC_RELAXED);
    *pass = hv[8] >= 2;
    return RSV_OK;
}
#undef STRY

// RSV_DISTINCT_ORDERED: the reference's exact RandomValues (strict `elemHash < maxHash` and the
// scala PriorityQueue's choice among equal hashes, Sampler.scala:394-409), without replaying the
// stream on the host unless a tie forces it.
//
// Let U be the distinct elements seen so far.  Once the heap is full its maximum M is the k-th
// smallest hash of U, and the heap holds every element of U with hash < M (an element below M was
// admitted on arrival -- M only falls -- and is never the maximum that leaves).  So M, and the set
// itself when U has exactly k elements with hash <= M, follow from set arithmetic: the GPU keeps
// the bottom-k by (h, key) of the elements the reference could admit (each chunk filtered strictly
// below the maximum at its start, a superset of the admitted; all of it while the heap fills) and
// the bucketed merge reports whether rank k ties rank k - 1 on h.  Only when more than k admitted
// elements have hash <= M (`over`, sticky while M stays) does the set depend on the heap's history;
// then the logged candidates of every chunk since the last replay go through the host replica in
// arrival order and the replica's set replaces the device set (`distinct_finalize`, at result /
// export / merge).  The log is replayed eagerly when it would outgrow log_limit.
template <typename KeyT>
static int ordered_sample_impl(DistinctState* d, const KeyT* keys, const int64_t* hashes, int64_t n,
                               hipStream_t st) {
#define OTRY(x)                                                                               \
    do {                                                                                      \
        hipError_t _e = (x);                                                                  \
        if (_e != hipSuccess) {                                                               \
            set_error(std::string("distinct (ordered): " #x ": ") + hipGetErrorString(_e));   \
            return _e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;            \
        }                                                                                     \
    } while (0)
    if (n <= 0) return RSV_OK;
    const int64_t k = d->k;
    const int64_t ccap = std::min<int64_t>(d->cand_limit, std::max<int64_t>(4096, 2 * std::min<int64_t>(n, d->cand_limit)));
    OTRY(ensure_caps(d, 0, std::min<int64_t>(k, ccap + d->m), st));
    int64_t pos = 0;
    int64_t m_next = 0;  // chunk length after an overflow retry
    bool sched_tried = !d->sched || d->log_bmax < 0;
    // the heap-filling chunk and the pass behind it in one enqueue (fused_fill_and_pass): its sizes
    int64_t fcap = 0;
    int32_t flb = 0;
    const bool fuse_ok = !sched_tried && n >= 9 * ccap && n < ((int64_t)1 << 31) && d->m < k &&
                         sched_sizes(k, sched_estimate(d, n), &fcap, &flb);
    if (!sched_tried && n >= 9 * ccap && n < ((int64_t)1 << 31)) OTRY(sched_prepare<KeyT>(d, n, st, fuse_ok));
    while (pos < n) {
        const bool full = d->m == k;
        if (full && d->max_h == INT64_MIN) break;  // nothing is < Long.MinValue
        // a full heap and a long rest: one scheduled pass (falls back to the chunks below)
        if (full && !sched_tried && n - pos >= 8 * ccap) {
            sched_tried = true;
            bool done = false;
            if (int rc = sched_sample<KeyT>(d, keys + pos, hashes ? hashes + pos : nullptr, n - pos, st, &done))
                return rc;
            if (done) {
                pos = n;
                break;
            }
            continue;
        }
        const int64_t tinc = full ? d->max_h - 1 : INT64_MAX;
        int64_t m;
        if (m_next) {
            m = m_next;
        } else if (!full) {
            m = std::max<int64_t>(1024, 2 * (k - d->m) + 1024);  // all survive: bounded by the buffer
        } else if (d->rate_m > 0 && d->rate_c > 0) {
            // aim at ~3k candidates (the buffer holds 4k + 4096): the last full chunk's candidate
            // rate, scaled by how far the threshold fell since (the scrambled hash is uniform)
            const double span_now = (double)((uint64_t)tinc - (uint64_t)INT64_MIN) + 1.0;
            const double rate = (double)d->rate_c / (double)d->rate_m * (span_now / d->rate_span);
            m = (int64_t)std::min<double>(std::max<double>(0.75 * (double)ccap / rate, 65536.0), (double)(1ll << 31));
        } else {
            // first chunk at a full heap: a distinct element passes with probability ~ the span
            // below the threshold (the scrambled hash is uniform); repeats of members pass too,
            // so aim at half the usual target (an overflow only costs a shorter retry)
            const double frac = ((double)((uint64_t)tinc - (uint64_t)INT64_MIN) + 1.0) / 18446744073709551616.0;
            m = (int64_t)std::min<double>(std::max<double>(0.375 * (double)ccap / std::max(frac, 1e-18), 65536.0),
                                          (double)(1ll << 31));
        }
        m = std::min(std::min(m, n - pos), std::min<int64_t>(full ? ((int64_t)1 << 31) : ccap, (int64_t)1 << 31));
        if (d->log_n + ccap > d->log_limit && !d->segs.empty()) OTRY(replay_log<KeyT>(d, st));
        OTRY(ensure_log(d, d->log_n + ccap, st));
        int64_t* lh = d->log_h + d->log_n;
        KeyT* lk = (KeyT*)d->log_k + d->log_n;
        const bool bucketed = d->log_bmax >= 0 && d->set_cap >= k;
        int64_t* hp = d->h_pinned + 4;
        // the chunk that may fill the heap, with the pass over the rest planned on the device behind
        // it when the plan's buffers are in place (sched_sample plans on the host: ~18 us of idle GPU
        // between the chunk's merge and the pass, rocprof timeline r03)
        bool pass = false, spec = false;
        int64_t hv[9];
        if (fuse_ok && !sched_tried && !full && bucketed && !m_next && d->m + m >= k && n - pos - m >= 8 * ccap &&
            d->log_n + ccap + fcap <= d->log_limit) {
            sched_tried = true;
            OTRY(ensure_log(d, d->log_n + ccap + fcap, st));
            OTRY(sched_ensure<KeyT>(d, flb, st, true));
            if (int rc = fused_fill_and_pass<KeyT>(d, keys + pos, hashes ? hashes + pos : nullptr, m, n - pos, ccap,
                                                   fcap, flb, st, hp, hv, &pass, &spec))
                return rc;
            if (!pass) sched_tried = false;  // no plan: the chunk loop may still schedule the rest
        } else {
            // candidate counter and overflow word: zeroed at creation and re-armed by every read_ctl
            if (d->timer) d->timer->mark(st);
            OTRY(launch_filter_idx<KeyT>(d, keys + pos, hashes ? hashes + pos : nullptr, m, tinc, lh, lk,
                                         d->log_i + d->log_n, ccap, st));
            if (d->timer) d->timer->mark(st);
            if (bucketed) OTRY(launch_bucket_merge<KeyT>(d, tinc, st, lh, lk, ccap));
            OTRY(read_ctl(d, hp, st));
        }
        const int64_t c = hp[0];
        if (c > ccap) {  // repeats of members (or a degenerate hash) overflowed the buffer: shorter chunk
            m_next = std::max<int64_t>(1, (int64_t)((double)m * ccap / (double)c / 2));
            continue;
        }
        m_next = 0;
        const int64_t old_max = d->max_h;
        bool tie;
        if (bucketed && hp[1] == 0) {  // merged on the device already
            d->m = std::min<int64_t>(hp[2], k);
            if (d->m) d->set_top = hp[3];
            if (d->m == k) d->max_h = d->set_top;
            tie = hp[5] != 0;
        } else {
            if (bucketed)  // bucket overflow: the scatter's counts were not consumed
                OTRY(hipMemsetAsync(d->ctl + kCtlWords, 0, (size_t)kCountStride * 4 << d->log_bmax, st));
            int64_t nd = 0;
            OTRY(merge_into_set<KeyT>(d, lh, lk, c, &nd, st, tinc));
            tie = d->last_tie;
        }
        if (d->m == k) d->over = tie || (full && d->over && d->max_h == old_max);
        if (full) {  // candidate rate at this threshold (chunk sizing)
            d->rate_c = c;
            d->rate_m = m;
            d->rate_span = (double)((uint64_t)tinc - (uint64_t)INT64_MIN) + 1.0;
        }
        d->segs.push_back(DistinctState::Seg{d->log_n, c, m});
        d->log_n += c;
        pos += m;
        d->seen += m;
        if (pass) {  // the pass's verdict, after the chunk's (its log right behind the chunk's)
            bool done = false;
            if (int rc = sched_finish<KeyT>(d, hv, n - pos, d->max_h - 1, fcap, 1u << flb, spec, st, &done)) return rc;
            if (done) {
                pos = n;
                break;
            }
        }
    }
    d->seen += n - pos;  // the rest was rejected wholesale (maxHash == Long.MinValue)
    d->exact = d->m < k || !d->over;
    return RSV_OK;
#undef OTRY
}

int distinct_sample_device(DistinctState* d, const void* keys, const int64_t* hashes, int64_t n,
                           hipStream_t st) {
    if (d->wide) return wide_sample_device(d->wide, keys, hashes, n, st);
    if (int rc = distinct_settle(d, st)) return rc;
    if (d->merged && n > 0) {  // sampling on after a merge: the pre-merge candidates are history
        d->merged = false;
        d->pre_segs.clear();
        if (d->segs.empty()) d->log_n = 0;
        archive_drop(d);
    }
    if (d->ordered)
        return d->kw == 8 ? ordered_sample_impl<int64_t>(d, (const int64_t*)keys, hashes, n, st)
                          : ordered_sample_impl<int32_t>(d, (const int32_t*)keys, hashes, n, st);
    return d->kw == 8 ? sample_impl<int64_t>(d, (const int64_t*)keys, hashes, n, st)
                      : sample_impl<int32_t>(d, (const int32_t*)keys, hashes, n, st);
}

int distinct_finalize(DistinctState* d, hipStream_t st) {
    if (d->wide) return wide_finalize(d->wide, st);
    if (int rc = distinct_settle(d, st)) return rc;
    if (!d->ordered || d->exact) return RSV_OK;
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = d->kw == 8 ? replay_log<int64_t>(d, st) : replay_log<int32_t>(d, st);
    const auto t1 = std::chrono::steady_clock::now();
    if (e == hipSuccess) e = d->kw == 8 ? upload_replica<int64_t>(d, st) : upload_replica<int32_t>(d, st);
    static const bool debug = std::getenv("RSV_REPLAY_DEBUG") != nullptr;
    if (debug)
        std::fprintf(stderr, "[rsv replay] finalize: replay_us=%.1f upload_us=%.1f\n",
                     std::chrono::duration<double, std::micro>(t1 - t0).count(),
                     std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count());
    if (e != hipSuccess) {
        set_error(std::string("distinct (ordered) replay: ") + hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;
    }
    d->exact = true;
    return RSV_OK;
}

int distinct_export(DistinctState* d, void* keys_dev, int64_t* hash_dev, hipStream_t st) {
    if (d->wide) return wide_export(d->wide, keys_dev, hash_dev, st);
    if (d->m == 0) return RSV_OK;
    if (keys_dev) RSV_HIP_TRY(hipMemcpyAsync(keys_dev, d->set_k, d->m * d->kw, hipMemcpyDeviceToDevice, st));
    if (hash_dev) RSV_HIP_TRY(hipMemcpyAsync(hash_dev, d->set_h, d->m * 8, hipMemcpyDeviceToDevice, st));
    return RSV_OK;
}

void distinct_info(const DistinctState* d, int32_t* ordered, int32_t* tied, int32_t* retained, int64_t* size,
                   int64_t* max_hash, int64_t* log_entries, int64_t* sched_passes, int64_t* sched_fallbacks) {
    if (d->wide) {
        *sched_passes = *sched_fallbacks = 0;
        wide_info(d->wide, ordered, tied, retained, size, max_hash, log_entries);
        return;
    }
    *sched_passes = d->sched_passes;
    *sched_fallbacks = d->sched_fallbacks;
    *ordered = d->ordered;
    *tied = d->m == d->k && d->over;
    *retained = d->ordered && d->retain && d->arch_ok;
    *size = d->m;
    *max_hash = d->m ? d->set_top : INT64_MIN;
    int64_t c = (int64_t)d->arch_h.size();
    for (const DistinctState::Seg& g : d->pre_segs) c += g.c;
    for (const DistinctState::Seg& g : d->segs) c += g.c;
    *log_entries = d->ordered ? c : 0;
}

// After a merge replaced the set: an ordered sampler's replica starts over from the union (rebuilt
// lazily, rep_stale); the logged segments stay readable for rsv_export_log until the next sample.
static void merged_bookkeeping(DistinctState* d) {
    d->spec_ok = false;
    if (!d->ordered) return;
    d->rep_stale = true;
    d->pre_segs.insert(d->pre_segs.end(), d->segs.begin(), d->segs.end());
    d->segs.clear();
    d->exact = true;
    d->merged = true;
}

// Merge `parts` external (key, hash) runs (device; run p at keys + p part_len, part_n[p] entries)
// into the set: bottom-k of the union by (h, key).  `over` afterwards says whether more distinct
// elements of the union share the boundary hash than the set keeps (sticky across the chunked
// merges while the maximum stays).  An ordered sampler rebuilds its replica from the union in
// (h, key) order (a merged set has no single arrival order; rsv_merge_log is the exact form) and
// keeps its logged candidates for rsv_export_log until it samples again.
int distinct_merge_parts(DistinctState* d, const void* keys_dev, const int64_t* hash_dev, const int64_t* part_n,
                         int32_t parts, int64_t part_len, hipStream_t st) {
    if (d->wide) return wide_merge_parts(d->wide, keys_dev, hash_dev, part_n, parts, part_len, st);
    int64_t total = 0;
    for (int32_t p = 0; p < parts; ++p) total += std::max<int64_t>(0, std::min(part_n[p], part_len));
    if (int rc = distinct_settle(d, st)) return rc;
    if (total == 0) return RSV_OK;
    if (int rc = distinct_finalize(d, st)) return rc;
    bool tie = d->m == d->k && d->over;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t n = std::max<int64_t>(0, std::min(part_n[p], part_len));
        const uint8_t* kp = (const uint8_t*)keys_dev + (size_t)p * part_len * d->kw;
        const int64_t* hp = hash_dev + (size_t)p * part_len;
        for (int64_t off = 0; off < n;) {  // chunks that fit the merge buffer
            const int64_t c = std::min<int64_t>(n - off, d->cand_limit);
            const int64_t old_max = d->max_h;
            const bool was_full = d->m == d->k;
            int64_t nd = 0;
            hipError_t e = d->kw == 8
                               ? merge_into_set<int64_t>(d, hp + off, (const int64_t*)kp + off, c, &nd, st)
                               : merge_into_set<int32_t>(d, hp + off, (const int32_t*)kp + off, c, &nd, st);
            if (e != hipSuccess) {
                set_error(std::string("distinct_merge: ") + hipGetErrorString(e));
                return RSV_E_DEVICE;
            }
            tie = d->m == d->k && (d->last_tie || (tie && was_full && d->max_h == old_max));
            off += c;
        }
    }
    d->over = tie;
    merged_bookkeeping(d);
    return RSV_OK;
}

// ---- packed rows (rsv_export_packed / rsv_merge_packed) ----------------------------------------

int distinct_export_row(DistinctState* d, int64_t* row, int64_t count, hipStream_t st) {
    if (d->wide) return wide_export_row(d->wide, row, count, st);
    if (int rc = distinct_settle(d, st)) return rc;
    if (int rc = distinct_finalize(d, st)) return rc;
    const int64_t k = d->k;
    const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid_1d(k), 1), 2048);
    const int64_t tied = d->m == k && d->over, mx = d->m ? d->set_top : INT64_MIN;
    const int64_t ret = d->ordered && d->retain && d->arch_ok;
    if (d->kw == 8)
        hipLaunchKernelGGL(export_row_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, st, (const int64_t*)d->set_h,
                           (const int64_t*)d->set_k, d->m, k, row, count, tied, mx, ret, (int64_t)d->ordered);
    else
        hipLaunchKernelGGL(export_row_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, st, (const int64_t*)d->set_h,
                           (const int32_t*)d->set_k, d->m, k, row, count, tied, mx, ret, (int64_t)d->ordered);
    RSV_HIP_TRY(hipGetLastError());
    return RSV_OK;
}

// The radix-sort form of a rows merge (host waits): rows whose merge overflows a bucket (a
// degenerate hash), more than 64 rows, or buckets beyond 1 GiB.  `over` as the device form sets it.
template <typename KeyT>
static int merge_rows_radix(DistinctState* d, const int64_t* rows, int32_t parts, int64_t stride, hipStream_t st) {
    const int64_t k = d->k;
    std::vector<int64_t> meta((size_t)parts * kRowMeta);
    for (int32_t p = 0; p < parts; ++p)
        RSV_HIP_TRY(hipMemcpyAsync(meta.data() + (size_t)p * kRowMeta, rows + (size_t)p * stride + 2 * k,
                                   kRowMeta * 8, hipMemcpyDeviceToHost, st));
    RSV_HIP_TRY(hipStreamSynchronize(st));
    // the cut's tie rule (runs_top): the smallest maximum of a full run, tied there
    int64_t T = d->m == k ? d->set_top : INT64_MAX;
    bool tiedT = d->m == k && d->over;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t* mt = meta.data() + (size_t)p * kRowMeta;
        if (std::min(std::max<int64_t>(mt[0], 0), k) != k) continue;
        if (mt[3] < T) {
            T = mt[3];
            tiedT = mt[2] != 0;
        } else if (mt[3] == T) {
            tiedT = tiedT || mt[2] != 0;
        }
    }
    bool tie = d->m == k && d->over;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t n = std::min(std::max<int64_t>(meta[(size_t)p * kRowMeta], 0), k);
        if (n == 0) continue;
        const int64_t* rk = rows + (size_t)p * stride;
        const KeyT* keys = (const KeyT*)rk;
        if constexpr (sizeof(KeyT) == 4) {  // row keys are int64-widened
            RSV_HIP_TRY(ensure_caps(d, std::min<int64_t>(n, d->cand_limit), 0, st));
            keys = (const KeyT*)d->cand_k;
        }
        for (int64_t off = 0; off < n;) {  // chunks that fit the merge buffer
            const int64_t c = std::min<int64_t>(n - off, d->cand_limit);
            if constexpr (sizeof(KeyT) == 4) {
                hipLaunchKernelGGL(narrow_keys<KeyT>, dim3((unsigned)std::min<int64_t>(grid_1d(c), 1024)), dim3(kBlock),
                                   0, st, rk + off, c, (KeyT*)d->cand_k);
                RSV_HIP_TRY(hipGetLastError());
            }
            const int64_t old_max = d->max_h;
            const bool was_full = d->m == k;
            int64_t nd = 0;
            RSV_HIP_TRY(merge_into_set<KeyT>(d, rk + k + off, sizeof(KeyT) == 4 ? keys : keys + off, c, &nd, st));
            tie = d->m == k && (d->last_tie || (tie && was_full && d->max_h == old_max));
            off += c;
        }
    }
    d->over = d->m == k && (tie || (tiedT && d->set_top == T));
    return RSV_OK;
}

// Settle a pending device merge: wait for its published words (normally long since there) and take
// the new set's size, maximum and tie state; a bucket overflow redoes the merge on the radix path.
template <typename KeyT>
static int settle_impl(DistinctState* d, hipStream_t st) {
    d->pend = false;
    uint32_t* flag = (uint32_t*)(d->shc + 12);
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == d->pend_gen) {
            seen = true;
            break;
        }
        __builtin_ia32_pause();
        if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) break;
    }
    if (!seen) {
        RSV_HIP_TRY(hipStreamSynchronize(st));
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != d->pend_gen) RSV_HIP_TRY(hipErrorUnknown);
    }
    int64_t hv[8];
    for (int i = 0; i < 8; ++i) hv[i] = __atomic_load_n(d->shc + i, __ATOMIC_RELAXED);
    const int64_t k = d->k;
    if (hv[1])  // a bucket overflowed (rows_sort): nothing was merged
        return merge_rows_radix<KeyT>(d, d->pend_rows, d->pend_parts, d->pend_stride, st);
    d->m = std::min<int64_t>(hv[2], k);
    if (d->m) d->set_top = hv[3];
    if (d->m == k) d->max_h = d->set_top;
    d->over = d->m == k && (hv[5] != 0 || ((hv[6] & 2) && d->set_top == hv[7]));
    return RSV_OK;
}

int distinct_settle(DistinctState* d, hipStream_t st) {
    if (!d->pend) return RSV_OK;  // (wide-key merges complete before they return: never pending)
    return d->kw == 8 ? settle_impl<int64_t>(d, st) : settle_impl<int32_t>(d, st);
}

template <typename KeyT>
static int merge_rows_impl(DistinctState* d, const int64_t* rows, int32_t parts, int64_t stride, hipStream_t st) {
    const int64_t k = d->k;
    const int64_t total = d->m + (int64_t)parts * k;
    int32_t lb = 1;  // <= 64 entries per bucket on average: most sort in one 64-lane pass
    while (((int64_t)1 << (lb + 6)) < total) ++lb;
    const bool device = parts <= 64 && (((int64_t)kBucketCap * (8 + (int64_t)sizeof(KeyT)) + 20) << lb) <= ((int64_t)1 << 30);
    if (!device) {
        if (int rc = merge_rows_radix<KeyT>(d, rows, parts, stride, st)) return rc;
        merged_bookkeeping(d);
        return RSV_OK;
    }
    RSV_HIP_TRY(ensure_caps(d, 0, k, st));  // bucket_emit writes the set by rank: full-size arrays
    RSV_HIP_TRY(sched_ensure<KeyT>(d, lb, st));
    const uint32_t B = 1u << lb;
    const int64_t need = (int64_t)(parts + 1) * (B + 1);
    if (need > d->mstart_cap) {
        RSV_HIP_TRY(grow((void**)&d->mstart, 0, (size_t)need * 4, false, st));
        d->mstart_cap = need;
    }
    const Runs<KeyT> R{rows, stride, k, d->set_h, (const KeyT*)d->set_k, d->m};
    RSV_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)d->mstart, 0xFFFFFFFFu, (size_t)need, st));
    const int64_t longest = std::max<int64_t>(d->m, k) + 1;
    const dim3 bgrid((unsigned)std::min<int64_t>((longest + kBlock - 1) / kBlock, 1024), (unsigned)(parts + 1));
    hipLaunchKernelGGL(rows_bounds<KeyT>, bgrid, dim3(kBlock), 0, st, R, parts, d->m ? d->set_top : INT64_MIN,
                       (int32_t)(d->m == k && d->over), (uint32_t)lb, d->sctl, d->log_bmax_s, d->mstart);
    hipLaunchKernelGGL(rows_fill, dim3((unsigned)(parts + 1)), dim3(1024), 0, st, (uint32_t)lb, d->mstart);
    KeyT* bk = (KeyT*)d->sbk;
    hipLaunchKernelGGL(rows_sort<KeyT>, dim3((B + kBlock / 64 - 1) / (kBlock / 64)), dim3(kBlock), 0, st, R, parts,
                       (uint32_t)lb, (const uint32_t*)d->mstart, d->sctl, d->log_bmax_s, d->sbh, bk);
    hipLaunchKernelGGL(bucket_emit<KeyT>, dim3((B + kEmitBuckets - 1) / kEmitBuckets), dim3(kBlock), 0, st, d->m,
                       INT64_MAX, d->sctl, d->log_bmax_s, (const int64_t*)d->sbh, (const KeyT*)bk, k, d->set_h,
                       (KeyT*)d->set_k, lb);
    const uint32_t gen = ++d->sgen;
    hipLaunchKernelGGL(merge_publish, dim3(1), dim3(64), 0, st, d->sctl, d->shc_dev, (uint32_t*)(d->shc_dev + 12), gen);
    RSV_HIP_TRY(hipGetLastError());
    // the rows as merged, in engine memory: a degenerate hash that overflows a bucket is redone from
    // them at the settle, while the caller may already be reusing its gather buffer (stream-ordered
    // behind the merge kernels: parts x (2k + 6) words, ~8 MB at 8 x 65536)
    const int64_t rw = 2 * k + kRowMeta;
    if ((int64_t)parts * rw > d->rows_copy_cap) {
        RSV_HIP_TRY(grow((void**)&d->rows_copy, 0, (size_t)parts * rw * 8, false, st));
        d->rows_copy_cap = (int64_t)parts * rw;
    }
    RSV_HIP_TRY(hipMemcpy2DAsync(d->rows_copy, (size_t)rw * 8, rows, (size_t)stride * 8, (size_t)rw * 8, (size_t)parts,
                                 hipMemcpyDeviceToDevice, st));
    d->pend = true;
    d->pend_gen = gen;
    d->pend_lb = (uint32_t)lb;
    d->pend_rows = d->rows_copy;
    d->pend_parts = parts;
    d->pend_stride = rw;
    merged_bookkeeping(d);
    return RSV_OK;
}

int distinct_merge_rows(DistinctState* d, const int64_t* rows, int32_t parts, int64_t stride, hipStream_t st) {
    if (d->wide) return parts > 0 ? wide_merge_rows(d->wide, rows, parts, stride, st) : RSV_OK;
    if (int rc = distinct_settle(d, st)) return rc;
    if (parts <= 0) return RSV_OK;
    if (int rc = distinct_finalize(d, st)) return rc;  // an ordered set must be exact before it merges
    return d->kw == 8 ? merge_rows_impl<int64_t>(d, rows, parts, stride, st)
                      : merge_rows_impl<int32_t>(d, rows, parts, stride, st);
}

void distinct_retain_log(DistinctState* d, bool on) {
    if (d->wide) return wide_retain_log(d->wide, on);
    if (on && !d->retain && d->seen > 0) d->arch_ok = false;  // earlier candidates are gone
    d->retain = on;
    if (!on) archive_drop(d);
}

template <typename KeyT>
static int log_export_impl(DistinctState* d, int64_t bound, int64_t* out_h, KeyT* out_k, int64_t cap, int64_t* out_n,
                           hipStream_t st) {
    const bool all = bound == INT64_MAX;
    int64_t cnt = 0;
    auto emit = [&](int64_t h, int64_t key) {
        if (all || h < bound) {
            if (cnt < cap) {
                out_h[cnt] = h;
                out_k[cnt] = (KeyT)key;
            }
            ++cnt;
        }
    };
    for (size_t i = 0; i < d->arch_h.size(); ++i)
        emit(d->arch_h[i], sizeof(KeyT) == 8 ? d->arch_k[i] : (int64_t)d->arch_k4[i]);
    for (const std::vector<DistinctState::Seg>* v : {&d->pre_segs, &d->segs})
        for (const DistinctState::Seg& g : *v) {
            if (g.c == 0) continue;
            if (hipError_t e = segment_to_host<KeyT>(d, g, st, false)) {
                set_error(std::string("rsv_export_log: ") + hipGetErrorString(e));
                return e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;
            }
            const KeyT* pk = (const KeyT*)d->pk;
            for (int64_t t = 0; t < g.c; ++t) emit(d->ph[t], (int64_t)pk[t]);
        }
    *out_n = cnt;
    if (cnt > cap && cap > 0) {  // (cap 0: a count-only query)
        set_error("rsv_export_log: cap is smaller than the number of candidates (*out_n)");
        return RSV_E_ILLEGAL_ARGUMENT;
    }
    return RSV_OK;
}

int distinct_log_export(DistinctState* d, int64_t bound, int64_t* out_h, void* out_k, int64_t cap, int64_t* out_n,
                        hipStream_t st) {
    if (d->wide) return wide_log_export(d->wide, bound, out_h, out_k, cap, out_n, st);
    if (int rc = distinct_settle(d, st)) return rc;
    if (!d->ordered || !d->retain || !d->arch_ok) {
        set_error(!d->ordered  ? "rsv_export_log needs an RSV_DISTINCT_ORDERED sampler"
                  : !d->retain ? "rsv_export_log: the candidate log was not retained (rsv_retain_log before sampling)"
                               : "rsv_export_log: the candidate log was not retained (archive limit, or sampled "
                                 "after a merge)");
        return RSV_E_UNSUPPORTED;
    }
    return d->kw == 8 ? log_export_impl<int64_t>(d, bound, out_h, (int64_t*)out_k, cap, out_n, st)
                      : log_export_impl<int32_t>(d, bound, out_h, (int32_t*)out_k, cap, out_n, st);
}

// The exact multi-rank merge: a fresh replica runs RandomValues.sample over the concatenated
// candidate run (every rank's rsv_export_log output, in rank = global arrival order) and becomes
// the sampler's state, as if it had seen the whole stream.
int distinct_log_merge(DistinctState* d, const int64_t* h, const void* keys, int64_t n, int64_t seen,
                       hipStream_t st) {
    if (d->wide) return wide_log_merge(d->wide, h, keys, n, seen, st);
    if (!d->ordered) {
        set_error("rsv_merge_log needs an RSV_DISTINCT_ORDERED sampler");
        return RSV_E_UNSUPPORTED;
    }
    if (int rc = distinct_settle(d, st)) return rc;
    d->rep.reset(d->k);
    d->rep_stale = false;
    if (d->kw == 8) {
        const int64_t* kk = (const int64_t*)keys;
        d->rep.sample_run(n, [&](int64_t t) { return kk[t]; }, [&](int64_t t) { return h[t]; });
    } else {
        const int32_t* kk = (const int32_t*)keys;
        d->rep.sample_run(n, [&](int64_t t) { return (int64_t)kk[t]; }, [&](int64_t t) { return h[t]; });
    }
    d->segs.clear();
    d->pre_segs.clear();
    d->log_n = 0;
    archive_drop(d);
    hipError_t e = d->kw == 8 ? upload_replica<int64_t>(d, st) : upload_replica<int32_t>(d, st);
    if (e != hipSuccess) {
        set_error(std::string("rsv_merge_log: ") + hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;
    }
    d->over = false;
    d->exact = true;
    d->merged = true;
    d->spec_ok = false;
    d->seen = std::max(d->seen, seen);
    return RSV_OK;
}

}  // namespace rsv
