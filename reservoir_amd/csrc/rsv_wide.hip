// rsv_wide.hip -- Sampler.distinct over fixed-width byte keys (RandomValues, Sampler.scala:383-412,
// for a B of key_width = 16..256 bytes with value equality: java.util.UUID, a case class of
// primitives).  The hash is the caller's `hash: B => Long` (RSV_HASH_PRECOMPUTED, int64 per element
// beside the keys) or, for 16-byte keys, java.util.UUID.hashCode of the row (RSV_HASH_DEFAULT).
//
// The reference keeps the k distinct elements with the smallest scrambled hash
// h = byteswap64(r1 ^ byteswap64(r0 ^ hash(e))) (Sampler.scala:396-407); `elements.contains` is
// B.equals, i.e. equality of the key bytes.  Layout and passes (DESIGN.md §5 "wide distinct"):
//   filter   one streaming pass per chunk over the HASHES (8 B per element; the key rows are not
//            read): h <= bound (the set's maximum once full, inclusive) -> (h, batch offset)
//            staged per wave in LDS, appended B at a time
//   gather   the candidates' rows (key_width bytes each) -- the only key bytes that move
//   merge    set + candidates -> radix sort by h -> runs of equal h ordered by the key words
//            (one thread per run; a run longer than 64 entries takes a comparison merge sort of the
//            whole merge instead) -> drop equal (h, key) -> the first k are the new set, ascending by
//            (h, key words as unsigned 64-bit, word 0 first)
// The chunks grow geometrically (each ~4 seen lengths long, so ~4k candidates a chunk), so a 5e8-key
// batch takes ~6 chunks.  Ordered mode (the reference's sequential semantics for any hash) logs every
// candidate (h, global index, row) on the device; when the set's boundary hash bucket holds more
// distinct elements than the set keeps, the log is replayed in arrival order through the host replica
// HostValuesWide (scala PriorityQueue tie order) -- the same scheme as rsv_distinct.hip's ordered mode.
#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/reservoir_hip.h"
#include "rsv_device.h"
#include "rsv_host_values.h"
#include "rsv_internal.h"

namespace rsv {

namespace {

constexpr int kWBlock = 256;
constexpr int kRunMax = 64;         // longest run of equal h ordered by one thread
constexpr int kWideU = 8;           // 16-B loads in flight per lane in the filter
constexpr int64_t kWideGrid = 256 * 32;
typedef long long w2i64 __attribute__((ext_vector_type(2)));

inline unsigned wgrid(int64_t n, int64_t cap = 65535) {
    return (unsigned)std::min<int64_t>(std::max<int64_t>((n + kWBlock - 1) / kWBlock, 1), cap);
}

// The ordered mode's scheduled pass (see wide_sample_device): ranges [s_r, s_r+1) of the rest with
// falling bounds B_r; device table = starts [R + 1] then bounds [R].
constexpr int kWMaxR = 64;

// the proof needs >= k distinct hashes under each predicted bound, ~Poisson(beta k) of them: below
// k = 64 it fails too often to pay (k = 1: ~1 in 4 passes proves), so small k keep the chunk loop
constexpr int32_t kSchedMinK = 64;
constexpr int kSchedCounts = 192;                       // counts' offset in the table buffer
constexpr int kSchedWords = kSchedCounts + kWMaxR + 1;  // table [2 kWMaxR + 1] + counts [kWMaxR + 1]
static_assert(2 * kWMaxR + 1 <= kSchedCounts, "range table overlaps the counts");

// the filter's per-element bound: the iteration covers ranges [rl, rh] (wave-uniform), element i
// takes the bound of the range that holds it
struct WRanges {
    int64_t* rs;  // LDS starts [R + 1]
    int64_t* rb;  // LDS bounds [R]
    int32_t R;
    __device__ __forceinline__ void load(const int64_t* __restrict__ tab) {
        for (int t = threadIdx.x; t <= R; t += blockDim.x) rs[t] = tab[t];
        for (int t = threadIdx.x; t < R; t += blockDim.x) rb[t] = tab[R + 1 + t];
        __syncthreads();
    }
    // advance rl to the range holding lo, and rh to the one holding hi - 1 (uniform arguments)
    __device__ __forceinline__ void span(int64_t lo, int64_t hi, int32_t& rl, int32_t& rh) const {
        while (rl + 1 < R && rs[rl + 1] <= lo) ++rl;
        rh = rl;
        while (rh + 1 < R && rs[rh + 1] < hi) ++rh;
    }
    __device__ __forceinline__ int64_t at(int64_t i, int32_t rl, int32_t rh) const {
        int64_t b = rb[rl];
        for (int32_t r = rl + 1; r <= rh; ++r) b = i >= rs[r] ? rb[r] : b;
        return b;
    }
};

__device__ __forceinline__ unsigned long long lanemask_lt_w() {
    const uint32_t lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

template <int SRC>
__device__ __forceinline__ int64_t wide_hash(const int64_t* hashes, const uint64_t* rows, int64_t i) {
    if constexpr (SRC == kWideSrcHashes) return hashes[i];
    else return uuid_hash_code(rows[2 * i], rows[2 * i + 1]);
}

// Candidate output of the filter: each wave stages (h, offset) in LDS and appends B at a time under
// one reservation atomic (the counter is a single contended word); the workgroup's leftovers go out
// under one atomic at the end.
struct WideOut {
    static constexpr uint32_t B = 128;
    static constexpr uint32_t Q = B + 64;
    int64_t* qh;
    int64_t* qi;
    uint32_t qn;
    int64_t* cand_h;
    int64_t* cand_i;
    unsigned long long* counter;
    int64_t cap;

    __device__ __forceinline__ void write_at(unsigned long long base, uint32_t from, uint32_t cnt) {
        const uint32_t lane = threadIdx.x & 63;
        for (uint32_t j = lane; j < cnt; j += 64) {
            const unsigned long long pos = base + j;
            if ((int64_t)pos < cap) {
                cand_h[pos] = qh[from + j];
                cand_i[pos] = qi[from + j];
            }
        }
    }
    __device__ __forceinline__ void push(bool c, int64_t h, int64_t idx) {
        const unsigned long long bal = __ballot(c);
        if (bal == 0) return;
        if (c) {
            const uint32_t pos = qn + __popcll(bal & lanemask_lt_w());
            qh[pos] = h;
            qi[pos] = idx;
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= B) {
            qn -= B;
            __builtin_amdgcn_wave_barrier();
            unsigned long long base = 0;
            if ((threadIdx.x & 63) == 0) base = atomicAdd(counter, (unsigned long long)B);
            base = __shfl(base, 0);
            write_at(base, qn, B);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __device__ __forceinline__ void flush_block(uint32_t* s_q, unsigned long long* s_base) {
        const uint32_t w = threadIdx.x >> 6;
        __builtin_amdgcn_wave_barrier();
        if ((threadIdx.x & 63) == 0) s_q[w] = qn;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (int i = 0; i < kWBlock / 64; ++i) tot += s_q[i];
            *s_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t i = 0; i < w; ++i) pre += s_q[i];
        if (qn) write_at(*s_base + pre, 0, qn);
        qn = 0;
    }
};

// The filter over precomputed hashes: 16-B non-temporal loads (two hashes each), kWideU in flight per
// lane; the <= 1 head element before the first 16-B boundary and the odd tail go through the scalar
// loops.  Loop bounds are wave-uniform (tile starts), so the ballots see every lane.
// With R > 0 ranges (rtab), element i's bound is its range's (the ordered mode's scheduled pass).
__global__ __launch_bounds__(kWBlock) void wide_filter_hashes(const int64_t* __restrict__ hashes, int64_t n, int64_t r0,
                                                              int64_t r1, int64_t bound, int64_t* __restrict__ cand_h,
                                                              int64_t* __restrict__ cand_i,
                                                              unsigned long long* __restrict__ counter, int64_t cap,
                                                              const int64_t* __restrict__ rtab, int32_t R) {
    __shared__ int64_t sh_h[kWBlock / 64][WideOut::Q];
    __shared__ int64_t sh_i[kWBlock / 64][WideOut::Q];
    __shared__ uint32_t s_q[kWBlock / 64];
    __shared__ unsigned long long s_base;
    __shared__ int64_t s_rs[kWMaxR + 1], s_rb[kWMaxR];
    WideOut out{sh_h[threadIdx.x >> 6], sh_i[threadIdx.x >> 6], 0u, cand_h, cand_i, counter, cap};
    WRanges rg{s_rs, s_rb, R};
    if (R) rg.load(rtab);
    int32_t rl = 0, rh = 0;
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t head = std::min<int64_t>(n, (int64_t)(((16u - ((uintptr_t)hashes & 15u)) & 15u) / 8u));
    const w2i64* hv = reinterpret_cast<const w2i64*>(hashes + head);
    const int64_t n_vec = (n - head) / 2;
    for (int64_t t0 = 0; t0 < n_vec; t0 += T * kWideU) {
        w2i64 x[kWideU];
#pragma unroll
        for (int u = 0; u < kWideU; ++u) {
            const int64_t v = t0 + u * T + tid;
            x[u] = __builtin_nontemporal_load(hv + (v < n_vec ? v : n_vec - 1));
        }
        if (R) rg.span(head + 2 * t0, head + 2 * (t0 + T * kWideU), rl, rh);
        int64_t h[kWideU][2];
        bool c[kWideU][2];
        bool any = false;
#pragma unroll
        for (int u = 0; u < kWideU; ++u) {
            const bool ok = t0 + u * T + tid < n_vec;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int64_t i = head + (t0 + u * T + tid) * 2 + e;
                h[u][e] = scramble(r0, r1, x[u][e]);
                c[u][e] = ok && h[u][e] <= (R ? rg.at(i, rl, rh) : bound);
                any |= c[u][e];
            }
        }
        if (__any(any)) {
#pragma unroll
            for (int u = 0; u < kWideU; ++u)
#pragma unroll
                for (int e = 0; e < 2; ++e) out.push(c[u][e], h[u][e], head + (t0 + u * T + tid) * 2 + e);
        }
    }
    for (int64_t i0 = 0; i0 < head; i0 += T) {
        const int64_t i = i0 + tid;
        const int64_t hh = i < head ? scramble(r0, r1, hashes[i]) : 0;
        out.push(i < head && hh <= (R ? rg.at(i, 0, R - 1) : bound), hh, i);
    }
    for (int64_t i0 = head + 2 * n_vec; i0 < n; i0 += T) {
        const int64_t i = i0 + tid;
        const int64_t hh = i < n ? scramble(r0, r1, hashes[i]) : 0;
        out.push(i < n && hh <= (R ? rg.at(i, 0, R - 1) : bound), hh, i);
    }
    out.flush_block(s_q, &s_base);
}

// The filter over 16-byte UUID rows (the hash is UUID.hashCode of the row): two 8-B non-temporal
// loads per row (rows need only 8-B alignment), kWideU rows in flight per lane.
__global__ __launch_bounds__(kWBlock) void wide_filter_uuid(const uint64_t* __restrict__ rows, int64_t n, int64_t r0,
                                                            int64_t r1, int64_t bound, int64_t* __restrict__ cand_h,
                                                            int64_t* __restrict__ cand_i,
                                                            unsigned long long* __restrict__ counter, int64_t cap,
                                                            const int64_t* __restrict__ rtab, int32_t R) {
    __shared__ int64_t sh_h[kWBlock / 64][WideOut::Q];
    __shared__ int64_t sh_i[kWBlock / 64][WideOut::Q];
    __shared__ uint32_t s_q[kWBlock / 64];
    __shared__ unsigned long long s_base;
    __shared__ int64_t s_rs[kWMaxR + 1], s_rb[kWMaxR];
    WideOut out{sh_h[threadIdx.x >> 6], sh_i[threadIdx.x >> 6], 0u, cand_h, cand_i, counter, cap};
    WRanges rg{s_rs, s_rb, R};
    if (R) rg.load(rtab);
    int32_t rl = 0, rh = 0;
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t t0 = 0; t0 < n; t0 += T * kWideU) {
        uint64_t a[kWideU], b[kWideU];
#pragma unroll
        for (int u = 0; u < kWideU; ++u) {
            const int64_t i = std::min<int64_t>(t0 + u * T + tid, n - 1);
            a[u] = __builtin_nontemporal_load(rows + 2 * i);
            b[u] = __builtin_nontemporal_load(rows + 2 * i + 1);
        }
        if (R) rg.span(t0, t0 + T * kWideU, rl, rh);
        int64_t h[kWideU];
        bool c[kWideU];
        bool any = false;
#pragma unroll
        for (int u = 0; u < kWideU; ++u) {
            const int64_t i = t0 + u * T + tid;
            h[u] = scramble(r0, r1, uuid_hash_code(a[u], b[u]));
            c[u] = i < n && h[u] <= (R ? rg.at(i, rl, rh) : bound);
            any |= c[u];
        }
        if (__any(any)) {
#pragma unroll
            for (int u = 0; u < kWideU; ++u) out.push(c[u], h[u], t0 + u * T + tid);
        }
    }
    out.flush_block(s_q, &s_base);
}

// No bound (the set still filling): every element is a candidate, element i goes to place i
template <int SRC>
__global__ __launch_bounds__(kWBlock) void wide_hash_all(const int64_t* __restrict__ hashes,
                                                         const uint64_t* __restrict__ rows, int64_t n, int64_t r0,
                                                         int64_t r1, int64_t* __restrict__ out_h,
                                                         int64_t* __restrict__ out_i) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        out_h[i] = scramble(r0, r1, wide_hash<SRC>(hashes, rows, i));
        out_i[i] = i;
    }
}

// candidate rows: out[j] = keys[idx[j]] (one thread per 8-B word: a row's words are adjacent lanes)
__global__ __launch_bounds__(kWBlock) void wide_gather_rows(const uint64_t* __restrict__ keys,
                                                            const int64_t* __restrict__ idx, int64_t c, int32_t words,
                                                            uint64_t* __restrict__ out,
                                                            const int64_t* __restrict__ cdev = nullptr) {
    if (cdev) {  // the count on the device (the filter's counter; above the room c: nothing to gather)
        const int64_t cd = *cdev;
        c = cd <= c ? cd : 0;
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t total = c * words;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const int64_t j = t / words;
        out[t] = keys[idx[j] * words + (t - j * words)];
    }
}

// ordered mode: the chunk's candidates onto the log as (h, global index, row)
__global__ __launch_bounds__(kWBlock) void wide_log_append(const int64_t* __restrict__ ch, const int64_t* __restrict__ ci,
                                                           const uint64_t* __restrict__ ck, int64_t c, int32_t words,
                                                           int64_t base, int64_t* __restrict__ lh,
                                                           int64_t* __restrict__ lg, uint64_t* __restrict__ lk) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < c * words; t += stride) {
        lk[t] = ck[t];
        if (t < c) {
            lh[t] = ch[t];
            lg[t] = base + ci[t];
        }
    }
}

// entries of a merge: [0, m) the set, [m, N) the candidates
struct WRows {
    const uint64_t* set_k;
    const uint64_t* cand_k;
    int64_t m;
    int32_t words;
    __host__ __device__ const uint64_t* operator()(uint32_t e) const {
        return (int64_t)e < m ? set_k + (size_t)e * words : cand_k + ((size_t)e - (size_t)m) * words;
    }
};

__host__ __device__ inline int row_cmp(const uint64_t* a, const uint64_t* b, int32_t words) {
    for (int32_t w = 0; w < words; ++w)
        if (a[w] != b[w]) return a[w] < b[w] ? -1 : 1;
    return 0;
}

// the comparison sort of the fallback: (h, key words)
struct WLess {
    const int64_t* h;
    WRows R;
    __host__ __device__ bool operator()(uint32_t a, uint32_t b) const {
        if (h[a] != h[b]) return h[a] < h[b];
        return row_cmp(R(a), R(b), R.words) < 0;
    }
};

__global__ __launch_bounds__(kWBlock) void wide_merge_init(const int64_t* __restrict__ set_h,
                                                           const int64_t* __restrict__ cand_h, int64_t m, int64_t N,
                                                           int64_t* __restrict__ eh, uint32_t* __restrict__ ev) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += stride) {
        eh[e] = e < m ? set_h[e] : cand_h[e - m];
        ev[e] = (uint32_t)e;
    }
}

// after the radix sort by h: each run of equal h (almost always one entry; a run is one key's
// duplicates, or distinct keys whose hashes collide) is ordered by its key words, in place, by the
// thread at its start.  A run longer than kRunMax sets ctl[1]: the merge redoes its order with the
// comparison sort.
__global__ __launch_bounds__(kWBlock) void wide_run_fix(const int64_t* __restrict__ eh, uint32_t* __restrict__ ev,
                                                        int64_t N, WRows R, int64_t* __restrict__ ctl) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
        const int64_t h = eh[p];
        if (p > 0 && eh[p - 1] == h) continue;  // not a run start
        if (p + 1 >= N || eh[p + 1] != h) continue;
        int64_t L = 2;
        while (p + L < N && eh[p + L] == h && L <= kRunMax) ++L;
        if (L > kRunMax) {
            atomicOr((unsigned long long*)(ctl + 1), 1ull);
            continue;
        }
        for (int64_t i = 1; i < L; ++i) {
            const uint32_t x = ev[p + i];
            int64_t j = i;
            while (j > 0 && row_cmp(R(ev[p + j - 1]), R(x), R.words) > 0) {
                ev[p + j] = ev[p + j - 1];
                --j;
            }
            ev[p + j] = x;
        }
    }
}

__global__ __launch_bounds__(kWBlock) void wide_gather_h(const int64_t* __restrict__ eh_by_entry,
                                                         const uint32_t* __restrict__ ev, int64_t N,
                                                         int64_t* __restrict__ eh) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) eh[p] = eh_by_entry[ev[p]];
}

// flag = first of each run of identical (h, key)
__global__ __launch_bounds__(kWBlock) void wide_flags(const int64_t* __restrict__ eh, const uint32_t* __restrict__ ev,
                                                      int64_t N, WRows R, uint32_t* __restrict__ flags) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride)
        flags[p] = (p == 0 || eh[p] != eh[p - 1] || row_cmp(R(ev[p]), R(ev[p - 1]), R.words) != 0) ? 1u : 0u;
}

// the first k distinct entries -> the new set; ctl[2] = distinct count, ctl[3] = the largest kept h,
// ctl[4] = rank k ties rank k - 1 on h (the boundary bucket holds more distinct elements than kept)
__global__ __launch_bounds__(kWBlock) void wide_emit(const int64_t* __restrict__ eh, const uint32_t* __restrict__ ev,
                                                     const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos,
                                                     int64_t N, int64_t k, WRows R, int64_t* __restrict__ out_h,
                                                     uint64_t* __restrict__ out_k, int64_t* __restrict__ ctl) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
        const int64_t r = pos[p];
        if (flags[p]) {
            if (r < k) {
                out_h[r] = eh[p];
                const uint64_t* src = R(ev[p]);
                for (int32_t w = 0; w < R.words; ++w) out_k[r * R.words + w] = src[w];
                if (r == k - 1) ctl[3] = eh[p];
            } else if (r == k && eh[p - 1] == eh[p]) {
                ctl[4] = 1;
            }
        }
        if (p == N - 1) {
            const int64_t nd = r + (int64_t)flags[p];
            ctl[2] = nd;
            if (nd <= k) ctl[3] = eh[p];
        }
    }
}

// The scheduled pass's proof (ordered mode): range r's bound B_r covered every element the
// reference could admit in range r iff at least k distinct elements with h < B_r arrived before s_r
// (the set's members count as arrived): the heap's maximum at s_r is then below B_r.  Over the merge
// (set + the pass's candidates, in (h, key) order, `flags` = first of each run of one element), each
// distinct element with first arrival a and hash h counts for the ranges r with range(a) < r and
// B_r > h -- one difference-array interval per element, summed per workgroup in LDS.
__global__ __launch_bounds__(kWBlock) void wide_verify(const int64_t* __restrict__ eh, const uint32_t* __restrict__ ev,
                                                       const uint32_t* __restrict__ flags, int64_t N, int64_t m_old,
                                                       const int64_t* __restrict__ cand_i,
                                                       const int64_t* __restrict__ rtab, int32_t R,
                                                       unsigned long long* __restrict__ diff) {
    __shared__ int64_t s_rs[kWMaxR + 1], s_rb[kWMaxR];
    __shared__ int s_d[kWMaxR + 1];
    WRanges rg{s_rs, s_rb, R};
    for (int t = threadIdx.x; t <= R; t += blockDim.x) s_d[t] = 0;
    rg.load(rtab);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
        if (!flags[p]) continue;
        int64_t a = INT64_MAX;  // the element's first arrival (-1: a set member)
        for (int64_t q = p; q < N && (q == p || !flags[q]); ++q) {
            const uint32_t e = ev[q];
            a = std::min<int64_t>(a, (int64_t)e < m_old ? -1 : cand_i[(int64_t)e - m_old]);
        }
        const int64_t h = eh[p];
        int32_t ra = -1;  // the range holding a
        while (ra + 1 < R && s_rs[ra + 1] <= a) ++ra;
        int32_t rh = -1;  // the last range whose bound exceeds h (bounds fall with r)
        while (rh + 1 < R && s_rb[rh + 1] > h) ++rh;
        if (ra + 1 <= rh) {
            atomicAdd(&s_d[ra + 1], 1);
            atomicAdd(&s_d[rh + 1], -1);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t <= R; t += blockDim.x)
        if (s_d[t]) atomicAdd(&diff[t], (unsigned long long)(int64_t)s_d[t]);
}

__global__ __launch_bounds__(kWBlock) void wide_iota(uint32_t* __restrict__ v, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) v[i] = (uint32_t)i;
}

// the log in arrival order: out[j] = log[perm[j]]
__global__ __launch_bounds__(kWBlock) void wide_log_permute(const uint32_t* __restrict__ perm,
                                                            const int64_t* __restrict__ lh,
                                                            const uint64_t* __restrict__ lk, int64_t n, int32_t words,
                                                            int64_t* __restrict__ oh, uint64_t* __restrict__ ok) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * words; t += stride) {
        const int64_t j = t / words;
        const int64_t src = perm[j];
        ok[t] = lk[src * words + (t - j * words)];
        if (t < n) oh[t] = lh[perm[t]];
    }
}

// first-occurrence flags of the log for the host replay: the entries [members | the log in arrival
// order] sorted stably by h and, within a run of equal h, stably by the key words, so each key's
// entries sit together in entry order; a log entry is flagged when it heads its key's group (no
// member and no earlier log entry carries the key).  flag[t] for log position t (arrival order).
__global__ __launch_bounds__(kWBlock) void wide_mark_first(const int64_t* __restrict__ eh, const uint32_t* __restrict__ ev,
                                                           int64_t N, WRows R, uint32_t* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += stride) {
        const uint32_t e = ev[p];
        if ((int64_t)e < R.m) continue;
        const bool head = p == 0 || eh[p] != eh[p - 1] || row_cmp(R(ev[p - 1]), R(e), R.words) != 0;
        flag[(int64_t)e - R.m] = head ? 1u : 0u;
    }
}

// packed row: [key words (k x words) | hashes (k) | n, count, tied, max_hash, log_retained, ordered]
__global__ __launch_bounds__(kWBlock) void wide_export_row(const int64_t* __restrict__ set_h,
                                                           const uint64_t* __restrict__ set_k, int64_t m, int64_t k,
                                                           int32_t words, int64_t* __restrict__ row, int64_t count,
                                                           int64_t tied, int64_t mx, int64_t retained,
                                                           int64_t ordered) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t kw = k * words;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < kw + k; t += stride) {
        if (t < kw) row[t] = t < m * words ? (int64_t)set_k[t] : 0;
        else row[t] = t - kw < m ? set_h[t - kw] : 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int64_t* meta = row + kw + k;
        meta[0] = m;
        meta[1] = count;
        meta[2] = tied;
        meta[3] = mx;
        meta[4] = retained;
        meta[5] = ordered;
    }
}

// ---- bucketed merge (round 6) --------------------------------------------------------------------
// set ∪ candidates -> buckets by h (a monotone map of [INT64_MIN, span_hi] onto B = 2^lb buckets,
// ~64 entries each: the scrambled hash is uniform) -> one wave per bucket sorts (h, entry) in
// registers (bitonic network over DPP lane exchanges), puts each run of equal h in key-word order in
// LDS (the lane at the run's start; runs are one key's repeats or colliding hashes), keeps the first
// of each distinct (h, key) with its element's first arrival -> each bucket's distinct entries land
// at their global rank (the first k are the new set).  Three dispatches instead of the radix sort's
// eight passes, the scan and the flag kernels.  A bucket above kWCap entries or a run above kRunMax
// (a degenerate hash) sets ctl[1]: the host then runs the sort-based merge instead.
//   bucket area: bh / be / ba [B x kWCap] (h, entry id, first arrival), cnt [B x kWStride] (one
//   128-B line per counter: neighbouring atomics would serialise on a shared line; wb_sort re-zeroes
//   what it consumed), bdist [B] distinct per bucket, gsum [B / 16 + 1] their group sums.
constexpr uint32_t kWCap = 256;
constexpr uint32_t kWAvgLog = 6;
constexpr uint32_t kWStride = 32;
constexpr uint32_t kWEmitBuckets = 16;

// The bucket map: a piecewise-linear, monotone map of h onto B buckets.  Segment s covers h in
// [lo_s, lo_(s+1)) (lo_0 = INT64_MIN) and owns buckets [b0_s, b0_s + nb_s), linearly:
// floor((h - lo_s) nb_s / (span_s + 1)) = umulhi(h - lo_s, mult_s), mult_s = nb_s floor((2^64 - 1) /
// (span_s + 1)) (0: a span below nb_s buckets directly).  The host gives each segment buckets in
// proportion to the entries expected there, so a merge whose density varies along h (the scheduled
// pass: every range adds candidates below its own bound, the lowest band ~2^R / (1.6 R) times the
// mean) still fills ~64 entries a bucket.  Table (int64 words, device): lo [kWSegMax + 1] | b0
// [kWSegMax + 1] | mult [kWSegMax] | nb [kWSegMax].
constexpr int kWSegMax = 72;
constexpr int kWSegWords = 4 * kWSegMax + 2;

struct WSegMap {
    const int64_t* lo;
    const int64_t* b0;
    const int64_t* mult;
    const int64_t* nb;
    int32_t ns;
    __device__ __forceinline__ uint32_t operator()(int64_t h) const {
        int32_t a = 0, z = ns - 1;  // the last segment with lo <= h (lo[0] = INT64_MIN)
        while (a < z) {
            const int32_t mid = (a + z + 1) >> 1;
            if (lo[mid] <= h) a = mid;
            else z = mid - 1;
        }
        const uint64_t u = (uint64_t)h - (uint64_t)lo[a];
        const uint64_t mu = (uint64_t)mult[a], n = (uint64_t)nb[a];
        uint64_t b = mu ? __umul64hi(u, mu) : u;
        b = b < n ? b : n - 1;
        return (uint32_t)((uint64_t)b0[a] + b);
    }
};

// the segment table as a kernel argument (2.3 KB of kernarg: no copy of its own on the stream)
struct WSegTable {
    int64_t w[kWSegWords];
};

// the merge's control words ctl[1..6] zeroed, and (first use of a bucket area) its counters: one
// dispatch in place of the small memsets (a misaligned hipMemsetAsync is up to three fill kernels)
__global__ __launch_bounds__(kWBlock) void wb_prep(int64_t* __restrict__ ctl, uint32_t* __restrict__ cnt,
                                                   uint32_t n_cnt) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 6) ctl[1 + t] = 0;
    for (uint32_t i = t; i < n_cnt; i += gridDim.x * blockDim.x) cnt[i] = 0;
}

__global__ __launch_bounds__(kWBlock) void wb_scatter(const int64_t* __restrict__ set_h, int64_t m,
                                                      const int64_t* __restrict__ cand_h, int64_t c,
                                                      const WSegTable seg, int32_t ns, uint32_t B,
                                                      int64_t* __restrict__ bh, uint32_t* __restrict__ be,
                                                      uint32_t* __restrict__ cnt, uint32_t* __restrict__ gsum,
                                                      int64_t* __restrict__ ctl, bool c_on_device) {
    __shared__ int64_t s_seg[kWSegWords];
    for (int i = threadIdx.x; i < kWSegWords; i += blockDim.x) s_seg[i] = seg.w[i];
    if (blockIdx.x == 0)
        for (uint32_t i = threadIdx.x; i <= (B >> 4); i += blockDim.x) gsum[i] = 0;
    __syncthreads();
    if (c_on_device) {  // c = the filter's counter ctl[0]; above the room c the filter dropped some:
        const int64_t cd = ctl[0];  // nothing is merged (the host reruns the chunk with room)
        if (cd > c) {
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl[1] = 1;
            return;
        }
        c = cd;
    }
    const WSegMap map{s_seg, s_seg + kWSegMax + 1, s_seg + 2 * kWSegMax + 2, s_seg + 3 * kWSegMax + 2, ns};
    const int64_t total = m + c, stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
        const int64_t h = e < m ? set_h[e] : cand_h[e - m];
        const uint32_t b = map(h);
        const uint32_t p = atomicAdd(&cnt[(size_t)b * kWStride], 1u);
        if (p < kWCap) {
            bh[(size_t)b * kWCap + p] = h;
            be[(size_t)b * kWCap + p] = (uint32_t)e;
        } else {
            ctl[1] = 1;
        }
    }
}

// (u, e) ascending, u = h - INT64_MIN (unsigned order = signed order of h), e the entry id
__device__ __forceinline__ bool ue_less(uint64_t ua, uint32_t ea, uint64_t ub, uint32_t eb) {
    return ua < ub || (ua == ub && ea < eb);
}

// bitonic network over 64 R entries, entry i = r * 64 + lane in register slot r
template <int R>
__device__ __forceinline__ void wb_bitonic(uint64_t (&u)[R], uint32_t (&e)[R]) {
    const uint32_t lane = threadIdx.x & 63;
    constexpr uint32_t N = 64u * R;
#pragma unroll
    for (uint32_t size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {
                const uint32_t rs = stride / 64;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if ((r & rs) == 0) {
                        const int r2 = r + rs;
                        const bool up = ((r * 64u + lane) & size) == 0;
                        if (ue_less(u[r2], e[r2], u[r], e[r]) == up) {
                            const uint64_t tu = u[r];
                            const uint32_t te = e[r];
                            u[r] = u[r2];
                            e[r] = e[r2];
                            u[r2] = tu;
                            e[r2] = te;
                        }
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint64_t ou = xor_any(u[r], (int)stride);
                    const uint32_t oe = xor_any(e[r], (int)stride);
                    const bool lower = (lane & stride) == 0;
                    const bool up = ((r * 64u + lane) & size) == 0;
                    const bool take = (lower == up) ? ue_less(ou, oe, u[r], e[r]) : ue_less(u[r], e[r], ou, oe);
                    if (take) {
                        u[r] = ou;
                        e[r] = oe;
                    }
                }
            }
        }
    }
}

template <int R>
__device__ __forceinline__ void wb_sort_regs(const int64_t* gh, const uint32_t* ge, uint32_t n, uint64_t* su,
                                             uint32_t* se) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t u[R];
    uint32_t e[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * 64u + lane;
        u[r] = i < n ? ((uint64_t)gh[i] ^ 0x8000000000000000ull) : ~0ull;
        e[r] = i < n ? ge[i] : ~0u;
    }
    wb_bitonic<R>(u, e);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = r * 64u + lane;
        if (i < n) {
            su[i] = u[r];
            se[i] = e[r];
        }
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// One wave per bucket: sort, order runs of equal h by the key words, keep the first entry of each
// distinct (h, key) compacted at the bucket's start (with the element's first arrival when cand_i is
// given: -1 for a set member, else the earliest batch offset among its candidate entries).
__global__ __launch_bounds__(kWBlock) void wb_sort(int64_t m, uint32_t B, int64_t* __restrict__ bh,
                                                   uint32_t* __restrict__ be, int64_t* __restrict__ ba,
                                                   uint32_t* __restrict__ cnt, uint32_t* __restrict__ bdist,
                                                   uint32_t* __restrict__ gsum, WRows R,
                                                   const int64_t* __restrict__ cand_i, int64_t* __restrict__ ctl) {
    __shared__ uint64_t s_u[kWBlock / 64][kWCap];
    __shared__ uint32_t s_e[kWBlock / 64][kWCap];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x * (kWBlock / 64) + w;
    if (b >= B) return;
    uint32_t* pc = cnt + (size_t)b * kWStride;
    const uint32_t n = *pc;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) *pc = 0;  // consumed: zero for the next merge
    if (n == 0 || n > kWCap) {  // (an overfull bucket set ctl[1] in the scatter)
        if (lane == 0) bdist[b] = 0;
        return;
    }
    int64_t* gh = bh + (size_t)b * kWCap;
    uint32_t* ge = be + (size_t)b * kWCap;
    uint64_t* su = s_u[w];
    uint32_t* se = s_e[w];
    if (n <= 64) wb_sort_regs<1>(gh, ge, n, su, se);
    else if (n <= 128) wb_sort_regs<2>(gh, ge, n, su, se);
    else wb_sort_regs<4>(gh, ge, n, su, se);
    wave_lds_sync();
    // runs of equal h: the lane at the run's start orders it by the key words (insertion sort)
    for (uint32_t i = lane; i < n; i += 64) {
        if ((i > 0 && su[i - 1] == su[i]) || i + 1 >= n || su[i + 1] != su[i]) continue;
        uint32_t L = 2;
        while (i + L < n && su[i + L] == su[i] && L <= (uint32_t)kRunMax) ++L;
        if (L > (uint32_t)kRunMax) {
            ctl[1] = 1;
            continue;
        }
        for (uint32_t a = 1; a < L; ++a) {
            const uint32_t x = se[i + a];
            uint32_t j = a;
            while (j > 0 && row_cmp(R(se[i + j - 1]), R(x), R.words) > 0) {
                se[i + j] = se[i + j - 1];
                --j;
            }
            se[i + j] = x;
        }
    }
    wave_lds_sync();
    // the first of each distinct (h, key), compacted; its element's first arrival
    uint32_t base = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        bool first = false;
        if (i < n) first = i == 0 || su[i - 1] != su[i] || row_cmp(R(se[i - 1]), R(se[i]), R.words) != 0;
        const unsigned long long bal = __ballot(first);
        if (first) {
            const uint32_t o = base + (uint32_t)__popcll(bal & lanemask_lt_w());
            if (ba) {
                const uint32_t e0 = se[i];
                int64_t a = (int64_t)e0 < m ? -1 : cand_i[(int64_t)e0 - m];
                for (uint32_t j = i + 1; j < n && su[j] == su[i] && row_cmp(R(se[j]), R(e0), R.words) == 0; ++j) {
                    const int64_t aj = (int64_t)se[j] < m ? -1 : cand_i[(int64_t)se[j] - m];
                    a = aj < a ? aj : a;
                }
                ba[(size_t)b * kWCap + o] = a;
            }
            gh[o] = (int64_t)(su[i] ^ 0x8000000000000000ull);
            ge[o] = se[i];
        }
        base += (uint32_t)__popcll(bal);
    }
    if (lane == 0) {
        bdist[b] = base;
        atomicAdd(gsum + (b >> 4), base);
    }
}

// each bucket's distinct entries to their global rank (ranks < k): the set's hashes and key rows.
// ctl[2] = distinct count, ctl[3] = the largest kept h, ctl[4] = rank k ties rank k - 1 on h (equal h
// share a bucket: the map is monotone)
__global__ __launch_bounds__(kWBlock) void wb_emit(uint32_t B, const int64_t* __restrict__ bh,
                                                   const uint32_t* __restrict__ be, const uint32_t* __restrict__ bdist,
                                                   const uint32_t* __restrict__ gsum, int64_t k, WRows R,
                                                   int64_t* __restrict__ out_h, uint64_t* __restrict__ out_k,
                                                   int64_t* __restrict__ ctl) {
    __shared__ uint64_t s_pre[kWBlock / 64], s_tot[kWBlock / 64];
    __shared__ uint64_t s_base[kWEmitBuckets + 1];
    const uint32_t b0 = blockIdx.x * kWEmitBuckets;
    if (b0 >= B) return;
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t G = (B + 15) >> 4, g0 = b0 >> 4;
    uint64_t pre = 0, tot = 0;
    for (uint32_t i = t; i < G; i += kWBlock) {
        const uint64_t v = gsum[i];
        tot += v;
        if (i < g0) pre += v;
    }
    for (uint32_t i = (g0 << 4) + t; i < b0; i += kWBlock) pre += bdist[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        pre += (uint64_t)__shfl_xor((long long)pre, off);
        tot += (uint64_t)__shfl_xor((long long)tot, off);
    }
    if (lane == 0) {
        s_pre[w] = pre;
        s_tot[w] = tot;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t p = 0, q = 0;
        for (int i = 0; i < kWBlock / 64; ++i) {
            p += s_pre[i];
            q += s_tot[i];
        }
        const uint32_t nb = std::min<uint32_t>(kWEmitBuckets, B - b0);
        for (uint32_t i = 0; i < nb; ++i) {
            s_base[i] = p;
            p += bdist[b0 + i];
        }
        s_base[kWEmitBuckets] = q;
        if (b0 == 0) ctl[2] = (int64_t)q;
    }
    __syncthreads();
    tot = s_base[kWEmitBuckets];
    const uint64_t mk = std::min<uint64_t>(tot, (uint64_t)k);
    for (uint32_t j = 0; j < kWEmitBuckets / (kWBlock / 64); ++j) {
        const uint32_t bi = w * (kWEmitBuckets / (kWBlock / 64)) + j;
        const uint32_t b = b0 + bi;
        if (b >= B) break;
        const uint64_t base = s_base[bi];
        if (base > (uint64_t)k) break;  // later buckets rank higher still
        const uint32_t cnt = bdist[b];
        const int64_t* gh = bh + (size_t)b * kWCap;
        const uint32_t* ge = be + (size_t)b * kWCap;
        for (uint32_t r = lane; r < cnt; r += 64) {
            const uint64_t rank = base + r;
            if (rank < (uint64_t)k) {
                const int64_t h = gh[r];
                out_h[rank] = h;
                const uint64_t* src = R(ge[r]);
                for (int32_t q = 0; q < R.words; ++q) out_k[rank * R.words + q] = src[q];
                if (rank + 1 == mk) ctl[3] = h;
            } else if (rank == (uint64_t)k && r > 0 && gh[r - 1] == gh[r]) {
                ctl[4] = 1;
            }
        }
    }
}

// the scheduled pass's proof over the bucketed merge (wide_verify's rule: each distinct element with
// first arrival a and hash h counts for the ranges r with range(a) < r and B_r > h)
__global__ __launch_bounds__(kWBlock) void wb_verify(uint32_t B, const int64_t* __restrict__ bh,
                                                     const int64_t* __restrict__ ba, const uint32_t* __restrict__ bdist,
                                                     const int64_t* __restrict__ rtab, int32_t R,
                                                     unsigned long long* __restrict__ diff) {
    __shared__ int64_t s_rs[kWMaxR + 1], s_rb[kWMaxR];
    __shared__ int s_d[kWMaxR + 1];
    WRanges rg{s_rs, s_rb, R};
    for (int t = threadIdx.x; t <= R; t += blockDim.x) s_d[t] = 0;
    rg.load(rtab);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wstride = gridDim.x * (kWBlock / 64);
    for (uint32_t b = blockIdx.x * (kWBlock / 64) + (threadIdx.x >> 6); b < B; b += wstride) {
        const uint32_t cnt = bdist[b];
        for (uint32_t r = lane; r < cnt; r += 64) {
            const int64_t h = bh[(size_t)b * kWCap + r], a = ba[(size_t)b * kWCap + r];
            int32_t ra = -1;  // the range holding a
            while (ra + 1 < R && s_rs[ra + 1] <= a) ++ra;
            int32_t rh = -1;  // the last range whose bound exceeds h (bounds fall with r)
            while (rh + 1 < R && s_rb[rh + 1] > h) ++rh;
            if (ra + 1 <= rh) {
                atomicAdd(&s_d[ra + 1], 1);
                atomicAdd(&s_d[rh + 1], -1);
            }
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t <= R; t += blockDim.x)
        if (s_d[t]) atomicAdd(&diff[t], (unsigned long long)(int64_t)s_d[t]);
}

}  // namespace

struct WideDistinct {
    int32_t k = 0;
    int32_t words = 0;  // key_width / 8
    int src = kWideSrcHashes;
    int64_t r0 = 0, r1 = 0;
    bool ordered = false;
    int64_t m = 0;                // set size
    int64_t top = INT64_MIN;      // the set's largest h (valid when m > 0)
    bool tied = false;            // full, and the boundary hash bucket holds more distinct elements
    bool exact = true;            // ordered: the set arrays hold the reference's set
    int64_t seen = 0;             // elements sampled (chunk sizing)
    KernelTimer* timer = nullptr;
    // device
    int64_t* set_h = nullptr;     // [set_cap] ascending (h, key words)
    uint64_t* set_k = nullptr;
    int64_t* set_h2 = nullptr;    // the merge's output (swapped in)
    uint64_t* set_k2 = nullptr;
    int64_t set_cap = 0;
    int64_t* cand_h = nullptr;    // [cand_cap] candidates: h, batch offset, row
    int64_t* cand_i = nullptr;
    uint64_t* cand_k = nullptr;
    int64_t cand_cap = 0;
    int64_t *eh0 = nullptr, *eh1 = nullptr;  // [merge_cap] merge entries
    uint32_t *ev0 = nullptr, *ev1 = nullptr, *flags = nullptr, *pos = nullptr;
    int64_t merge_cap = 0;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    int64_t* ctl = nullptr;       // [8]: [0] candidate counter [1] long run [2] distinct [3] top [4] tie
    int64_t* hctl = nullptr;      // pinned copy
    // ordered mode: the candidate log since the replica's state (h, global index, row), device
    int64_t* log_h = nullptr;
    int64_t* log_g = nullptr;
    uint64_t* log_k = nullptr;
    int64_t log_n = 0, log_cap = 0, log_limit = 0;
    HostValuesWide rep;           // the exact RandomValues state before the log's first entry
    bool rep_stale = false;       // a merge replaced the set: rebuild the replica from it first
    bool merged = false;          // the log still describes the pre-merge history (rsv_export_log)
    bool retain = false;          // keep the consumed log on the host (rsv_retain_log)
    bool arch_ok = true;
    std::vector<int64_t> arch_h;  // consumed candidates in arrival order
    std::vector<uint64_t> arch_k;
    // ordered mode's scheduled pass: range table + verification counts (device [0, 2 kWMaxR + 1) the
    // table, [kSchedCounts, + kWMaxR + 1) the counts; pinned staging alike)
    int64_t* sched = nullptr;
    int64_t* hsched = nullptr;
    // the bucketed merge's area (wb_scatter / wb_sort / wb_emit), sized for wb_cap buckets
    int64_t* wb_h = nullptr;
    uint32_t* wb_e = nullptr;
    int64_t* wb_a = nullptr;
    uint32_t* wb_cnt = nullptr;
    uint32_t* wb_dist = nullptr;
    uint32_t* wb_gsum = nullptr;
    uint32_t wb_cap = 0;
    bool wb_cnt_dirty = false;    // a new bucket area: its counters are zeroed by the next wb_prep
    bool bucketed_on = true;      // RSV_WIDE_BUCKETED=0: the sort-based merge only (A/B, tests)
    bool last_bucketed = false;   // the last merge's sorted entries are in the bucket area (wb_verify)
    uint32_t last_B = 0;
    WSegTable hwb_seg;            // the bucket map's segment table (passed by value to wb_scatter)
    int64_t merges = 0;           // merges applied (a set swap each)
    // speculative publication (set mode's one-pass batches, wide_spec_target): armed around the pass,
    // enqueued behind its merge; valid when the pass proved its bound and no other merge followed
    void* spec_dst = nullptr;
    uint32_t* spec_flag = nullptr;
    uint32_t* spec_gen_ctr = nullptr;
    bool spec_arm = false, spec_ok = false;
    uint32_t spec_gen = 0;
    int64_t spec_merges = -1;
    double sched_beta = 1.6;      // bound margin over the predicted k-th smallest hash
    int64_t first_min = 4096;     // logs at least this long replay through first-occurrence flags
    bool sched_on = true;
    // pinned host copies of the log for the replay (hashes, rows, first-occurrence flags), kept
    // between replays: a fresh pageable vector per replay paid its page faults and zero fill, and
    // pageable copies run at about half the DMA rate
    int64_t* p_oh = nullptr;
    uint64_t* p_ok = nullptr;
    uint32_t* p_fl = nullptr;
    int64_t p_cap = 0;
};

namespace {

hipError_t walloc(void** p, size_t bytes) { return pool_device_alloc(p, bytes ? bytes : 16); }

// replace a device buffer by a larger one (contents kept when `keep`); the stream is synchronized
// before the old block goes back to the pool
hipError_t wgrow(void** p, size_t old_bytes, size_t new_bytes, bool keep, hipStream_t st) {
    void* q = nullptr;
    hipError_t e = walloc(&q, new_bytes);
    if (e != hipSuccess) return e;
    if (keep && *p && old_bytes) e = hipMemcpyAsync(q, *p, old_bytes, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && *p) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        pool_device_free(q);
        return e;
    }
    pool_device_free(*p);
    *p = q;
    return hipSuccess;
}

int64_t wgrown(int64_t cur, int64_t need) {
    int64_t c = std::max<int64_t>(cur, 1024);
    while (c < need) c *= 2;
    return c;
}

hipError_t ensure_set(WideDistinct* d, int64_t need, hipStream_t st) {
    need = std::min<int64_t>(need, d->k);
    if (need <= d->set_cap) return hipSuccess;
    const int64_t c = std::min<int64_t>(wgrown(d->set_cap, need), d->k);
    const size_t W = (size_t)d->words * 8;
    hipError_t e;
    if ((e = wgrow((void**)&d->set_h, (size_t)d->m * 8, (size_t)c * 8, true, st))) return e;
    if ((e = wgrow((void**)&d->set_k, (size_t)d->m * W, (size_t)c * W, true, st))) return e;
    if ((e = wgrow((void**)&d->set_h2, 0, (size_t)c * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->set_k2, 0, (size_t)c * W, false, st))) return e;
    d->set_cap = c;
    return hipSuccess;
}

hipError_t ensure_cand(WideDistinct* d, int64_t need, hipStream_t st) {
    if (need <= d->cand_cap) return hipSuccess;
    const int64_t c = wgrown(d->cand_cap, need);
    hipError_t e;
    if ((e = wgrow((void**)&d->cand_h, 0, (size_t)c * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->cand_i, 0, (size_t)c * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->cand_k, 0, (size_t)c * d->words * 8, false, st))) return e;
    d->cand_cap = c;
    return hipSuccess;
}

hipError_t ensure_merge(WideDistinct* d, int64_t N, hipStream_t st) {
    if (N <= d->merge_cap) return hipSuccess;
    const int64_t c = wgrown(d->merge_cap, N);
    hipError_t e;
    if ((e = wgrow((void**)&d->eh0, 0, (size_t)c * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->eh1, 0, (size_t)c * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->ev0, 0, (size_t)c * 4, false, st))) return e;
    if ((e = wgrow((void**)&d->ev1, 0, (size_t)c * 4, false, st))) return e;
    if ((e = wgrow((void**)&d->flags, 0, (size_t)c * 4, false, st))) return e;
    if ((e = wgrow((void**)&d->pos, 0, (size_t)c * 4, false, st))) return e;
    size_t a = 0, b = 0, g = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, a, (int64_t*)nullptr, (int64_t*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, (size_t)c)))
        return e;
    if ((e = rocprim::exclusive_scan(nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)c,
                                     rocprim::plus<uint32_t>())))
        return e;
    if ((e = rocprim::radix_sort_pairs(nullptr, g, (int64_t*)nullptr, (int64_t*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, (size_t)c)))
        return e;
    const size_t tb = std::max(a, std::max(b, g));
    if (tb > d->temp_bytes) {
        if ((e = wgrow(&d->temp, 0, tb, false, st))) return e;
        d->temp_bytes = tb;
    }
    d->merge_cap = c;
    return hipSuccess;
}

hipError_t ensure_temp(WideDistinct* d, size_t bytes, hipStream_t st) {
    if (bytes <= d->temp_bytes) return hipSuccess;
    hipError_t e = wgrow(&d->temp, 0, bytes, false, st);
    if (e == hipSuccess) d->temp_bytes = bytes;
    return e;
}

hipError_t read_ctl(WideDistinct* d, hipStream_t st) {
    hipError_t e = hipMemcpyAsync(d->hctl, d->ctl, 8 * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
}

// the bucket area for B buckets (the counters zeroed: every merge leaves the ones it used zero)
hipError_t ensure_buckets(WideDistinct* d, uint32_t B, hipStream_t st) {
    if (B <= d->wb_cap) return hipSuccess;
    const size_t c = std::max<uint32_t>(B, 64);
    hipError_t e;
    if ((e = wgrow((void**)&d->wb_h, 0, c * kWCap * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->wb_e, 0, c * kWCap * 4, false, st))) return e;
    if ((e = wgrow((void**)&d->wb_a, 0, c * kWCap * 8, false, st))) return e;
    if ((e = wgrow((void**)&d->wb_dist, 0, c * 4, false, st))) return e;
    if ((e = wgrow((void**)&d->wb_gsum, 0, (c / 16 + 1) * 4, false, st))) return e;
    if ((e = wgrow((void**)&d->wb_cnt, 0, c * kWStride * 4, false, st))) return e;
    d->wb_cnt_dirty = true;
    d->wb_cap = (uint32_t)c;
    return hipSuccess;
}

// A stretch of the hash axis with the entries expected in it: the bucket map's segments ascend
// by `lo` (the first from INT64_MIN), each reaching the next one's lo (the last: the merge's largest h)
struct WSeg {
    int64_t lo;
    double expect;
};

// The bucketed merge (wb_scatter -> wb_sort -> wb_emit) of set ∪ candidates [0, c); span_hi bounds
// every entry's h; `segs` (optional) describe how the entries spread along h (default: uniform).
// *done = false when a bucket or a run of equal h overflowed (a degenerate hash): the sort-based
// merge then runs instead (the counters are zero again, the set untouched).
hipError_t merge_bucketed(WideDistinct* d, int64_t c, int64_t span_hi, bool arrivals,
                          const std::vector<WSeg>* segs, hipStream_t st, bool* done, bool c_on_device = false) {
    // c_on_device: c is the candidates' room, the count itself is the filter's counter ctl[0] (no host
    // read between the filter and the merge); the caller reads ctl[0] afterwards
    *done = false;
    const int64_t N = d->m + c;
    int64_t hi = span_hi;
    if (d->m > 0 && d->top > hi) hi = d->top;
    std::vector<WSeg> one{WSeg{INT64_MIN, 1.0}};
    const std::vector<WSeg>& sg = segs && !segs->empty() && (int)segs->size() <= kWSegMax ? *segs : one;
    const int32_t ns = (int32_t)sg.size();
    hipError_t e;
    // buckets: ~64 entries each overall, shared out in proportion to each segment's expected entries
    const int64_t Bt = std::min<int64_t>(std::max<int64_t>((N + (1 << kWAvgLog) - 1) >> kWAvgLog, 1), 1 << 24);
    double tot = 0;
    for (const WSeg& x : sg) tot += std::max(x.expect, 0.0);
    int64_t* lo = d->hwb_seg.w;
    int64_t* b0 = lo + kWSegMax + 1;
    int64_t* mult = lo + 2 * kWSegMax + 2;
    int64_t* nb = lo + 3 * kWSegMax + 2;
    double cum = 0;
    int64_t B = 0;
    for (int32_t i = 0; i < ns; ++i) {
        cum += std::max(sg[i].expect, 0.0);
        const int64_t end = tot > 0 ? (int64_t)((double)Bt * cum / tot + 0.5) : Bt * (i + 1) / ns;
        const int64_t n = std::max<int64_t>(end - B, 1);
        lo[i] = i == 0 ? INT64_MIN : sg[i].lo;
        b0[i] = B;
        nb[i] = n;
        const int64_t seg_hi = i + 1 < ns ? sg[i + 1].lo - 1 : std::max(hi, lo[i]);
        const uint64_t span = (uint64_t)seg_hi - (uint64_t)lo[i];
        const uint64_t q = span == ~0ull ? 1ull : ~0ull / (span + 1);
        mult[i] = (int64_t)(q <= ~0ull / (uint64_t)n ? q * (uint64_t)n : 0ull);
        B += n;
    }
    lo[ns] = INT64_MAX;
    b0[ns] = B;
    if ((e = ensure_buckets(d, (uint32_t)B, st))) return e;
    const WRows R{d->set_k, d->cand_k, d->m, d->words};
    // ctl[1..6]; ctl[0] is the filter's count when c_on_device, ctl[7] the publication ticket (always 0)
    const uint32_t n_cnt = d->wb_cnt_dirty ? d->wb_cap * kWStride : 0u;
    hipLaunchKernelGGL(wb_prep, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n_cnt + 4 * kWBlock - 1) / (4 * kWBlock), 256))),
                       dim3(kWBlock), 0, st, d->ctl, d->wb_cnt, n_cnt);
    d->wb_cnt_dirty = false;
    hipLaunchKernelGGL(wb_scatter, dim3(wgrid(N, 8192)), dim3(kWBlock), 0, st, d->set_h, d->m, d->cand_h, c, d->hwb_seg,
                       ns, (uint32_t)B, d->wb_h, d->wb_e, d->wb_cnt, d->wb_gsum, d->ctl, c_on_device);
    hipLaunchKernelGGL(wb_sort, dim3((unsigned)((B + kWBlock / 64 - 1) / (kWBlock / 64))), dim3(kWBlock), 0, st, d->m,
                       (uint32_t)B, d->wb_h, d->wb_e, arrivals ? d->wb_a : nullptr, d->wb_cnt, d->wb_dist, d->wb_gsum, R,
                       d->cand_i, d->ctl);
    hipLaunchKernelGGL(wb_emit, dim3((unsigned)((B + kWEmitBuckets - 1) / kWEmitBuckets)), dim3(kWBlock), 0, st,
                       (uint32_t)B, d->wb_h, d->wb_e, d->wb_dist, d->wb_gsum, (int64_t)d->k, R, d->set_h2, d->set_k2,
                       d->ctl);
    if ((e = hipGetLastError())) return e;
    if (d->spec_arm && d->spec_dst) {  // the merged set straight to the host, before the host reads ctl
        const uint32_t gen = ++*d->spec_gen_ctr;
        if ((e = launch_publish_multi(d->set_k2, (int64_t)d->k * d->words * 8, d->spec_dst, d->spec_flag, gen,
                                      (uint32_t*)(d->ctl + 7), st)))
            return e;
        d->spec_gen = gen;
        d->spec_merges = d->merges + 1;
    }
    if ((e = read_ctl(d, st))) return e;
    if (d->hctl[1]) {
        d->spec_merges = -1;  // what was published is not a merge result
        return hipSuccess;
    }
    d->m = std::min<int64_t>(d->hctl[2], d->k);
    d->top = d->hctl[3];
    d->tied = d->m == d->k && d->hctl[4] != 0;
    std::swap(d->set_h, d->set_h2);
    std::swap(d->set_k, d->set_k2);
    d->last_bucketed = true;
    d->last_B = (uint32_t)B;
    ++d->merges;
    *done = true;
    return hipSuccess;
}

// set ∪ candidates [0, c) -> bottom-k by (h, key words), distinct by (h, key); `tied` from this merge.
// span_hi: no candidate's h exceeds it (the filter's bound); arrivals: keep each element's first
// arrival for the scheduled pass's proof
hipError_t merge_cands(WideDistinct* d, int64_t c, hipStream_t st, int64_t span_hi = INT64_MAX,
                       bool arrivals = false, const std::vector<WSeg>* segs = nullptr, bool sort_only = false) {
    if (c <= 0) return hipSuccess;
    const int64_t N = d->m + c;
    hipError_t e;
    if ((e = ensure_set(d, std::min<int64_t>(N, d->k), st))) return e;
    d->last_bucketed = false;
    if (d->bucketed_on && !sort_only && N < ((int64_t)1 << 30)) {
        bool done = false;
        if ((e = merge_bucketed(d, c, span_hi, arrivals, segs, st, &done))) return e;
        if (done) return hipSuccess;
    }
    // the sort-based merge: a 64-bit radix sort by h, runs of equal h by the key words
    if ((e = ensure_merge(d, N, st))) return e;
    const WRows R{d->set_k, d->cand_k, d->m, d->words};
    const unsigned g = wgrid(N, 4096);
    hipLaunchKernelGGL(wide_merge_init, dim3(g), dim3(kWBlock), 0, st, d->set_h, d->cand_h, d->m, N, d->eh0, d->ev0);
    size_t tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->eh0, d->eh1, d->ev0, d->ev1, (size_t)N, 0, 64, st))) return e;
    if ((e = hipMemsetAsync(d->ctl, 0, 8 * 8, st))) return e;
    hipLaunchKernelGGL(wide_run_fix, dim3(g), dim3(kWBlock), 0, st, d->eh1, d->ev1, N, R, d->ctl);
    auto finish = [&]() -> hipError_t {
        hipLaunchKernelGGL(wide_flags, dim3(g), dim3(kWBlock), 0, st, d->eh1, d->ev1, N, R, d->flags);
        size_t sb = d->temp_bytes;
        hipError_t e2 = rocprim::exclusive_scan(d->temp, sb, d->flags, d->pos, 0u, (size_t)N, rocprim::plus<uint32_t>(),
                                                st);
        if (e2) return e2;
        hipLaunchKernelGGL(wide_emit, dim3(g), dim3(kWBlock), 0, st, d->eh1, d->ev1, d->flags, d->pos, N,
                           (int64_t)d->k, R, d->set_h2, d->set_k2, d->ctl);
        if ((e2 = hipGetLastError())) return e2;
        return read_ctl(d, st);
    };
    if ((e = finish())) return e;
    if (d->hctl[1]) {  // a run of > kRunMax equal hashes: the comparison sort orders the whole merge
        size_t mb = 0;
        const WLess less{d->eh0, R};
        if ((e = rocprim::merge_sort(nullptr, mb, d->ev1, d->ev1, (size_t)N, less, st))) return e;
        if ((e = ensure_temp(d, mb, st))) return e;
        hipLaunchKernelGGL(wide_iota, dim3(g), dim3(kWBlock), 0, st, d->ev0, N);
        mb = d->temp_bytes;
        if ((e = rocprim::merge_sort(d->temp, mb, d->ev0, d->ev1, (size_t)N, less, st))) return e;
        hipLaunchKernelGGL(wide_gather_h, dim3(g), dim3(kWBlock), 0, st, d->eh0, d->ev1, N, d->eh1);
        if ((e = hipMemsetAsync(d->ctl, 0, 8 * 8, st))) return e;
        if ((e = finish())) return e;
    }
    const int64_t nd = d->hctl[2];
    d->m = std::min<int64_t>(nd, d->k);
    d->top = d->hctl[3];
    d->tied = d->m == d->k && d->hctl[4] != 0;
    std::swap(d->set_h, d->set_h2);
    std::swap(d->set_k, d->set_k2);
    ++d->merges;
    return hipSuccess;
}

// the device set := the replica's members, put in ascending (h, key words) order on the device (the
// merge of an empty set with them as candidates; a host sort of 65536 rows took ~10 ms)
hipError_t upload_replica(WideDistinct* d, hipStream_t st) {
    std::vector<int64_t> hs;
    std::vector<uint64_t> rows;
    d->rep.members_heap(hs, rows);
    const int64_t nm = (int64_t)hs.size();
    hipError_t e;
    if ((e = ensure_set(d, nm, st))) return e;
    d->m = 0;
    if (!nm) return hipSuccess;
    if ((e = ensure_cand(d, nm, st))) return e;
    if ((e = hipMemcpyAsync(d->cand_h, hs.data(), (size_t)nm * 8, hipMemcpyHostToDevice, st))) return e;
    if ((e = hipMemcpyAsync(d->cand_k, rows.data(), (size_t)nm * d->words * 8, hipMemcpyHostToDevice, st))) return e;
    const bool tied = d->tied;
    if ((e = merge_cands(d, nm, st))) return e;  // synchronizes (its control words): hs / rows may go
    d->tied = tied;
    return hipSuccess;
}

// the replica from the device set (after a merge replaced it): its members inserted in (h, key) order
hipError_t rebuild_replica(WideDistinct* d, hipStream_t st) {
    d->rep.reset(d->k, d->words);
    d->rep_stale = false;
    if (!d->m) return hipSuccess;
    std::vector<int64_t> hs((size_t)d->m);
    std::vector<uint64_t> rows((size_t)(d->m * d->words));
    hipError_t e = hipMemcpyAsync(hs.data(), d->set_h, hs.size() * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(rows.data(), d->set_k, rows.size() * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    for (int64_t i = 0; i < d->m; ++i) d->rep.sample(hs[(size_t)i], rows.data() + (size_t)i * d->words);
    return hipSuccess;
}

// the log in arrival order on the host: sort by global index on the device, permute, copy back
// into oh[n] / ok[n x words] (synchronized when `sync`)
hipError_t log_to_host(WideDistinct* d, int64_t* oh, uint64_t* ok, hipStream_t st, bool sync = true) {
    const int64_t n = d->log_n;
    if (!n) return hipSuccess;
    hipError_t e;
    if ((e = ensure_merge(d, n, st))) return e;
    if ((e = ensure_cand(d, n, st))) return e;
    const unsigned g = wgrid(n, 4096);
    hipLaunchKernelGGL(wide_iota, dim3(g), dim3(kWBlock), 0, st, d->ev0, n);
    size_t tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->log_g, d->eh1, d->ev0, d->ev1, (size_t)n, 0, 64, st)))
        return e;
    hipLaunchKernelGGL(wide_log_permute, dim3(g), dim3(kWBlock), 0, st, d->ev1, d->log_h, d->log_k, n, d->words,
                       d->cand_h, d->cand_k);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync(oh, d->cand_h, (size_t)n * 8, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipMemcpyAsync(ok, d->cand_k, (size_t)n * d->words * 8, hipMemcpyDeviceToHost, st))) return e;
    return sync ? hipStreamSynchronize(st) : hipSuccess;
}

hipError_t log_to_host(WideDistinct* d, std::vector<int64_t>& oh, std::vector<uint64_t>& ok, hipStream_t st) {
    oh.resize((size_t)d->log_n);
    ok.resize((size_t)(d->log_n * d->words));
    return log_to_host(d, oh.data(), ok.data(), st);
}

// the replay's pinned copies for a log of n entries
hipError_t ensure_pinned_log(WideDistinct* d, int64_t n) {
    if (n <= d->p_cap) return hipSuccess;
    const int64_t c = std::max<int64_t>(n, 2 * d->p_cap);
    pool_host_free(d->p_oh);
    pool_host_free(d->p_ok);
    pool_host_free(d->p_fl);
    d->p_oh = nullptr;
    d->p_ok = nullptr;
    d->p_fl = nullptr;
    d->p_cap = 0;
    hipError_t e;
    if ((e = pool_host_alloc((void**)&d->p_oh, (size_t)c * 8, hipHostMallocDefault))) return e;
    if ((e = pool_host_alloc((void**)&d->p_ok, (size_t)c * d->words * 8, hipHostMallocDefault))) return e;
    if ((e = pool_host_alloc((void**)&d->p_fl, (size_t)c * 4, hipHostMallocDefault))) return e;
    d->p_cap = c;
    return hipSuccess;
}

// First-occurrence flags of the log (already in arrival order in cand_h / cand_k, log_to_host):
// entries [the replica's members | the log] through the merge's sort (stable radix by h, runs of
// equal h stably by the key words, or the comparison sort for runs > kRunMax), then wide_mark_first.
hipError_t first_flags(WideDistinct* d, uint32_t* flags, hipStream_t st) {
    const int64_t n = d->log_n;
    std::vector<int64_t> mh;
    std::vector<uint64_t> mk;
    d->rep.members_heap(mh, mk);  // (any order: the sort below groups the keys)
    const int64_t nm = (int64_t)mh.size(), N = nm + n;
    hipError_t e;
    if ((e = ensure_set(d, nm, st))) return e;
    if ((e = ensure_merge(d, N, st))) return e;
    if (nm) {
        if ((e = hipMemcpyAsync(d->set_h2, mh.data(), (size_t)nm * 8, hipMemcpyHostToDevice, st))) return e;
        if ((e = hipMemcpyAsync(d->set_k2, mk.data(), (size_t)nm * d->words * 8, hipMemcpyHostToDevice, st))) return e;
    }
    const WRows R{d->set_k2, d->cand_k, nm, d->words};
    const unsigned g = wgrid(N, 4096);
    hipLaunchKernelGGL(wide_merge_init, dim3(g), dim3(kWBlock), 0, st, d->set_h2, d->cand_h, nm, N, d->eh0, d->ev0);
    size_t tb = d->temp_bytes;
    if ((e = rocprim::radix_sort_pairs(d->temp, tb, d->eh0, d->eh1, d->ev0, d->ev1, (size_t)N, 0, 64, st))) return e;
    if ((e = hipMemsetAsync(d->ctl, 0, 8 * 8, st))) return e;
    hipLaunchKernelGGL(wide_run_fix, dim3(g), dim3(kWBlock), 0, st, d->eh1, d->ev1, N, R, d->ctl);
    if ((e = read_ctl(d, st))) return e;
    if (d->hctl[1]) {  // a run longer than kRunMax: the (stable) comparison sort over (h, key words)
        size_t mb = 0;
        const WLess less{d->eh0, R};
        if ((e = rocprim::merge_sort(nullptr, mb, d->ev1, d->ev1, (size_t)N, less, st))) return e;
        if ((e = ensure_temp(d, mb, st))) return e;
        hipLaunchKernelGGL(wide_iota, dim3(g), dim3(kWBlock), 0, st, d->ev0, N);
        mb = d->temp_bytes;
        if ((e = rocprim::merge_sort(d->temp, mb, d->ev0, d->ev1, (size_t)N, less, st))) return e;
        hipLaunchKernelGGL(wide_gather_h, dim3(g), dim3(kWBlock), 0, st, d->eh0, d->ev1, N, d->eh1);
    }
    hipLaunchKernelGGL(wide_mark_first, dim3(g), dim3(kWBlock), 0, st, d->eh1, d->ev1, N, R, d->pos);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync(flags, d->pos, (size_t)n * 4, hipMemcpyDeviceToHost, st))) return e;
    return hipStreamSynchronize(st);
}

// Consume the log: replay it in arrival order through the replica (the reference's sequential
// RandomValues), archive it if retained, and make the device set the replica's (exact) set.  Long
// logs replay first occurrences only, through the heap alone (sample_first: no element set).
hipError_t replay_log(WideDistinct* d, hipStream_t st) {
    hipError_t e;
    if (d->rep_stale && (e = rebuild_replica(d, st))) return e;
    const bool first = d->log_n > 0 && d->log_n >= d->first_min;
    const int64_t n_log = d->log_n;
    const auto t0 = std::chrono::steady_clock::now();
    if ((e = ensure_pinned_log(d, n_log))) return e;
    const int64_t* oh = d->p_oh;
    const uint64_t* ok = d->p_ok;
    // the log's copies are enqueued before the flags' sort (one wait for both when first)
    if ((e = log_to_host(d, d->p_oh, d->p_ok, st, !first))) return e;
    const auto t1 = std::chrono::steady_clock::now();
    auto t2 = t1;
    if (first) {
        const uint32_t* fl = d->p_fl;
        if ((e = first_flags(d, d->p_fl, st))) return e;
        t2 = std::chrono::steady_clock::now();
        // members name log entries during the run (no row moves per replacement), then take slots
        for (int64_t t = 0; t < n_log; ++t)
            if (fl[t]) d->rep.sample_first_at(oh[t], t);
        d->rep.adopt(ok);
        d->rep.table_rebuild();
    } else {
        for (int64_t t = 0; t < n_log; ++t) d->rep.sample(oh[t], ok + t * d->words);
    }
    const auto t3 = std::chrono::steady_clock::now();
    if (d->retain && d->arch_ok) {
        if ((int64_t)d->arch_h.size() + n_log > ((int64_t)1 << 27)) {
            d->arch_ok = false;
            d->arch_h.clear();
            d->arch_k.clear();
        } else {
            d->arch_h.insert(d->arch_h.end(), oh, oh + n_log);
            d->arch_k.insert(d->arch_k.end(), ok, ok + n_log * d->words);
        }
    }
    d->log_n = 0;
    if ((e = upload_replica(d, st))) return e;
    d->exact = true;
    if (std::getenv("RSV_REPLAY_DEBUG")) {
        const auto t4 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        std::fprintf(stderr, "[rsv wide replay] log=%lld first=%d to_host_us=%.1f flags_us=%.1f run_us=%.1f upload_us=%.1f\n",
                     (long long)n_log, (int)first, us(t0, t1), us(t1, t2), us(t2, t3), us(t3, t4));
    }
    return hipSuccess;
}

hipError_t ensure_log(WideDistinct* d, int64_t need, hipStream_t st) {
    if (need <= d->log_cap) return hipSuccess;
    const int64_t c = wgrown(d->log_cap, need);
    const size_t W = (size_t)d->words * 8;
    void* nb[3] = {nullptr, nullptr, nullptr};
    const size_t bytes[3] = {(size_t)c * 8, (size_t)c * 8, (size_t)c * W};
    const size_t used[3] = {(size_t)d->log_n * 8, (size_t)d->log_n * 8, (size_t)d->log_n * W};
    void** old[3] = {(void**)&d->log_h, (void**)&d->log_g, (void**)&d->log_k};
    hipError_t e = hipSuccess;
    for (int i = 0; i < 3 && e == hipSuccess; ++i) e = walloc(&nb[i], bytes[i]);
    for (int i = 0; i < 3 && e == hipSuccess; ++i)
        if (*old[i] && used[i]) e = hipMemcpyAsync(nb[i], *old[i], used[i], hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && (d->log_h || d->log_g || d->log_k)) e = hipStreamSynchronize(st);  // one wait, three copies
    if (e != hipSuccess) {
        for (void* p : nb) pool_device_free(p);
        return e;
    }
    for (int i = 0; i < 3; ++i) {
        pool_device_free(*old[i]);
        *old[i] = nb[i];
    }
    d->log_cap = c;
    return hipSuccess;
}

// one chunk [off, off + L) of the batch: filter (bound: the set's maximum, or `bound_in` when given),
// rows, log, merge
hipError_t sample_chunk(WideDistinct* d, const void* keys, const int64_t* hashes, int64_t off, int64_t L,
                        int64_t gbase, hipStream_t st, const int64_t* bound_in = nullptr, int32_t R = 0,
                        int64_t* c_out = nullptr, const std::vector<WSeg>* segs = nullptr) {
    const uint64_t* rows = (const uint64_t*)keys + (size_t)off * d->words;
    const int64_t* hv = hashes ? hashes + off : nullptr;
    hipError_t e;
    int64_t c;
    // bounded log: replay what it holds before this chunk's candidates take the scratch buffers
    if (d->ordered && d->log_n > 0 && d->log_n + std::min<int64_t>(L, 8 * (int64_t)d->k + 4096) > d->log_limit)
        if ((e = replay_log(d, st))) return e;
    if (d->m < d->k && !bound_in) {  // still filling, no predicted bound: every element is a candidate
        if ((e = ensure_cand(d, L, st))) return e;
        if (d->src == kWideSrcHashes)
            hipLaunchKernelGGL(wide_hash_all<kWideSrcHashes>, dim3(wgrid(L, 8192)), dim3(kWBlock), 0, st, hv, rows, L,
                               d->r0, d->r1, d->cand_h, d->cand_i);
        else
            hipLaunchKernelGGL(wide_hash_all<kWideSrcUuid>, dim3(wgrid(L, 8192)), dim3(kWBlock), 0, st, hv, rows, L,
                               d->r0, d->r1, d->cand_h, d->cand_i);
        if ((e = hipGetLastError())) return e;
        c = L;
    } else {
        const int64_t bound = bound_in ? *bound_in : d->top;  // inclusive: the boundary bucket stays
        if ((e = ensure_cand(d, 8 * (int64_t)d->k + 4096, st))) return e;
        const unsigned g = (unsigned)std::min<int64_t>(
            std::max<int64_t>((L / (d->src == kWideSrcHashes ? 2 * kWideU : kWideU) + kWBlock - 1) / kWBlock, 1),
            kWideGrid);
        if (!d->ordered && d->bucketed_on && R == 0 && d->m + d->cand_cap < ((int64_t)1 << 30)) {
            // Set mode: filter, rows and the bucketed merge enqueued together -- the candidate count
            // stays on the device (the kernels read the filter's counter), one host read at the end
            for (;;) {
                if ((e = hipMemsetAsync(d->ctl, 0, 8, st))) return e;
                if (d->timer) d->timer->mark(st);
                if (d->src == kWideSrcHashes)
                    hipLaunchKernelGGL(wide_filter_hashes, dim3(g), dim3(kWBlock), 0, st, hv, L, d->r0, d->r1, bound,
                                       d->cand_h, d->cand_i, (unsigned long long*)d->ctl, d->cand_cap, d->sched, 0);
                else
                    hipLaunchKernelGGL(wide_filter_uuid, dim3(g), dim3(kWBlock), 0, st, rows, L, d->r0, d->r1, bound,
                                       d->cand_h, d->cand_i, (unsigned long long*)d->ctl, d->cand_cap, d->sched, 0);
                if (d->timer) d->timer->mark(st);
                hipLaunchKernelGGL(wide_gather_rows, dim3(wgrid(d->cand_cap * d->words, 8192)), dim3(kWBlock), 0, st,
                                   rows, d->cand_i, d->cand_cap, d->words, d->cand_k, (const int64_t*)d->ctl);
                if ((e = hipGetLastError())) return e;
                if ((e = ensure_set(d, std::min<int64_t>(d->m + d->cand_cap, d->k), st))) return e;
                d->last_bucketed = false;
                bool done = false;
                if ((e = merge_bucketed(d, d->cand_cap, bound, false, nullptr, st, &done, true))) return e;
                c = d->hctl[0];
                if (c > d->cand_cap) {  // more candidates than room (nothing merged): again, with room
                    if ((e = ensure_cand(d, c, st))) return e;
                    continue;
                }
                if (c_out) *c_out = c;
                // a degenerate hash overflowed a bucket: the sort-based merge of the same candidates
                if (!done && (e = merge_cands(d, c, st, bound, false, nullptr, true))) return e;
                return hipSuccess;
            }
        }
        for (;;) {
            if ((e = hipMemsetAsync(d->ctl, 0, 8, st))) return e;
            if (d->timer) d->timer->mark(st);
            if (d->src == kWideSrcHashes)
                hipLaunchKernelGGL(wide_filter_hashes, dim3(g), dim3(kWBlock), 0, st, hv, L, d->r0, d->r1, bound,
                                   d->cand_h, d->cand_i, (unsigned long long*)d->ctl, d->cand_cap, d->sched, R);
            else
                hipLaunchKernelGGL(wide_filter_uuid, dim3(g), dim3(kWBlock), 0, st, rows, L, d->r0, d->r1, bound,
                                   d->cand_h, d->cand_i, (unsigned long long*)d->ctl, d->cand_cap, d->sched, R);
            if (d->timer) d->timer->mark(st);
            if ((e = hipGetLastError())) return e;
            if ((e = read_ctl(d, st))) return e;
            c = d->hctl[0];
            if (c <= d->cand_cap) break;
            if ((e = ensure_cand(d, c, st))) return e;  // more candidates than room: again, with room
        }
    }
    if (c_out) *c_out = c;
    if (c == 0) return hipSuccess;
    hipLaunchKernelGGL(wide_gather_rows, dim3(wgrid(c * d->words, 8192)), dim3(kWBlock), 0, st, (const uint64_t*)keys +
                       (size_t)off * d->words, d->cand_i, c, d->words, d->cand_k);
    if ((e = hipGetLastError())) return e;
    if (d->ordered) {
        if ((e = ensure_log(d, d->log_n + c, st))) return e;
        hipLaunchKernelGGL(wide_log_append, dim3(wgrid(c * d->words, 8192)), dim3(kWBlock), 0, st, d->cand_h,
                           d->cand_i, d->cand_k, c, d->words, gbase + off, d->log_h + d->log_n, d->log_g + d->log_n,
                           d->log_k + (size_t)d->log_n * d->words);
        if ((e = hipGetLastError())) return e;
        d->log_n += c;
    }
    // no candidate's h exceeds the filter's bound (hash_all: any h)
    const int64_t span_hi = (d->m < d->k && !bound_in) ? INT64_MAX : (bound_in ? *bound_in : d->top);
    const int64_t hi = R > 0 ? d->hsched[R + 1] : span_hi;  // the scheduled pass: range 0's bound is the largest
    if ((e = merge_cands(d, c, st, std::max(hi, span_hi), d->ordered, segs))) return e;
    if (d->ordered) d->exact = !d->tied;  // an uncut boundary bucket leaves one possible set
    return hipSuccess;
}

// Ordered mode over a long rest (the set full): ONE filter pass whose bound falls with the index,
// like rsv_distinct.hip's scheduled pass.  Range 0 = [0, seen) of the rest takes the set's maximum
// (exact: the heap's maximum never rises); range r >= 1 = [(2^r - 1) seen, (2^(r+1) - 1) seen)
// takes B_r = MIN + (top - MIN) beta / 2^r -- the scrambled hash is uniform, so the k-th smallest of
// the 2^r seen lengths before the range sits near (top - MIN) / 2^r.  Every candidate is logged and
// merged as in a chunk; wide_verify then proves each range's bound (>= k distinct elements under
// B_r arrived before it, so the log holds every element the reference can admit there).  A failed
// proof restores the set and the log, and the chunk loop takes the rest (*ok = false).
hipError_t sample_sched(WideDistinct* d, const void* keys, const int64_t* hashes, int64_t off, int64_t rest,
                        int64_t gbase, hipStream_t st, bool* ok) {
    *ok = false;
    hipError_t e;
    if (!d->sched) {
        if ((e = walloc((void**)&d->sched, kSchedWords * 8))) return e;
        if ((e = pool_host_alloc((void**)&d->hsched, kSchedWords * 8, hipHostMallocDefault))) return e;
    }
    // a bounded log is replayed first (as sample_chunk would), so the state saved below is the one
    // the pass starts from
    if (d->log_n > 0 && d->log_n + std::min<int64_t>(rest, 8 * (int64_t)d->k + 4096) > d->log_limit)
        if ((e = replay_log(d, st))) return e;
    // the ranges (host; the pinned table's previous contents were consumed by a synchronized pass)
    const int64_t seen = std::max<int64_t>(d->seen, 1);
    const uint64_t span = (uint64_t)d->top - (uint64_t)INT64_MIN;
    int64_t* rs = d->hsched;
    int32_t R = 1;  // ranges [0, R): s_r = 2 s_(r-1) + seen = (2^r - 1) seen
    rs[0] = 0;
    while (R < kWMaxR && rs[R - 1] < (rest - seen) / 2) {
        rs[R] = 2 * rs[R - 1] + seen;
        ++R;
    }
    rs[R] = rest;
    int64_t* rb = rs + R + 1;
    rb[0] = d->top;
    for (int32_t r = 1; r < R; ++r) {
        const double frac = d->sched_beta / (double)((int64_t)1 << r);
        rb[r] = frac >= 1.0 ? d->top : (int64_t)((uint64_t)INT64_MIN + (uint64_t)((double)span * frac));
    }
    // room for the expected candidates (each range's length x the share of hashes under its bound,
    // +25 %): an overflow would run the whole filter again
    double expect = 0;
    for (int32_t r = 0; r < R; ++r)
        expect += (double)(rs[r + 1] - rs[r]) * ((double)((uint64_t)rb[r] - (uint64_t)INT64_MIN) / 18446744073709551616.0);
    // a set whose maximum sits high in the hash range (few distinct keys beyond k) would make most of
    // the rest candidates: the chunk loop bounds each chunk's instead
    if (expect > 32.0 * (double)d->k + (double)(1 << 22)) return hipSuccess;
    const int64_t room = (int64_t)(1.25 * expect) + 65536;
    if ((e = ensure_cand(d, room, st))) return e;
    if (d->ordered && (e = ensure_log(d, d->log_n + room, st))) return e;  // no log growth after the filter
    if ((e = hipMemcpyAsync(d->sched, rs, (size_t)(2 * R + 1) * 8, hipMemcpyHostToDevice, st))) return e;
    if ((e = hipMemsetAsync(d->sched + kSchedCounts, 0, (kWMaxR + 1) * 8, st))) return e;
    // the set and the scalars before the pass: the pass's one merge writes the other set buffers, so
    // a failed proof swaps back instead of restoring a copy
    const int64_t m0 = d->m, top0 = d->top, log0 = d->log_n, merges0 = d->merges;
    const bool tied0 = d->tied, exact0 = d->exact;
    // how the pass's merge entries spread along h (the bucket map, merge_bucketed): range r adds its
    // candidates uniformly below its bound B_r, so band (B_(j+1), B_j] holds ranges 0..j's; the set's
    // members spread uniformly below its maximum
    std::vector<WSeg> segs;
    {
        const double two64 = 18446744073709551616.0;
        const double tspan = (double)((uint64_t)d->top - (uint64_t)INT64_MIN) + 1.0;
        auto width = [](int64_t a, int64_t b) { return (double)((uint64_t)b - (uint64_t)a); };
        double lens = 0;  // ranges 0..R-1: all of them contribute to the lowest band
        for (int32_t r = 0; r < R; ++r) lens += (double)(rs[r + 1] - rs[r]);
        const double w0 = width(INT64_MIN, rb[R - 1]) + 1.0;
        segs.push_back(WSeg{INT64_MIN, lens * w0 / two64 + (double)d->m * w0 / tspan});
        for (int32_t j = R - 2; j >= 0; --j) {
            if (rb[j] <= rb[j + 1]) continue;  // an empty band (equal bounds)
            double lj = 0;
            for (int32_t r = 0; r <= j; ++r) lj += (double)(rs[r + 1] - rs[r]);
            const double wj = width(rb[j + 1], rb[j]);
            segs.push_back(WSeg{rb[j + 1] + 1, lj * wj / two64 + (double)d->m * wj / tspan});
        }
    }
    int64_t c = 0;
    if ((e = sample_chunk(d, keys, hashes, off, rest, gbase, st, nullptr, R, &c, &segs))) return e;
    if (d->merges - merges0 > 1) {  // (sample_chunk's bounded-log replay cannot run here: sample_sched ran it)
        set_error("wide scheduled pass: more than one merge");
        return hipErrorUnknown;
    }
    bool good = false;
    if (c > 0 && d->m == d->k) {  // the merge's sorted entries: the bucket area, or eh1 / ev1 / flags
        const int64_t N = m0 + c;
        if (d->last_bucketed)
            hipLaunchKernelGGL(wb_verify, dim3(std::min<uint32_t>((d->last_B + 3) / 4, 4096)), dim3(kWBlock), 0,
                               st, d->last_B, d->wb_h, d->wb_a, d->wb_dist, d->sched, R,
                               (unsigned long long*)(d->sched + kSchedCounts));
        else
            hipLaunchKernelGGL(wide_verify, dim3(wgrid(N, 4096)), dim3(kWBlock), 0, st, d->eh1, d->ev1, d->flags, N, m0,
                               d->cand_i, d->sched, R, (unsigned long long*)(d->sched + kSchedCounts));
        if ((e = hipGetLastError())) return e;
        if ((e = hipMemcpyAsync(d->hsched + kSchedCounts, d->sched + kSchedCounts, (size_t)(R + 1) * 8, hipMemcpyDeviceToHost, st)))
            return e;
        if ((e = hipStreamSynchronize(st))) return e;
        good = true;
        int64_t cnt = 0;
        for (int32_t r = 0; r < R; ++r) {
            cnt += d->hsched[kSchedCounts + r];
            if (r >= 1 && cnt < d->k) good = false;
        }
    }
    const bool debug = std::getenv("RSV_WIDE_SCHED_DEBUG") != nullptr;  // (read per pass: tests toggle it)
    if (debug)
        std::fprintf(stderr, "[rsv wide sched] rest=%lld ranges=%d candidates=%lld proof=%s merge=%s\n", (long long)rest,
                     R, (long long)c, good ? "ok" : "failed", d->last_bucketed ? "bucketed" : "sort");
    if (good) {
        *ok = true;
        return hipSuccess;
    }
    // the proof failed: the set (the merge's input, intact in the other buffers) and the log as before
    if (d->merges != merges0) {
        std::swap(d->set_h, d->set_h2);
        std::swap(d->set_k, d->set_k2);
        d->merges = merges0;
    }
    d->m = m0;
    d->top = top0;
    d->tied = tied0;
    d->exact = exact0;
    d->log_n = log0;
    return hipStreamSynchronize(st);
}

int fail_hip(hipError_t e, const char* what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? RSV_E_OUT_OF_MEMORY : RSV_E_DEVICE;
}

// a merge of external entries (rows of other ranks, exported states): bottom-k of the union; the
// replica restarts from the union when next needed (a merged set has no single arrival order --
// rsv_merge_log is the exact form), the log stays readable for rsv_export_log until the next sample
int merge_external(WideDistinct* d, const std::vector<std::pair<const int64_t*, const uint64_t*>>& src,
                   const std::vector<int64_t>& counts, const std::vector<int64_t>& tops,
                   const std::vector<int32_t>& part_tied, hipStream_t st) {
    // the tie rule across full runs: the smallest maximum among full parts, tied there
    int64_t T = d->m == d->k ? d->top : INT64_MAX;
    bool tiedT = d->m == d->k && d->tied;
    for (size_t p = 0; p < counts.size(); ++p) {
        if (counts[p] != d->k) continue;
        if (tops[p] < T) {
            T = tops[p];
            tiedT = part_tied[p] != 0;
        } else if (tops[p] == T) {
            tiedT = tiedT || part_tied[p] != 0;
        }
    }
    bool tie = d->m == d->k && d->tied;
    for (size_t p = 0; p < src.size(); ++p) {
        const int64_t n = counts[p];
        for (int64_t off = 0; off < n;) {
            const int64_t c = std::min<int64_t>(n - off, 8 * (int64_t)d->k + 4096);
            hipError_t e;
            if ((e = ensure_cand(d, c, st))) return fail_hip(e, "distinct merge");
            if ((e = hipMemcpyAsync(d->cand_h, src[p].first + off, (size_t)c * 8, hipMemcpyDeviceToDevice, st)))
                return fail_hip(e, "distinct merge");
            if ((e = hipMemcpyAsync(d->cand_k, src[p].second + (size_t)off * d->words, (size_t)c * d->words * 8,
                                    hipMemcpyDeviceToDevice, st)))
                return fail_hip(e, "distinct merge");
            const int64_t old_top = d->top;
            const bool was_full = d->m == d->k;
            if ((e = merge_cands(d, c, st))) return fail_hip(e, "distinct merge");
            tie = d->m == d->k && (d->tied || (tie && was_full && d->top == old_top));
            off += c;
        }
    }
    d->tied = d->m == d->k && (tie || (tiedT && d->top == T));
    if (d->ordered) {
        d->rep_stale = true;
        d->exact = true;
        d->merged = true;
    }
    return RSV_OK;
}

}  // namespace

// ---- entry points (rsv_internal.h) -------------------------------------------------------------

WideDistinct* wide_create(int32_t k, int key_width, int src, int64_t r0, int64_t r1, bool ordered, int* status) {
    WideDistinct* d = new WideDistinct();
    d->k = k;
    d->words = key_width / 8;
    d->src = src;
    d->r0 = r0;
    d->r1 = r1;
    d->ordered = ordered;
    d->log_limit = std::min<int64_t>(std::max<int64_t>(32 * (int64_t)k + 65536, (int64_t)1 << 22), (int64_t)1 << 27);
    if (const char* v = std::getenv("RSV_ORDERED_LOG_LIMIT"))  // test hook: force eager replays
        d->log_limit = std::max<int64_t>(1, std::atoll(v));
    if (ordered) d->rep.reset(k, d->words);
    if (const char* v = std::getenv("RSV_WIDE_SCHED")) d->sched_on = std::atoi(v) != 0;  // test hook: the chunk loop only
    if (const char* v = std::getenv("RSV_WIDE_SCHED_BETA"))  // test hook: tight bounds, failed proofs
        d->sched_beta = std::atof(v);
    if (const char* v = std::getenv("RSV_FIRST_MIN"))  // test hook: which replay form serves a log
        d->first_min = std::max<int64_t>(0, std::atoll(v));
    if (const char* v = std::getenv("RSV_WIDE_BUCKETED")) d->bucketed_on = std::atoi(v) != 0;  // A/B hook
    hipError_t e = walloc((void**)&d->ctl, 8 * 8);
    if (e == hipSuccess) e = hipMemset(d->ctl, 0, 8 * 8);  // ctl[7]: the publication ticket
    if (e == hipSuccess) e = pool_host_alloc((void**)&d->hctl, 8 * 8, hipHostMallocDefault);
    if (e != hipSuccess) {
        *status = fail_hip(e, "distinct_create (wide keys)");
        wide_destroy(d);
        return nullptr;
    }
    *status = RSV_OK;
    return d;
}

void wide_destroy(WideDistinct* d) {
    if (!d) return;
    void* ps[] = {d->set_h, d->set_k, d->set_h2, d->set_k2, d->cand_h, d->cand_i, d->cand_k, d->eh0, d->eh1,
                  d->ev0, d->ev1, d->flags, d->pos, d->temp, d->ctl, d->log_h, d->log_g, d->log_k};
    for (void* p : ps) pool_device_free(p);  // the owner's stream is idle (rsv_destroy)
    pool_device_free(d->sched);
    void* wb[] = {d->wb_h, d->wb_e, d->wb_a, d->wb_cnt, d->wb_dist, d->wb_gsum};
    for (void* p : wb) pool_device_free(p);
    pool_host_free(d->hsched);
    pool_host_free(d->hctl);
    pool_host_free(d->p_oh);
    pool_host_free(d->p_ok);
    pool_host_free(d->p_fl);
    delete d;
}

void wide_set_timer(WideDistinct* d, KernelTimer* t) { d->timer = t; }
int64_t wide_size(const WideDistinct* d) { return d->m; }
const void* wide_keys_dev(const WideDistinct* d) { return d->set_k; }
bool wide_is_ordered(const WideDistinct* d) { return d->ordered; }

int wide_sample_device(WideDistinct* d, const void* keys, const int64_t* hashes, int64_t n, hipStream_t st) {
    if (n <= 0) return RSV_OK;
    if (d->merged) {  // sampling on after a merge: the pre-merge candidates are history
        d->merged = false;
        d->log_n = 0;
        d->arch_h.clear();
        d->arch_k.clear();
        d->arch_ok = false;
    }
    const int64_t seen0 = d->seen;
    bool predicted = false;
    for (int64_t off = 0; off < n;) {
        const int64_t rest = n - off;
        if (d->ordered && d->sched_on && d->k >= kSchedMinK && d->m == d->k && !predicted && rest > 4 * d->seen) {
            predicted = true;
            bool ok = false;
            if (hipError_t e = sample_sched(d, keys, hashes, off, rest, seen0, st, &ok))
                return fail_hip(e, "distinct sample");
            if (ok) {
                d->seen += rest;
                break;
            }
            continue;  // a range's bound was short: the chunk loop below covers the same rest
        }
        if (!d->ordered && d->m == 0 && d->seen == 0 && !predicted && rest >= 64 * (int64_t)d->k) {
            // Set mode, a fresh sampler and a long batch: no filling chunk -- ONE pass under the bound
            // the batch's k-th smallest hash is predicted under if at least 1 / 2.5 of it is distinct
            // (uniform scrambled hashes: k / D of the range).  Proved like the pass below: a full
            // set whose maximum is <= B saw every element under it; else the chunk loop redoes the
            // batch (what the pass merged is seen again: duplicates merge away).
            predicted = true;
            const double frac = 2.5 * (double)d->k / (double)rest;
            const int64_t B = (int64_t)((uint64_t)INT64_MIN + (uint64_t)(18446744073709551616.0 * frac));
            d->spec_arm = true;
            hipError_t e = sample_chunk(d, keys, hashes, off, rest, seen0, st, &B);
            d->spec_arm = false;
            if (e) return fail_hip(e, "distinct sample");
            if (d->m == d->k && d->top <= B) {
                d->spec_ok = d->spec_dst && d->merges == d->spec_merges;  // the published set is the final one
                d->seen += rest;
                break;
            }
            continue;
        }
        if (!d->ordered && d->m == d->k && !predicted && rest > 4 * d->seen) {
            // Set mode, a long rest: ONE pass with the bound the rest's bottom-k is predicted under.
            // The scrambled hash is uniform, so the k-th smallest of D distinct values sits near
            // k / D of the range; with the rest's distinct share like the seen part's, the final
            // maximum is about (top - MIN) seen / (seen + rest) above MIN -- times beta = 2.  The
            // merge proves it: a full set whose maximum is <= B saw every element under it; else the
            // rest is filtered again by the chunk loop (duplicate candidates are merged away).
            predicted = true;
            const double frac = 2.0 * (double)d->seen / (double)(d->seen + rest);
            const uint64_t span = (uint64_t)d->top - (uint64_t)INT64_MIN;
            const int64_t B = frac >= 1.0 ? d->top : (int64_t)((uint64_t)INT64_MIN + (uint64_t)((double)span * frac));
            if (hipError_t e = sample_chunk(d, keys, hashes, off, rest, seen0, st, &B))
                return fail_hip(e, "distinct sample");
            if (d->m == d->k && d->top <= B) {
                d->seen += rest;
                break;
            }
            continue;  // the prediction was short: the chunk loop below covers the same rest
        }
        // filling: enough for the set plus slack; full: ~4 seen lengths (~4k candidates a chunk)
        const int64_t L = d->m < d->k ? std::min<int64_t>(rest, 4 * ((int64_t)d->k - d->m) + 4096)
                                      : std::min<int64_t>(rest, std::max<int64_t>(4 * d->seen, 1 << 16));
        if (hipError_t e = sample_chunk(d, keys, hashes, off, L, seen0, st)) return fail_hip(e, "distinct sample");
        off += L;
        d->seen += L;
    }
    return RSV_OK;
}

int wide_finalize(WideDistinct* d, hipStream_t st) {
    if (!d->ordered || d->exact) return RSV_OK;
    if (hipError_t e = replay_log(d, st)) return fail_hip(e, "distinct (ordered) replay");
    return RSV_OK;
}

int wide_publish(WideDistinct* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st) {
    const int64_t bytes = d->m * d->words * 8;
    // one workgroup's posted PCIe writes run at ~20 GB/s (a 1 MB UUID set: 45 us): large sets from
    // several workgroups (ctl[7] is the ticket: zero at creation, re-armed by every publication)
    if (bytes >= (64 << 10))
        RSV_HIP_TRY(launch_publish_multi(d->set_k, bytes, dst_host_dev, flag_dev, gen, (uint32_t*)(d->ctl + 7), st));
    else
        RSV_HIP_TRY(launch_publish(d->set_k, bytes, dst_host_dev, flag_dev, gen, st));
    return RSV_OK;
}

int wide_export(WideDistinct* d, void* keys_dev, int64_t* hash_dev, hipStream_t st) {
    if (d->m == 0) return RSV_OK;
    if (keys_dev)
        RSV_HIP_TRY(hipMemcpyAsync(keys_dev, d->set_k, (size_t)d->m * d->words * 8, hipMemcpyDeviceToDevice, st));
    if (hash_dev) RSV_HIP_TRY(hipMemcpyAsync(hash_dev, d->set_h, (size_t)d->m * 8, hipMemcpyDeviceToDevice, st));
    return RSV_OK;
}

void wide_info(const WideDistinct* d, int32_t* ordered, int32_t* tied, int32_t* retained, int64_t* size,
               int64_t* max_hash, int64_t* log_entries) {
    *ordered = d->ordered;
    *tied = d->m == d->k && d->tied;
    *retained = d->ordered && d->retain && d->arch_ok;
    *size = d->m;
    *max_hash = d->m ? d->top : INT64_MIN;
    *log_entries = d->ordered ? (int64_t)d->arch_h.size() + d->log_n : 0;
}

int wide_merge_parts(WideDistinct* d, const void* keys_dev, const int64_t* hash_dev, const int64_t* part_n,
                     int32_t parts, int64_t part_len, hipStream_t st) {
    if (int rc = wide_finalize(d, st)) return rc;
    std::vector<std::pair<const int64_t*, const uint64_t*>> src;
    std::vector<int64_t> counts, tops;
    std::vector<int32_t> ties;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t n = std::max<int64_t>(0, std::min(part_n[p], part_len));
        src.emplace_back(hash_dev + (size_t)p * part_len, (const uint64_t*)keys_dev + (size_t)p * part_len * d->words);
        counts.push_back(n);
        tops.push_back(INT64_MAX);  // no per-part tie information in this form
        ties.push_back(0);
    }
    return merge_external(d, src, counts, tops, ties, st);
}

int wide_export_row(WideDistinct* d, int64_t* row, int64_t count, hipStream_t st) {
    if (int rc = wide_finalize(d, st)) return rc;
    const int64_t k = d->k;
    const int64_t tied = d->m == k && d->tied, mx = d->m ? d->top : INT64_MIN;
    const int64_t ret = d->ordered && d->retain && d->arch_ok;
    hipLaunchKernelGGL(wide_export_row, dim3(wgrid(k * (d->words + 1), 4096)), dim3(kWBlock), 0, st, d->set_h,
                       d->set_k, d->m, k, d->words, row, count, tied, mx, ret, (int64_t)d->ordered);
    RSV_HIP_TRY(hipGetLastError());
    return RSV_OK;
}

int wide_merge_rows(WideDistinct* d, const int64_t* rows, int32_t parts, int64_t stride, hipStream_t st) {
    if (int rc = wide_finalize(d, st)) return rc;
    const int64_t k = d->k, kw = k * d->words;
    std::vector<int64_t> meta((size_t)parts * 6);
    for (int32_t p = 0; p < parts; ++p)
        RSV_HIP_TRY(hipMemcpyAsync(meta.data() + (size_t)p * 6, rows + (size_t)p * stride + kw + k, 6 * 8,
                                   hipMemcpyDeviceToHost, st));
    RSV_HIP_TRY(hipStreamSynchronize(st));
    std::vector<std::pair<const int64_t*, const uint64_t*>> src;
    std::vector<int64_t> counts, tops;
    std::vector<int32_t> ties;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t* mt = meta.data() + (size_t)p * 6;
        const int64_t* r = rows + (size_t)p * stride;
        src.emplace_back(r + kw, (const uint64_t*)r);
        counts.push_back(std::min(std::max<int64_t>(mt[0], 0), k));
        tops.push_back(mt[3]);
        ties.push_back(mt[2] != 0);
    }
    return merge_external(d, src, counts, tops, ties, st);
}

void wide_spec_target(WideDistinct* d, void* dst_host_dev, uint32_t* flag_dev, uint32_t* gen_counter) {
    if (d->ordered) return;  // (ordered mode: the scheduled pass's result waits for its proof)
    d->spec_dst = dst_host_dev;
    d->spec_flag = flag_dev;
    d->spec_gen_ctr = gen_counter;
    d->spec_ok = false;
}

bool wide_spec_take(WideDistinct* d, uint32_t* gen) {
    const bool ok = d->spec_ok && d->spec_dst;
    if (ok) *gen = d->spec_gen;
    d->spec_dst = nullptr;
    d->spec_arm = d->spec_ok = false;
    return ok;
}

void wide_retain_log(WideDistinct* d, bool on) {
    if (on && !d->retain && d->seen > 0) d->arch_ok = false;  // earlier candidates are gone
    d->retain = on;
    if (!on) {
        d->arch_h.clear();
        d->arch_k.clear();
    }
}

int wide_log_export(WideDistinct* d, int64_t bound, int64_t* out_h, void* out_k, int64_t cap, int64_t* out_n,
                    hipStream_t st) {
    if (!d->ordered || !d->retain || !d->arch_ok) {
        set_error(!d->ordered  ? "rsv_export_log needs an RSV_DISTINCT_ORDERED sampler"
                  : !d->retain ? "rsv_export_log: the candidate log was not retained (rsv_retain_log before sampling)"
                               : "rsv_export_log: the candidate log was not retained (archive limit, or sampled "
                                 "after a merge)");
        return RSV_E_UNSUPPORTED;
    }
    std::vector<int64_t> lh;
    std::vector<uint64_t> lk;
    if (hipError_t e = log_to_host(d, lh, lk, st)) return fail_hip(e, "rsv_export_log");
    const bool all = bound == INT64_MAX;
    const int64_t W = d->words;
    uint64_t* ok = (uint64_t*)out_k;
    int64_t cnt = 0;
    auto emit = [&](int64_t h, const uint64_t* r) {
        if (all || h < bound) {
            if (cnt < cap) {
                out_h[cnt] = h;
                std::memcpy(ok + cnt * W, r, (size_t)W * 8);
            }
            ++cnt;
        }
    };
    for (size_t i = 0; i < d->arch_h.size(); ++i) emit(d->arch_h[i], d->arch_k.data() + i * W);
    for (size_t i = 0; i < lh.size(); ++i) emit(lh[i], lk.data() + i * W);
    *out_n = cnt;
    if (cnt > cap && cap > 0) {
        set_error("rsv_export_log: cap is smaller than the number of candidates (*out_n)");
        return RSV_E_ILLEGAL_ARGUMENT;
    }
    return RSV_OK;
}

int wide_log_merge(WideDistinct* d, const int64_t* h, const void* keys, int64_t n, int64_t seen, hipStream_t st) {
    if (!d->ordered) {
        set_error("rsv_merge_log needs an RSV_DISTINCT_ORDERED sampler");
        return RSV_E_UNSUPPORTED;
    }
    d->rep.reset(d->k, d->words);
    d->rep_stale = false;
    const uint64_t* kk = (const uint64_t*)keys;
    for (int64_t t = 0; t < n; ++t) d->rep.sample(h[t], kk + (size_t)t * d->words);
    d->log_n = 0;
    d->arch_h.clear();
    d->arch_k.clear();
    if (hipError_t e = upload_replica(d, st)) return fail_hip(e, "rsv_merge_log");
    d->tied = false;
    d->exact = true;
    d->merged = true;
    d->seen = std::max(d->seen, seen);
    return RSV_OK;
}

}  // namespace rsv
