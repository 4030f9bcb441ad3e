// rsv_elements.hip -- gfx950 kernels for the element sampler (Sampler.apply, Sampler.scala:196-332)
// reformulated as data-parallel Algorithm R with counter-based draws (format R2, rsv_device.h).
//
//   K1  k1_last_writer   single stream: per-slot last writer (max index) of an index range
//   --  resolve          fill phase + gather of the winning keys into the reservoir
//   K1' replay_events    the reference's Algorithm-L eviction events -> per-slot last writer
//   --  merge_slots      multi-GPU combine of exported partial reservoirs (last writer wins)
//
// None of these kernels streams the key array: a draw depends only on (seed, stream, index), so
// only the k winning keys are ever read (DESIGN.md "Roofline").
#include <algorithm>

#include "rsv_device.h"
#include "rsv_internal.h"
#include "rsv_scan.h"

namespace rsv {

namespace {

constexpr int kBlock = 256;

// K1: grid-stride over level-0 blocks (16 indices each), two per lane per iteration; a pair with a
// zero byte is appended at once to the wave's LDS queue -- with its 32-bit zero-byte fold, so a
// sparse-region resolve needs no level-0 recompute -- and after every half window of 6 iterations
// the level-1 draws run 64 at a time, all lanes busy (rsv_scan.h k1_body_q).  Hits (k ln(n/k) of
// them) go straight to global atomicMax on the k-slot winner table: 14k atomics per 1e9 indices at k = 1024.
constexpr int kK1Unroll = 2;  // level-0 blocks per lane per iteration (two Philox chains in flight)

// ~20 four-wave workgroups per CU (6 resident: .sgpr_count 104): tools/micro_k1o r03ae/r03af, 1e9
// draws, 12-iteration windows: 85.0-85.5 us at 5086 workgroups (2 whole windows per wave) vs
// 87.5-89 us at 3072, 3390 (3 windows), 4096, 6144, 7629 and 10172 (1 window)
constexpr unsigned kK1Grid = 256 * 20;

// per-wave LDS of k1_body_q: pair queue (< 64 waiting + half a window of appends), the per-
// candidate queue.  12 iterations per window: tools/micro_k1o (r05k, 1e9 indices, grid 5086)
// 83.1-83.6 us vs 83.4-83.8 for 8 and 84.7-84.8 for 16, and 84.9-85.8 for the round-4 body
// (k1_body_p: window bits pushed in ballot rounds, tools/k1_dev_bodies.h), winners identical.
constexpr int kK1Win = 12;
struct K1Lds {
    uint64_t q[kBlock / 64][k1q_cap<kK1Win>()];
    uint64_t cq[kBlock / 64][kQueue];
};

// the launch-uniform conditions of k1_body_q's FAST resolve
__device__ __forceinline__ bool k1_fast(uint64_t lo, uint64_t hi) {
    return (lo >> 33) == ((hi - 1) >> 33) && hi <= (1ull << 40);
}

// the work layout of one K1 launch (k1_body_q): sch.A == 0 -- grid-stride windows; else the two-group
// schedule of half windows
struct K1Sched {
    uint32_t W1, A, B;
};

__global__ __launch_bounds__(kBlock) void k1_last_writer(DrawKey dk, uint32_t k, uint64_t lo,
                                                         uint64_t hi, uint64_t g_begin,
                                                         uint64_t n_groups,
                                                         unsigned long long* __restrict__ win, K1Sched sch) {
    __shared__ K1Lds L;
    const int w = threadIdx.x >> 6;
    if (k1_fast(lo, hi))
        k1_body_q<kK1Win, true>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], sch.W1, sch.A, sch.B);
    else
        k1_body_q<kK1Win, false>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], sch.W1, sch.A, sch.B);
}

// K1 + resolve_publish in one dispatch (single-launch batches, k <= kK1FusedMaxK): every
// workgroup takes a ticket after its winner atomics; the last one -- which then sees all of them --
// runs the resolve over the k slots (all loads of a lane issued before any store) and publishes
// the reservoir into coherent host memory, then re-arms the ticket.  Saves the kernel boundary
// and the resolve dispatch of the two-kernel form.
constexpr uint32_t kK1FusedMaxK = 8 * kBlock;

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void k1_resolve_publish(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi,
                                                             uint64_t g_begin, uint64_t n_groups,
                                                             unsigned long long* __restrict__ win,
                                                             uint32_t* ticket, const KeyT* __restrict__ keys,
                                                             int64_t base, int64_t n, KeyT* __restrict__ slot_key,
                                                             int64_t* __restrict__ slot_idx, int fresh, int64_t m,
                                                             KeyT* dst, uint32_t* flag, uint32_t gen, K1Sched sch) {
    __shared__ K1Lds L;
    __shared__ uint32_t last;
    const int w = threadIdx.x >> 6;
    if (k1_fast(lo, hi))
        k1_body_q<kK1Win, true>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], sch.W1, sch.A, sch.B);
    else
        k1_body_q<kK1Win, false>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], sch.W1, sch.A, sch.B);
    // This wave's winner atomics are performed once vmcnt drains: on gfx942/gfx950 a global atomic
    // without return still counts in vmcnt until the memory system acknowledges it (there is no
    // separate vscnt), and an agent-scope atomic is performed at the agent's coherence point (the
    // sc1 atomic path, LLVM AMDGPUUsage "Memory Model GFX942": agent-scope atomics bypass the
    // non-coherent per-XCD L2 state), where the last workgroup's agent-scope loads below read.
    // K1 makes no plain global stores, so there are no dirty L2 lines a release would have to
    // write back.  Measured alternatives: an agent-scope release/acquire fence per wave (a
    // buffer_wbl2 per wave + buffer_inv per workgroup) took the launch from 112 to 211 us at C2.
    // Only the last workgroup acquires (one L2 invalidate) before it reads the winners; the
    // parity tests (test_fused_k1_resolve_publish, the full-size C2 check) exercise this path.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == gridDim.x - 1;
        if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;  // workgroup-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    constexpr int R = kK1FusedMaxK / kBlock;
    unsigned long long wi[R];
    KeyT v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t j = threadIdx.x + r * kBlock;
        wi[r] = j < k ? __hip_atomic_load(&win[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = threadIdx.x + r * kBlock;
        if (j >= k) continue;
        if (wi[r]) v[r] = keys[(int64_t)wi[r] - base];
        else if (j >= base && j < base + n) v[r] = keys[j - base];
        else if (fresh) v[r] = 0;
        else v[r] = slot_key[j];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = threadIdx.x + r * kBlock;
        if (j >= k) continue;
        if (wi[r]) {
            slot_key[j] = v[r];
            slot_idx[j] = (int64_t)wi[r];
            win[j] = 0;
        } else if (j >= base && j < base + n) {
            slot_key[j] = v[r];
            slot_idx[j] = j;
        } else if (fresh) {
            slot_key[j] = 0;
            slot_idx[j] = -1;
        }
        if (j < m) dst[j] = v[r];
    }
    publish_flag(flag, gen);
}

// Per slot j: the batch's last writer (win[j], then cleared), else the fill of j < k from this
// batch, else -- first batch of a handle whose slots were never initialised (`fresh`) -- empty.
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void resolve_kernel(const KeyT* __restrict__ keys, int64_t base,
                                                         int64_t n, uint32_t k,
                                                         unsigned long long* __restrict__ win,
                                                         KeyT* __restrict__ slot_key,
                                                         int64_t* __restrict__ slot_idx, int fresh) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const unsigned long long wi = win[j];
    if (wi) {  // last eviction into slot j in this batch (Sampler.scala:243-246)
        slot_key[j] = keys[(int64_t)wi - base];
        if (slot_idx) slot_idx[j] = (int64_t)wi;
        win[j] = 0;
    } else if ((int64_t)j >= base && (int64_t)j < base + n) {  // fill phase (Sampler.scala:253-255)
        slot_key[j] = keys[j - base];
        if (slot_idx) slot_idx[j] = j;
    } else if (fresh) {
        slot_key[j] = 0;
        if (slot_idx) slot_idx[j] = -1;
    }
}

// resolve + publish in one dispatch (reservoirs of <= 8192 keys): one workgroup walks the k slots
// as resolve_kernel does, writes the first m final slot keys straight into coherent host memory,
// then publishes `gen` in the host flag with a system-scope release (as publish_kernel).
template <typename KeyT>
__global__ __launch_bounds__(1024) void resolve_publish_kernel(const KeyT* __restrict__ keys, int64_t base,
                                                               int64_t n, uint32_t k,
                                                               unsigned long long* __restrict__ win,
                                                               KeyT* __restrict__ slot_key,
                                                               int64_t* __restrict__ slot_idx, int fresh,
                                                               int64_t m, KeyT* dst, uint32_t* flag, uint32_t gen) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        const unsigned long long wi = win[j];
        KeyT v;
        if (wi) {
            v = keys[(int64_t)wi - base];
            slot_key[j] = v;
            slot_idx[j] = (int64_t)wi;
            win[j] = 0;
        } else if ((int64_t)j >= base && (int64_t)j < base + n) {
            v = keys[j - base];
            slot_key[j] = v;
            slot_idx[j] = j;
        } else if (fresh) {
            v = 0;
            slot_key[j] = 0;
            slot_idx[j] = -1;
        } else {
            v = slot_key[j];
        }
        if ((int64_t)j < m) dst[j] = v;
    }
    publish_flag(flag, gen);
}

// resolve_publish_kernel for one 256-thread workgroup with R slots per lane, all R winner loads
// issued before any key gather (k <= 256 R).  For a resolve forked onto a second stream beside the
// next batch's K1 (rsv_set_resolve_stream): 4 waves fit beside K1's six workgroups on a CU, where
// the 1024-thread form's 16 waves displace one of them (K1's first-generation schedule then ends late).
template <typename KeyT, int R>
__global__ __launch_bounds__(kBlock) void resolve_publish_small_kernel(const KeyT* __restrict__ keys, int64_t base,
                                                                       int64_t n, uint32_t k,
                                                                       unsigned long long* __restrict__ win,
                                                                       KeyT* __restrict__ slot_key,
                                                                       int64_t* __restrict__ slot_idx, int fresh,
                                                                       int64_t m, KeyT* dst, uint32_t* flag, uint32_t gen) {
    unsigned long long wi[R];
    KeyT v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t j = threadIdx.x + r * kBlock;
        wi[r] = j < k ? win[j] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = threadIdx.x + r * kBlock;
        if (j >= k) continue;
        if (wi[r]) v[r] = keys[(int64_t)wi[r] - base];
        else if (j >= base && j < base + n) v[r] = keys[j - base];
        else if (fresh) v[r] = 0;
        else v[r] = slot_key[j];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = threadIdx.x + r * kBlock;
        if (j >= k) continue;
        if (wi[r]) {
            slot_key[j] = v[r];
            slot_idx[j] = (int64_t)wi[r];
            win[j] = 0;
        } else if (j >= base && j < base + n) {
            slot_key[j] = v[r];
            slot_idx[j] = j;
        } else if (fresh) {
            slot_key[j] = 0;
            slot_idx[j] = -1;
        }
        if (j < m) dst[j] = v[r];
    }
    publish_flag(flag, gen);
}

__global__ __launch_bounds__(kBlock) void replay_kernel(const int64_t* __restrict__ ev_pos,
                                                        const int32_t* __restrict__ ev_slot,
                                                        int64_t n_events, uint32_t k,
                                                        unsigned long long* __restrict__ win) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_events) return;
    const int32_t s = ev_slot[e];
    const int64_t p = ev_pos[e];
    if (s >= 0 && (uint32_t)s < k && p >= 2) atomicMax(&win[s], (unsigned long long)(p - 1));
}

__global__ __launch_bounds__(kBlock) void export_draws_kernel(DrawKey dk, uint64_t i0, int64_t n,
                                                              uint64_t* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint64_t i = i0 + (uint64_t)t;
    const u32x4 w = level0(dk, i >> 4);
    out[t] = exact_j(dk, i, level0_byte(w, (uint32_t)(i & 15)));
}

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void merge_slots_kernel(const int64_t* __restrict__ idx_parts,
                                                             const KeyT* __restrict__ key_parts,
                                                             int32_t parts, int64_t part_len,
                                                             uint32_t k, int64_t* __restrict__ slot_idx,
                                                             KeyT* __restrict__ slot_key) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    int64_t best = slot_idx[j];
    KeyT key = slot_key[j];
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t idx = idx_parts[(int64_t)p * part_len + j];
        if (idx > best) {
            best = idx;
            key = key_parts[(int64_t)p * part_len + j];
        }
    }
    slot_idx[j] = best;
    slot_key[j] = key;
}

// packed multi-GPU row: [slot_idx(k) | keys widened to int64 (k)]
template <typename KeyT>
__global__ __launch_bounds__(kBlock) void export_packed_kernel(const int64_t* __restrict__ slot_idx,
                                                               const KeyT* __restrict__ slot_key, uint32_t k,
                                                               int64_t* __restrict__ row) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    row[j] = slot_idx[j];
    row[k + j] = (int64_t)slot_key[j];
}

template <typename KeyT>
__global__ __launch_bounds__(kBlock) void merge_packed_kernel(const int64_t* __restrict__ rows, int32_t parts,
                                                              int64_t stride, uint32_t k,
                                                              int64_t* __restrict__ slot_idx,
                                                              KeyT* __restrict__ slot_key) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    int64_t best = slot_idx[j];
    KeyT key = slot_key[j];
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t* r = rows + (int64_t)p * stride;
        const int64_t idx = r[j];
        if (idx > best) {
            best = idx;
            key = (KeyT)r[k + j];
        }
    }
    slot_idx[j] = best;
    slot_key[j] = key;
}

// merge of packed rows + publication in one dispatch (k <= 8192, Int/Long keys): the multi-GPU
// combine's last step before result(), as resolve_publish_kernel is for a batch
template <typename KeyT>
__global__ __launch_bounds__(1024) void merge_packed_publish_kernel(const int64_t* __restrict__ rows, int32_t parts,
                                                                    int64_t stride, uint32_t k,
                                                                    int64_t* __restrict__ slot_idx,
                                                                    KeyT* __restrict__ slot_key, int64_t m, KeyT* dst,
                                                                    uint32_t* flag, uint32_t gen) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        int64_t best = slot_idx[j];
        KeyT key = slot_key[j];
        bool moved = false;
        for (int32_t p = 0; p < parts; ++p) {
            const int64_t* r = rows + (int64_t)p * stride;
            const int64_t idx = r[j];
            if (idx > best) {
                best = idx;
                key = (KeyT)r[k + j];
                moved = true;
            }
        }
        if (moved) {
            slot_idx[j] = best;
            slot_key[j] = key;
        }
        if ((int64_t)j < m) dst[j] = key;
    }
    publish_flag(flag, gen);
}

// ---- fixed-width byte keys (key_width a multiple of 8 above 8: UUIDs, composite keys) ----------
// The element sampler never looks inside a key, so wide keys only change the copies: each slot's
// key is `words` 32-bit words, moved word by word.  Same slot logic as resolve_kernel /
// resolve_publish_kernel (one kernel; `dst` non-null = publish, launched as one workgroup).
__global__ __launch_bounds__(1024) void resolve_wide_kernel(const uint32_t* __restrict__ keys, int64_t base,
                                                            int64_t n, uint32_t k, uint32_t words,
                                                            unsigned long long* __restrict__ win,
                                                            uint32_t* __restrict__ slot_key,
                                                            int64_t* __restrict__ slot_idx, int fresh, int64_t m,
                                                            uint32_t* dst, uint32_t* flag, uint32_t gen) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride) {
        const unsigned long long wi = win[j];
        const uint32_t* src = nullptr;
        if (wi) {
            src = keys + (size_t)((int64_t)wi - base) * words;
            if (slot_idx) slot_idx[j] = (int64_t)wi;
            win[j] = 0;
        } else if ((int64_t)j >= base && (int64_t)j < base + n) {
            src = keys + (size_t)(j - base) * words;
            if (slot_idx) slot_idx[j] = j;
        } else if (fresh && slot_idx) {
            slot_idx[j] = -1;
        }
        uint32_t* o = slot_key + (size_t)j * words;
        const bool out = dst && (int64_t)j < m;
        for (uint32_t q = 0; q < words; ++q) {
            const uint32_t v = src ? src[q] : (fresh ? 0u : o[q]);
            if (src || fresh) o[q] = v;
            if (out) dst[(size_t)j * words + q] = v;
        }
    }
    if (dst) publish_flag(flag, gen);
}

__global__ __launch_bounds__(kBlock) void merge_slots_wide_kernel(const int64_t* __restrict__ idx_parts,
                                                                  const uint32_t* __restrict__ key_parts,
                                                                  int32_t parts, int64_t part_len, uint32_t k,
                                                                  uint32_t words, int64_t* __restrict__ slot_idx,
                                                                  uint32_t* __restrict__ slot_key) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    int64_t best = slot_idx[j];
    int32_t from = -1;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t idx = idx_parts[(int64_t)p * part_len + j];
        if (idx > best) {
            best = idx;
            from = p;
        }
    }
    if (from < 0) return;
    slot_idx[j] = best;
    const uint32_t* src = key_parts + ((size_t)from * part_len + j) * words;
    for (uint32_t q = 0; q < words; ++q) slot_key[(size_t)j * words + q] = src[q];
}

// packed rows of wide keys: [slot_idx(k) | k keys of `words` 32-bit words]
__global__ __launch_bounds__(kBlock) void export_packed_wide_kernel(const int64_t* __restrict__ slot_idx,
                                                                    const uint32_t* __restrict__ slot_key, uint32_t k,
                                                                    uint32_t words, int64_t* __restrict__ row) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    row[j] = slot_idx[j];
    uint32_t* o = (uint32_t*)(row + k) + (size_t)j * words;
    for (uint32_t q = 0; q < words; ++q) o[q] = slot_key[(size_t)j * words + q];
}

__global__ __launch_bounds__(kBlock) void merge_packed_wide_kernel(const int64_t* __restrict__ rows, int32_t parts,
                                                                   int64_t stride, uint32_t k, uint32_t words,
                                                                   int64_t* __restrict__ slot_idx,
                                                                   uint32_t* __restrict__ slot_key) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    int64_t best = slot_idx[j];
    int32_t from = -1;
    for (int32_t p = 0; p < parts; ++p) {
        const int64_t idx = rows[(int64_t)p * stride + j];
        if (idx > best) {
            best = idx;
            from = p;
        }
    }
    if (from < 0) return;
    slot_idx[j] = best;
    const uint32_t* src = (const uint32_t*)(rows + (int64_t)from * stride + k) + (size_t)j * words;
    for (uint32_t q = 0; q < words; ++q) slot_key[(size_t)j * words + q] = src[q];
}

inline DrawKey make_key(const DrawParams& dp) {
    return DrawKey{(uint32_t)dp.seed, (uint32_t)(dp.seed >> 32), (uint32_t)dp.stream,
                   (uint32_t)(dp.stream >> 32)};
}

inline unsigned grid_for(uint64_t items, unsigned cap) {
    uint64_t b = (items + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    return (unsigned)(b < cap ? b : cap);
}

// K1's grid: a wave's last window, when partial, takes the per-block path (clip and dense
// checks, ~30 more VALU per iteration); so the grid is sized for whole windows per wave --
// m windows, m nearest to what kK1Grid workgroups would run -- where the launch is large enough
// (1e9 draws: 5086 workgroups, 2 windows of 12 iterations per wave)
inline unsigned k1_grid(uint64_t n_groups) {
    constexpr uint64_t per_window = (uint64_t)kK1Unroll * kBlock * kK1Win;  // blocks per workgroup-window
    // below ~3 whole-window workgroups per CU, every CU gets work instead (partial windows)
    if (n_groups < per_window * 768) return grid_for((n_groups + kK1Unroll - 1) / kK1Unroll, kK1Grid);
    const uint64_t m = std::max<uint64_t>(1, (n_groups + per_window * kK1Grid / 2) / (per_window * kK1Grid));
    return (unsigned)std::max<uint64_t>(1, n_groups / (per_window * m));
}

// The two-group schedule (k1_body_q), for launches of >= 10 half windows per first-group wave: the
// first kK1W1 waves (one generation of resident waves: 6 four-wave workgroups per CU) take ~75 % of
// the half windows, the rest go two per wave.  tools/micro_k1o s, 1e9 draws (81 k half windows):
// (6144, 10, 2) 81.7-81.8 us, (5120, 12, 2) 81.7-82.5, (4096, 16, 1) 82.1-82.7, (6144, 8, 2)
// 82.9-83.2, (6144, 13, 1) 89.3 (a long first group outlasts the rest) vs 83.0-83.2 us grid-stride.
constexpr uint32_t kK1W1 = 256 * 6 * (kBlock / 64);
inline unsigned k1_plan(uint64_t n_groups, K1Sched& sch) {
    sch = K1Sched{0, 0, 0};
    constexpr uint64_t UB = (uint64_t)kK1Unroll * 64 * (kK1Win / 2);  // blocks per half window
    const uint64_t units = (n_groups + UB - 1) / UB;
    const uint64_t A = (units * 755 / 1000 + kK1W1 / 2) / kK1W1;
    // from ~1e9 draws (A >= 10); below, the plan lost to the grid-stride launch (micro_k1o n: 4.5e8
    // 48.2 vs 44.7 us, 6e8 58.2 vs 55.7; 1e9 81.7 vs 82.8, 2e9 157.5 vs 158.8, 8e9 610.5 vs 616.9)
    if (n_groups < (uint64_t)kK1Unroll * kBlock * kK1Win * 768 || A < 10) return k1_grid(n_groups);
    sch.W1 = kK1W1;
    sch.A = (uint32_t)A;
    sch.B = 2;
    const uint64_t rest = units - (uint64_t)kK1W1 * A;  // > 0: A ~ 0.755 units / W1
    const uint64_t waves = kK1W1 + (rest + sch.B - 1) / sch.B;
    return (unsigned)((waves + kBlock / 64 - 1) / (kBlock / 64));
}

}  // namespace

hipError_t launch_k1_last_writer(const DrawParams& dp, uint32_t k, uint64_t lo, uint64_t hi,
                                 unsigned long long* batch_win, hipStream_t st) {
    if (hi <= lo) return hipSuccess;
    const uint64_t g_end = (hi + 15) >> 4;
    constexpr uint64_t kMaxGroups = 1ull << 31;  // block offsets are 32-bit queue entries
    uint64_t n_groups = 0;
    for (uint64_t g_begin = lo >> 4; g_begin < g_end; g_begin += n_groups) {
        // and no launch crosses a multiple of 2^32 blocks: the counter's high word is a scalar
        const uint64_t g_wrap = ((g_begin >> 32) + 1) << 32;
        n_groups = std::min<uint64_t>(std::min<uint64_t>(g_end, g_wrap) - g_begin, kMaxGroups);
        K1Sched sch;
        const unsigned grid = k1_plan(n_groups, sch);
        hipLaunchKernelGGL(k1_last_writer, dim3(grid), dim3(kBlock), 0, st, make_key(dp), k, lo, hi,
                           g_begin, n_groups, batch_win, sch);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

bool k1_fused_ok(uint64_t lo, uint64_t hi, uint32_t k, int key_width) {
    if (hi <= lo || k > kK1FusedMaxK || (key_width != 8 && key_width != 4)) return false;
    const uint64_t g_begin = lo >> 4, g_end = (hi + 15) >> 4;
    // one launch of launch_k1_last_writer: no 2^32-block crossing, fewer than 2^31 blocks
    return g_end - g_begin <= (1ull << 31) && g_end <= ((g_begin >> 32) + 1) << 32;
}

hipError_t launch_k1_resolve_publish(const DrawParams& dp, uint32_t k, uint64_t lo, uint64_t hi,
                                     unsigned long long* batch_win, uint32_t* ticket, const void* keys,
                                     int key_width, int64_t base, int64_t n, void* slot_key, int64_t* slot_idx,
                                     bool fresh, int64_t m, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen,
                                     hipStream_t st) {
    if (!k1_fused_ok(lo, hi, k, key_width)) return hipErrorInvalidValue;
    const uint64_t g_begin = lo >> 4, n_groups = ((hi + 15) >> 4) - g_begin;
    K1Sched sch;
    const unsigned grid = k1_plan(n_groups, sch);
    if (key_width == 8)
        hipLaunchKernelGGL(k1_resolve_publish<int64_t>, dim3(grid), dim3(kBlock), 0, st, make_key(dp), k, lo, hi,
                           g_begin, n_groups, batch_win, ticket, (const int64_t*)keys, base, n, (int64_t*)slot_key,
                           slot_idx, (int)fresh, m, (int64_t*)dst_host_dev, flag_dev, gen, sch);
    else
        hipLaunchKernelGGL(k1_resolve_publish<int32_t>, dim3(grid), dim3(kBlock), 0, st, make_key(dp), k, lo, hi,
                           g_begin, n_groups, batch_win, ticket, (const int32_t*)keys, base, n, (int32_t*)slot_key,
                           slot_idx, (int)fresh, m, (int32_t*)dst_host_dev, flag_dev, gen, sch);
    return hipGetLastError();
}

hipError_t launch_resolve(const void* keys, int key_width, int64_t base, int64_t n, uint32_t k,
                          unsigned long long* batch_win, void* slot_key, int64_t* slot_idx, bool fresh,
                          hipStream_t st) {
    const unsigned grid = (unsigned)((k + kBlock - 1) / kBlock);
    if (key_width > 8) {
        hipLaunchKernelGGL(resolve_wide_kernel, dim3(std::min<unsigned>(grid, 256 * 64)), dim3(kBlock), 0, st,
                           (const uint32_t*)keys, base, n, k, (uint32_t)key_width / 4, batch_win, (uint32_t*)slot_key,
                           slot_idx, (int)fresh, (int64_t)0, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u);
        return hipGetLastError();
    }
    if (key_width == 8)
        hipLaunchKernelGGL(resolve_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, st,
                           (const int64_t*)keys, base, n, k, batch_win, (int64_t*)slot_key, slot_idx, (int)fresh);
    else
        hipLaunchKernelGGL(resolve_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, st,
                           (const int32_t*)keys, base, n, k, batch_win, (int32_t*)slot_key, slot_idx, (int)fresh);
    return hipGetLastError();
}

// fresh handle: batch_win = 0, slot_idx = -1 (empty), slot_key = 0
__global__ __launch_bounds__(kBlock) void init_slots_kernel(uint8_t* slot_key, int key_width, int64_t* slot_idx,
                                                            unsigned long long* win, uint32_t k, uint32_t* ticket) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if (ticket && blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride) {
        win[j] = 0;
        slot_idx[j] = -1;
        if (key_width == 8)
            ((int64_t*)slot_key)[j] = 0;
        else if (key_width == 4)
            ((int32_t*)slot_key)[j] = 0;
        else
            for (int q = 0; q < key_width / 4; ++q) ((uint32_t*)slot_key)[(size_t)j * (key_width / 4) + q] = 0;
    }
}

hipError_t launch_init_slots(void* slot_key, int key_width, int64_t* slot_idx, unsigned long long* win, uint32_t k,
                             hipStream_t st, uint32_t* ticket) {
    const unsigned grid = (unsigned)std::min<uint64_t>((k + kBlock - 1) / kBlock, 256 * 64);
    hipLaunchKernelGGL(init_slots_kernel, dim3(grid), dim3(kBlock), 0, st, (uint8_t*)slot_key, key_width, slot_idx,
                       win, k, ticket);
    return hipGetLastError();
}

// result() tail: copy the k-slot reservoir straight into coherent pinned host memory, then publish
// `gen` in the host flag with a system-scope release.  The host spins on the flag: ~7 us less
// than hipMemcpyAsync D2H + hipStreamSynchronize for an 8 KB reservoir (tools/probe_latency.hip).
__global__ __launch_bounds__(1024) void publish_kernel(const uint32_t* __restrict__ src, uint32_t* dst,
                                                      int64_t words, uint32_t* flag, uint32_t gen) {
    // 16-B stores: a quarter of the PCIe write transactions of 4-B ones (both ends 16-B aligned)
    const int64_t vecs = words >> 2;
    for (int64_t i = threadIdx.x; i < vecs; i += blockDim.x)
        ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (int64_t i = (vecs << 2) + threadIdx.x; i < words; i += blockDim.x) dst[i] = src[i];
    publish_flag(flag, gen);
}

// Publication of a large buffer (a distinct set: up to 512 KB at k = 65536) by several workgroups:
// one workgroup's posted PCIe writes run at ~20 GB/s.  Each workgroup releases its stores at system
// scope and takes a ticket; the last one stores the flag (and re-arms the ticket).
__global__ __launch_bounds__(1024) void publish_multi_kernel(const uint32_t* __restrict__ src, uint32_t* dst,
                                                            int64_t words, uint32_t* flag, uint32_t gen,
                                                            uint32_t* ticket) {
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

hipError_t launch_publish_multi(const void* src, int64_t bytes, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen,
                                uint32_t* ticket_dev, hipStream_t st) {
    const int64_t per = 32 * 1024;  // bytes per workgroup
    const unsigned grid = (unsigned)std::min<int64_t>(32, std::max<int64_t>(1, (bytes + per - 1) / per));
    hipLaunchKernelGGL(publish_multi_kernel, dim3(grid), dim3(1024), 0, st, (const uint32_t*)src,
                       (uint32_t*)dst_host_dev, bytes / 4, flag_dev, gen, ticket_dev);
    return hipGetLastError();
}

hipError_t launch_publish(const void* src, int64_t bytes, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen,
                          hipStream_t st) {
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(1024), 0, st, (const uint32_t*)src, (uint32_t*)dst_host_dev,
                       bytes / 4, flag_dev, gen);
    return hipGetLastError();
}

hipError_t launch_resolve_publish(const void* keys, int key_width, int64_t base, int64_t n, uint32_t k,
                                  unsigned long long* batch_win, void* slot_key, int64_t* slot_idx, bool fresh,
                                  int64_t m, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st,
                                  bool small) {
    if (small && k <= 8 * kBlock && (key_width == 8 || key_width == 4)) {
#define RSV_SMALL(T, R)                                                                                              \
    hipLaunchKernelGGL((resolve_publish_small_kernel<T, R>), dim3(1), dim3(kBlock), 0, st, (const T*)keys, base, n, \
                       k, batch_win, (T*)slot_key, slot_idx, (int)fresh, m, (T*)dst_host_dev, flag_dev, gen)
        if (key_width == 8) {
            if (k <= 2 * kBlock) RSV_SMALL(int64_t, 2);
            else if (k <= 4 * kBlock) RSV_SMALL(int64_t, 4);
            else RSV_SMALL(int64_t, 8);
        } else {
            if (k <= 2 * kBlock) RSV_SMALL(int32_t, 2);
            else if (k <= 4 * kBlock) RSV_SMALL(int32_t, 4);
            else RSV_SMALL(int32_t, 8);
        }
#undef RSV_SMALL
        return hipGetLastError();
    }
    const unsigned threads = std::min<unsigned>(1024, std::max<unsigned>(64, (k + 63) / 64 * 64));
    if (key_width > 8) {
        hipLaunchKernelGGL(resolve_wide_kernel, dim3(1), dim3(threads), 0, st, (const uint32_t*)keys, base, n, k,
                           (uint32_t)key_width / 4, batch_win, (uint32_t*)slot_key, slot_idx, (int)fresh, m,
                           (uint32_t*)dst_host_dev, flag_dev, gen);
        return hipGetLastError();
    }
    if (key_width == 8)
        hipLaunchKernelGGL(resolve_publish_kernel<int64_t>, dim3(1), dim3(threads), 0, st, (const int64_t*)keys, base,
                           n, k, batch_win, (int64_t*)slot_key, slot_idx, (int)fresh, m, (int64_t*)dst_host_dev,
                           flag_dev, gen);
    else
        hipLaunchKernelGGL(resolve_publish_kernel<int32_t>, dim3(1), dim3(threads), 0, st, (const int32_t*)keys, base,
                           n, k, batch_win, (int32_t*)slot_key, slot_idx, (int)fresh, m, (int32_t*)dst_host_dev,
                           flag_dev, gen);
    return hipGetLastError();
}

// ---- index-only batches (rsv_sample_indexed / rsv_fill_slots) -------------------------------
// The resolve of a batch sampled by index alone: per slot j the batch's last writer (win[j]), else
// the fill of j < k from this batch, becomes slot_idx[j], and offs[j] = its offset in the batch
// (-1: the slot did not change).  The keys arrive later from the caller (fill_slots_kernel).
__global__ __launch_bounds__(kBlock) void resolve_indices_kernel(int64_t base, int64_t n, uint32_t k,
                                                                 unsigned long long* __restrict__ win,
                                                                 int64_t* __restrict__ slot_idx, int fresh,
                                                                 uint8_t* __restrict__ slot_key, int key_width,
                                                                 int64_t* __restrict__ offs) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride) {
        const unsigned long long wi = win[j];
        int64_t off = -1;
        if (wi) {  // last eviction into slot j (Sampler.scala:243-246)
            slot_idx[j] = (int64_t)wi;
            win[j] = 0;
            off = (int64_t)wi - base;
        } else if ((int64_t)j >= base && (int64_t)j < base + n) {  // fill phase (Sampler.scala:253-255)
            slot_idx[j] = (int64_t)j;
            off = (int64_t)j - base;
        } else if (fresh) {
            slot_idx[j] = -1;
            for (int q = 0; q < key_width; ++q) slot_key[j * key_width + q] = 0;
        }
        offs[j] = off;
    }
}

// keys[j] (host-supplied, one per slot, slot order) into every slot the index-only batch changed
__global__ __launch_bounds__(kBlock) void fill_slots_kernel(const int64_t* __restrict__ offs, const uint8_t* __restrict__ keys,
                                                            uint32_t k, int key_width, uint8_t* __restrict__ slot_key) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride) {
        if (offs[j] < 0) continue;
        if (key_width == 8) ((int64_t*)slot_key)[j] = ((const int64_t*)keys)[j];
        else if (key_width == 4) ((int32_t*)slot_key)[j] = ((const int32_t*)keys)[j];
        else
            for (int q = 0; q < key_width; ++q) slot_key[j * key_width + q] = keys[j * key_width + q];
    }
}

// resolve_indices_kernel + publication of offs[] into coherent host memory (flag = gen) in one
// dispatch, for k <= kIdxPublishMaxK: the host spins on the flag instead of a D2H copy + stream
// synchronize (the winners-only host batches and rsv_sample_indexed)
constexpr uint32_t kIdxPublishMaxK = 8192;

__global__ __launch_bounds__(1024) void resolve_indices_publish_kernel(int64_t base, int64_t n, uint32_t k,
                                                                       unsigned long long* __restrict__ win,
                                                                       int64_t* __restrict__ slot_idx, int fresh,
                                                                       uint8_t* __restrict__ slot_key, int key_width,
                                                                       int64_t* __restrict__ offs, int64_t* offs_host,
                                                                       uint32_t* flag, uint32_t gen) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        const unsigned long long wi = win[j];
        int64_t off = -1;
        if (wi) {
            slot_idx[j] = (int64_t)wi;
            win[j] = 0;
            off = (int64_t)wi - base;
        } else if ((int64_t)j >= base && (int64_t)j < base + n) {
            slot_idx[j] = (int64_t)j;
            off = (int64_t)j - base;
        } else if (fresh) {
            slot_idx[j] = -1;
            for (int q = 0; q < key_width; ++q) slot_key[(size_t)j * key_width + q] = 0;
        }
        offs[j] = off;
        offs_host[j] = off;
    }
    publish_flag(flag, gen);
}

// fill_slots_kernel + publication of the first m slot keys (resolve_publish's form) for k <= 8192
// and 4- / 8-byte keys: the host-keyed batch's reservoir is published with its last kernel
template <typename KeyT>
__global__ __launch_bounds__(1024) void fill_slots_publish_kernel(const int64_t* __restrict__ offs,
                                                                  const KeyT* __restrict__ keys, uint32_t k,
                                                                  KeyT* __restrict__ slot_key, int64_t m, KeyT* dst,
                                                                  uint32_t* flag, uint32_t gen) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        KeyT v;
        if (offs[j] >= 0) {
            v = keys[j];
            slot_key[j] = v;
        } else {
            v = slot_key[j];
        }
        if ((int64_t)j < m) dst[j] = v;
    }
    publish_flag(flag, gen);
}

bool resolve_indices_publish_ok(uint32_t k) { return k <= kIdxPublishMaxK; }

hipError_t launch_resolve_indices_publish(int64_t base, int64_t n, uint32_t k, unsigned long long* batch_win,
                                          int64_t* slot_idx, bool fresh, void* slot_key, int key_width, int64_t* offs,
                                          int64_t* offs_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st) {
    if (k > kIdxPublishMaxK) return hipErrorInvalidValue;
    const unsigned threads = std::min<unsigned>(1024, std::max<unsigned>(64, (k + 63) / 64 * 64));
    hipLaunchKernelGGL(resolve_indices_publish_kernel, dim3(1), dim3(threads), 0, st, base, n, k, batch_win, slot_idx,
                       (int)fresh, (uint8_t*)slot_key, key_width, offs, offs_host_dev, flag_dev, gen);
    return hipGetLastError();
}

bool fill_slots_publish_ok(uint32_t k, int key_width) {
    return k <= kIdxPublishMaxK && (key_width == 4 || key_width == 8);
}

hipError_t launch_fill_slots_publish(const int64_t* offs, const void* keys, uint32_t k, int key_width, void* slot_key,
                                     int64_t m, void* dst_host_dev, uint32_t* flag_dev, uint32_t gen, hipStream_t st) {
    if (!fill_slots_publish_ok(k, key_width)) return hipErrorInvalidValue;
    const unsigned threads = std::min<unsigned>(1024, std::max<unsigned>(64, (k + 63) / 64 * 64));
    if (key_width == 8)
        hipLaunchKernelGGL(fill_slots_publish_kernel<int64_t>, dim3(1), dim3(threads), 0, st, offs,
                           (const int64_t*)keys, k, (int64_t*)slot_key, m, (int64_t*)dst_host_dev, flag_dev, gen);
    else
        hipLaunchKernelGGL(fill_slots_publish_kernel<int32_t>, dim3(1), dim3(threads), 0, st, offs,
                           (const int32_t*)keys, k, (int32_t*)slot_key, m, (int32_t*)dst_host_dev, flag_dev, gen);
    return hipGetLastError();
}

hipError_t launch_resolve_indices(int64_t base, int64_t n, uint32_t k, unsigned long long* batch_win, int64_t* slot_idx,
                                  bool fresh, void* slot_key, int key_width, int64_t* offs, hipStream_t st) {
    hipLaunchKernelGGL(resolve_indices_kernel, dim3(grid_for(k, 256 * 64)), dim3(kBlock), 0, st, base, n, k, batch_win,
                       slot_idx, (int)fresh, (uint8_t*)slot_key, key_width, offs);
    return hipGetLastError();
}

hipError_t launch_fill_slots(const int64_t* offs, const void* keys, uint32_t k, int key_width, void* slot_key,
                             hipStream_t st) {
    hipLaunchKernelGGL(fill_slots_kernel, dim3(grid_for(k, 256 * 64)), dim3(kBlock), 0, st, offs, (const uint8_t*)keys,
                       k, key_width, (uint8_t*)slot_key);
    return hipGetLastError();
}

hipError_t launch_replay_events(const int64_t* ev_pos, const int32_t* ev_slot, int64_t n_events,
                                uint32_t k, unsigned long long* batch_win, hipStream_t st) {
    if (n_events <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((n_events + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(replay_kernel, dim3(grid), dim3(kBlock), 0, st, ev_pos, ev_slot, n_events, k,
                       batch_win);
    return hipGetLastError();
}

hipError_t launch_export_draws(const DrawParams& dp, uint64_t i0, int64_t n, uint64_t* j,
                               hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(export_draws_kernel, dim3(grid), dim3(kBlock), 0, st, make_key(dp), i0, n, j);
    return hipGetLastError();
}

hipError_t launch_merge_slots(const int64_t* idx_parts, const void* key_parts, int key_width,
                              int32_t parts, int64_t part_len, uint32_t k, int64_t* slot_idx,
                              void* slot_key, hipStream_t st) {
    const unsigned grid = (unsigned)((k + kBlock - 1) / kBlock);
    if (key_width > 8) {
        hipLaunchKernelGGL(merge_slots_wide_kernel, dim3(grid), dim3(kBlock), 0, st, idx_parts,
                           (const uint32_t*)key_parts, parts, part_len, k, (uint32_t)key_width / 4, slot_idx,
                           (uint32_t*)slot_key);
        return hipGetLastError();
    }
    if (key_width == 8)
        hipLaunchKernelGGL(merge_slots_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, st, idx_parts,
                           (const int64_t*)key_parts, parts, part_len, k, slot_idx, (int64_t*)slot_key);
    else
        hipLaunchKernelGGL(merge_slots_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, st, idx_parts,
                           (const int32_t*)key_parts, parts, part_len, k, slot_idx, (int32_t*)slot_key);
    return hipGetLastError();
}

hipError_t launch_export_packed(const int64_t* slot_idx, const void* slot_key, int key_width, uint32_t k,
                                int64_t* row, hipStream_t st) {
    const unsigned grid = (unsigned)((k + kBlock - 1) / kBlock);
    if (key_width > 8) {
        hipLaunchKernelGGL(export_packed_wide_kernel, dim3(grid), dim3(kBlock), 0, st, slot_idx,
                           (const uint32_t*)slot_key, k, (uint32_t)key_width / 4, row);
        return hipGetLastError();
    }
    if (key_width == 8)
        hipLaunchKernelGGL(export_packed_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, st, slot_idx,
                           (const int64_t*)slot_key, k, row);
    else
        hipLaunchKernelGGL(export_packed_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, st, slot_idx,
                           (const int32_t*)slot_key, k, row);
    return hipGetLastError();
}

hipError_t launch_merge_packed(const int64_t* rows, int32_t parts, int64_t stride, uint32_t k, int64_t* slot_idx,
                               void* slot_key, int key_width, hipStream_t st) {
    const unsigned grid = (unsigned)((k + kBlock - 1) / kBlock);
    if (key_width > 8) {
        hipLaunchKernelGGL(merge_packed_wide_kernel, dim3(grid), dim3(kBlock), 0, st, rows, parts, stride, k,
                           (uint32_t)key_width / 4, slot_idx, (uint32_t*)slot_key);
        return hipGetLastError();
    }
    if (key_width == 8)
        hipLaunchKernelGGL(merge_packed_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, st, rows, parts, stride, k,
                           slot_idx, (int64_t*)slot_key);
    else
        hipLaunchKernelGGL(merge_packed_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, st, rows, parts, stride, k,
                           slot_idx, (int32_t*)slot_key);
    return hipGetLastError();
}

hipError_t launch_merge_packed_publish(const int64_t* rows, int32_t parts, int64_t stride, uint32_t k,
                                       int64_t* slot_idx, void* slot_key, int key_width, int64_t m, void* dst_host_dev,
                                       uint32_t* flag_dev, uint32_t gen, hipStream_t st) {
    const unsigned threads = std::min<unsigned>(1024, std::max<unsigned>(64, (k + 63) / 64 * 64));
    if (key_width == 8)
        hipLaunchKernelGGL(merge_packed_publish_kernel<int64_t>, dim3(1), dim3(threads), 0, st, rows, parts, stride, k,
                           slot_idx, (int64_t*)slot_key, m, (int64_t*)dst_host_dev, flag_dev, gen);
    else
        hipLaunchKernelGGL(merge_packed_publish_kernel<int32_t>, dim3(1), dim3(threads), 0, st, rows, parts, stride, k,
                           slot_idx, (int32_t*)slot_key, m, (int32_t*)dst_host_dev, flag_dev, gen);
    return hipGetLastError();
}

}  // namespace rsv
