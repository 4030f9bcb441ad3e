// rsv_k2.h -- the K2 segmented kernel (rsv_segmented.hip launches it).  See rsv_segmented.hip for
// the design.  (The cost-probe variants of earlier rounds live in tools/k2_dev_variants.h.)
#pragma once
#include <algorithm>
#include <type_traits>

#include "rsv_device.h"

namespace rsv {
namespace k2 {

constexpr int kWaves = 4;          // waves per workgroup
constexpr uint32_t kRing = 4;      // level-0 iterations whose block words stay addressable
constexpr uint32_t kQCap = 512;    // FIFO entries (an iteration that would overflow takes ballot rounds)
constexpr uint32_t kStashBytes = kRing * 64 * 16;
constexpr uint32_t kQueueBytes = kQCap * 2;
constexpr uint32_t kLut = 1024;    // blocks (16 indices each) whose threshold T is tabulated per workgroup
constexpr uint32_t kLutBytes = kLut * 2;
constexpr int64_t kSmallLen = 1ll << 27;  // streams shorter than this use 32-bit index arithmetic

// bytes of dynamic LDS per workgroup: T table + per wave (stash | FIFO | k-slot table)
__host__ __device__ inline size_t lds_bytes(uint32_t k) {
    return kLutBytes + (size_t)kWaves * (kStashBytes + kQueueBytes + (size_t)k * 8);
}

constexpr size_t kLdsMax = 160 * 1024;  // one workgroup's LDS

// T = ceil(256 k / (i0 + 1)), the block threshold of the dense region (T > 255: every byte is a
// candidate -> 256); 0 marks the sparse region (i0 + 1 >= 256 k: only b == 0 can hit)
__device__ __forceinline__ uint32_t block_threshold(uint64_t i0, uint64_t dense_lim) {
    if (i0 + 1 >= dense_lim) return 0;
    const uint64_t T = (dense_lim + i0) / (i0 + 1);
    return T > 255 ? 256u : (uint32_t)T;
}

// b_e < T for the 16 bytes of a block (1 <= T <= 255), bit-sliced: the borrow out of (T - 1) - b,
// planes LSB first, one v_bitop3 per plane (borrow' = bit p of T-1 ? plane & borrow : plane | borrow;
// table 0xD4 in the A = 0xF0, B = 0xCC, C = 0xAA convention).  The high 16 bits are don't-care.
__device__ __forceinline__ uint32_t lt_mask16_borrow(const u32x4& w, uint32_t T) {
    const uint32_t M = T - 1;
    const uint32_t words[4] = {w.x, w.y, w.z, w.w};
    uint32_t br = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const uint32_t plane = (p & 1) ? (words[p >> 1] >> 16) : words[p >> 1];
        const uint32_t mm = (uint32_t)((int32_t)(M << (31 - p)) >> 31);  // all ones iff bit p of T-1
        br = __builtin_amdgcn_bitop3_b32(plane, br, mm, 0xD4);
    }
    return ~br & 0xFFFFu;
}

// the level-0 bytes of indices e and e + 1 of a block (e even), as level0_byte twice
__device__ __forceinline__ void level0_byte_pair(const u32x4& w, uint32_t e, uint32_t& b0, uint32_t& b1) {
    // bits e, e+1 of the planes 2q (low half) and 2q+1 (high half) of word q, at 2q, 2q+1 / 16+2q, 17+2q
    const uint32_t u = ((w.x >> e) & 0x30003u) | (((w.y >> e) & 0x30003u) << 2) |
                       (((w.z >> e) & 0x30003u) << 4) | (((w.w >> e) & 0x30003u) << 6);
    b0 = (u & 0x55u) | ((u >> 15) & 0xAAu);
    b1 = ((u >> 1) & 0x55u) | ((u >> 16) & 0xAAu);
}

__device__ __forceinline__ uint32_t mask_for(const u32x4& w, uint32_t T) {
    return T == 0 ? zero_byte_mask16(w) : T > 255 ? 0xFFFFu : lt_mask16_borrow(w, T);
}

// mask_for for T <= 16 (T = 0, the sparse region's b == 0, is T = 1): b < T needs planes 4..7 zero
// (the high words' OR) and the low four planes below T -- 4 borrow steps instead of 8
__device__ __forceinline__ uint32_t mask_for_small(const u32x4& w, uint32_t T) {
    const uint32_t M = (T ? T : 1u) - 1u;
    const uint32_t words[2] = {w.x, w.y};
    uint32_t br = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t plane = (p & 1) ? (words[p >> 1] >> 16) : words[p >> 1];
        const uint32_t mm = (uint32_t)((int32_t)(M << (31 - p)) >> 31);
        br = __builtin_amdgcn_bitop3_b32(plane, br, mm, 0xD4);
    }
    const uint32_t hi = w.z | w.w;
    return ~(br | hi | (hi >> 16)) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t clip16(uint64_t i0, uint64_t lo, uint64_t hi) {
    uint32_t m = 0xFFFFu;
    if (i0 < lo) m = (lo - i0 >= 16) ? 0u : ((0xFFFFu << (uint32_t)(lo - i0)) & 0xFFFFu);
    if (i0 + 16 > hi) m &= (hi <= i0) ? 0u : (0xFFFFu >> (uint32_t)(16 - (hi - i0)));
    return m;
}

// inclusive prefix sum over the wave (DPP: row shifts within 16-lane rows, then row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

// j = floor(((b << 56) | (L >> 8)) (i + 1) / 2^64), L = Lh:Ll
__device__ __forceinline__ uint64_t draw_j(uint32_t b, uint32_t Lh, uint32_t Ll, uint64_t i1, bool small) {
    const uint32_t Uh = __builtin_amdgcn_alignbit(b, Lh, 8), Ul = __builtin_amdgcn_alignbit(Lh, Ll, 8);
    if (small) {  // i + 1 < 2^32: a 64 x 32 product, the high word of its high half
        const uint32_t x = (uint32_t)i1;
        return (uint32_t)(((uint64_t)Uh * x + __umulhi(Ul, x)) >> 32);
    }
    return __umul64hi(((uint64_t)Uh << 32) | Ul, i1);
}

struct Wave {
    u32x4* stash;
    uint16_t* q;
    void* tab;
    const uint16_t* lut;
    uint32_t lane, k, k0, k1;
    uint64_t dense_lim;
    uint32_t fifo_cap;  // bulk appends while pending + new <= fifo_cap (<= the FIFO size; tests lower it)
};

// One stream on one wave.  SMALL: n < 2^27 -- 32-bit indices, u32 winner table, and Philox counters
// whose high words are wave-uniform (level 0: g < 2^32; level 1: i/2 < 2^32).
// DEFER (k <= 64): the lane's winner index is returned (-1: none) and the caller gathers its key
// after storing the previous stream's, so the random gather's latency overlaps the next stream's draws.
// (k >= kWGMinK takes the workgroup form below, k2_segmented_wg.)
template <typename KeyT, bool SMALL, bool DEFER>
__device__ __forceinline__ int64_t k2_stream(const Wave& W, const KeyT* __restrict__ keys, int64_t off, int64_t len,
                                             uint64_t stream, KeyT* __restrict__ o) {
    using IdxT = typename std::conditional<SMALL, uint32_t, uint64_t>::type;
    constexpr uint32_t QC = kQCap, RG = kRing, WIN = RG * 1024;  // WIN: indices in the ring
    const uint32_t lane = W.lane, k = W.k;
    IdxT* tab = (IdxT*)W.tab;
    for (uint32_t j = lane; j < k; j += 64) tab[j] = 0;
    const uint32_t s0 = (uint32_t)stream, s1 = (uint32_t)(stream >> 32);
    const DrawKey dk{W.k0, W.k1, s0, s1};
    const IdxT n_groups = (IdxT)(((uint64_t)len + 15) >> 4);
    uint32_t head = 0, tail = 0;  // FIFO positions (wave-uniform, wrap mod 2^32)
    // iterations start at a multiple of 64 blocks (the blocks below k >> 4 are clipped: fill), so
    // block g sits in stash slot g mod 256 (ring = (g / 64) mod 4) and a FIFO entry is i mod 4096
    IdxT gb = (IdxT)((k >> 4) & ~63u);
    uint32_t ring = (k >> 10) & (RG - 1);

    // resolve FIFO entries [head, head + nvalid) (nvalid <= 64), one per lane; last_gb = the most
    // recently stashed iteration: every pending index lies in [16 (last_gb - 192), + 4096)
    auto resolve_round = [&](uint32_t nvalid, IdxT last_gb) {
        __builtin_amdgcn_wave_barrier();
        const bool valid = lane < nvalid;
        const uint32_t ent = valid ? W.q[(head + lane) & (QC - 1)] : 0u;
        const uint32_t e = ent & 15u;
        const u32x4 w = W.stash[ent >> 4];  // block g mod 256
        const IdxT wlo = (last_gb << 4) - (IdxT)(WIN - 1024);
        const IdxT i = wlo + (IdxT)((ent - (uint32_t)wlo) & (WIN - 1));
        const uint32_t b = level0_byte(w, e);
        const IdxT g1 = i >> 1;
        u32x4 w1;
        if constexpr (SMALL) w1 = philox4x32_10_uniform_hi((uint32_t)g1, kDomainLevel1, s0, s1, W.k0, W.k1);
        else w1 = philox4x32_10((uint32_t)g1, (uint32_t)((uint64_t)g1 >> 32) | kDomainLevel1, s0, s1, W.k0, W.k1);
        // all four words, then one select per half (else the compiler selects the last round's
        // operands instead: 7 v_cndmask for the one saved product)
        asm volatile("" : "+v"(w1.x), "+v"(w1.y), "+v"(w1.z), "+v"(w1.w));
        const bool odd = (i & 1) != 0;
        const uint64_t j = draw_j(b, odd ? w1.z : w1.x, odd ? w1.w : w1.y, (uint64_t)i + 1, SMALL);
        if (valid && j < k) atomicMax(&tab[(uint32_t)j], i);
        head += nvalid;
        __builtin_amdgcn_wave_barrier();
    };

    // The dense head [k, hend), hend = min(len, HM k): candidate density >= 256 / HM %, so it skips
    // the FIFO -- each lane takes a PAIR of indices (one level-1 Philox serves both) straight from
    // the stashed level-0 block; the FIFO path covers [hend, len).
    // The head is cut to whole 64-pair rounds (k = 64: [64, 192) instead of [64, 256): its 96 pairs
    // took two rounds, the second half empty; the 64 indices moved to the FIFO add ~20 candidates
    // to rounds it runs anyway): C3 1.75-1.76 -> 1.67-1.69 ms (tools/micro_k2 r, warm clock).
    constexpr uint32_t HM = 4;
    uint64_t hx = (uint64_t)HM * k;
    // (only where the head holds at least one whole round: below k = 43 the cut would remove it and
    // send the 25-100 % dense region through the FIFO)
    if (hx - k >= 128) hx = k + ((hx - k) & ~(uint64_t)127);
    const IdxT hend = (IdxT)std::min<uint64_t>((uint64_t)len, hx);
    const IdxT flo = std::max<IdxT>((IdxT)k, hend);
    for (; gb < n_groups; gb += 64, ring = (ring + 1) & (RG - 1)) {
        // the oldest pending candidate still refers to the ring slot about to be overwritten
        if (tail != head && ((uint32_t)__builtin_amdgcn_readfirstlane((int)W.q[head & (QC - 1)]) >> 10) == ring) {
            while (tail != head) resolve_round(std::min<uint32_t>(64u, tail - head), gb - 64);
        }
        const IdxT g = gb + lane;
        const bool valid = g < n_groups;
        u32x4 w;
        if constexpr (SMALL) w = philox4x32_10_uniform_hi((uint32_t)g, 0u, s0, s1, W.k0, W.k1);
        else w = level0(dk, (uint64_t)g);
        const uint64_t i0 = (uint64_t)g << 4;
        const uint32_t T = g < kLut ? (uint32_t)W.lut[(uint32_t)g] : block_threshold(i0, W.dense_lim);
        // T falls with the block index, so lane 0's (block gb) bounds the iteration's: past the first
        // blocks of a stream every lane has T <= 16 (C3: iterations 1..3) and takes the short compare
        const uint32_t Tmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)T);
        uint32_t mask = valid ? (Tmax <= 16u ? mask_for_small(w, T) : mask_for(w, T)) : 0u;
        bool clip;  // wave-uniform; 32-bit compares for SMALL (scalar: no 64-bit s_cmp_lt)
        if constexpr (SMALL) clip = ((uint32_t)gb << 4) < (uint32_t)flo || (((uint32_t)gb + 64) << 4) > (uint32_t)len;
        else clip = ((uint64_t)gb << 4) < (uint64_t)flo || (((uint64_t)gb + 64) << 4) > (uint64_t)len;
        if (clip) mask &= clip16(i0, (uint64_t)flo, (uint64_t)len);
        W.stash[ring * 64 + lane] = w;
        if (((uint64_t)gb << 4) < (uint64_t)hend) {  // this iteration holds head indices (uniform)
            __builtin_amdgcn_wave_barrier();
            const IdxT ia = std::max<IdxT>((IdxT)k & ~(IdxT)1, gb << 4);
            const IdxT ib = std::min<IdxT>(hend, (gb + 64) << 4);
            for (IdxT p0 = ia; p0 < ib; p0 += 128) {
                const IdxT i = p0 + 2 * lane;  // even
                const u32x4 wl = W.stash[(uint32_t)(i >> 4) & (RG * 64 - 1)];
                uint32_t b0, b1;
                level0_byte_pair(wl, (uint32_t)i & 15u, b0, b1);
                const IdxT g1 = i >> 1;
                u32x4 w1;
                if constexpr (SMALL) w1 = philox4x32_10_uniform_hi((uint32_t)g1, kDomainLevel1, s0, s1, W.k0, W.k1);
                else w1 = philox4x32_10((uint32_t)g1, (uint32_t)((uint64_t)g1 >> 32) | kDomainLevel1, s0, s1, W.k0, W.k1);
                asm volatile("" : "+v"(w1.x), "+v"(w1.y), "+v"(w1.z), "+v"(w1.w));
                const uint64_t j0 = draw_j(b0, w1.x, w1.y, (uint64_t)i + 1, SMALL);
                const uint64_t j1 = draw_j(b1, w1.z, w1.w, (uint64_t)i + 2, SMALL);
                if (i < ib && i >= (IdxT)k && j0 < k) atomicMax(&tab[(uint32_t)j0], i);
                if (i + 1 < ib && i + 1 >= (IdxT)k && j1 < k) atomicMax(&tab[(uint32_t)j1], i + 1);
            }
            __builtin_amdgcn_wave_barrier();
        }
        // FIFO offsets: one wave prefix sum of the per-lane candidate counts
        const uint32_t cnt = (uint32_t)__popc(mask);
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t tag = (ring << 10) | (lane << 4);  // = (g mod 256) << 4
        if (tail - head + tot <= W.fifo_cap) {  // uniform: the whole iteration fits
            uint32_t pos = tail + incl - cnt;
            if ((tail & (QC - 1)) + tot <= QC) {  // uniform: no ring wrap inside the iteration's span
                // the lane's run is contiguous: one address increment per entry (round 6: no
                // ring mask and address rebuild per entry, ~2 VALU per append-loop trip)
                uint16_t* qp = W.q + (pos & (QC - 1));
                while (mask) {
                    const uint32_t e = __builtin_ctz(mask);
                    mask &= mask - 1;
                    *qp++ = (uint16_t)(tag | e);
                }
            } else {
                while (mask) {
                    const uint32_t e = __builtin_ctz(mask);
                    mask &= mask - 1;
                    W.q[pos & (QC - 1)] = (uint16_t)(tag | e);
                    ++pos;
                }
            }
            tail += tot;
        } else {  // an iteration denser than the FIFO (never at random draws beyond the dense
                  // head: ~4 candidates per block): one candidate per lane per round, resolved
                  // as 64 wait, so at most 127 are ever pending
            for (;;) {
                const bool has = mask != 0;
                const unsigned long long bal = __builtin_amdgcn_ballot_w64(has);
                if (!bal) break;
                if (has) {
                    const uint32_t e = __builtin_ctz(mask);
                    mask &= mask - 1;
                    const uint32_t pos = tail + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    W.q[pos & (QC - 1)] = (uint16_t)(tag | e);
                }
                tail += (uint32_t)__popcll(bal);
                if (tail - head >= 64) resolve_round(64u, gb);
            }
        }
        while (tail - head >= 64) resolve_round(64u, gb);
    }
    while (tail != head) resolve_round(std::min<uint32_t>(64u, tail - head), gb - 64);
    __builtin_amdgcn_wave_barrier();
    if constexpr (DEFER) {  // the caller gathers (one load site, see k2_segmented)
        int64_t at = -1;
        if (lane < k) {
            const IdxT wi = tab[lane];
            at = wi ? (int64_t)wi : ((int64_t)lane < len ? (int64_t)lane : -1);
        }
        __builtin_amdgcn_wave_barrier();
        return at;
    }
    for (uint32_t j = lane; j < k; j += 64) {
        const IdxT wi = tab[j];
        o[j] = wi ? keys[off + (int64_t)wi] : ((int64_t)j < len ? keys[off + j] : (KeyT)0);
    }
    __builtin_amdgcn_wave_barrier();
    return -1;
}

template <typename KeyT>
__global__ __launch_bounds__(64 * kWaves) void k2_segmented(const KeyT* __restrict__ keys,
                                                            const int64_t* __restrict__ offsets, int64_t S,
                                                            uint32_t k, uint32_t k0, uint32_t k1, uint64_t stream_base,
                                                            KeyT* __restrict__ out, int64_t* __restrict__ counts,
                                                            uint32_t fifo_cap = kQCap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    uint16_t* lut = (uint16_t*)lds;
    const uint64_t dense_lim = 256ull * k;
    // (32-bit division while the dividend fits: the table is rebuilt by every workgroup, and the
    // 64-bit form was ~2.5 % of a C3 launch at 32768 workgroups)
    for (uint32_t g = threadIdx.x; g < kLut; g += blockDim.x) {
        const uint64_t i0 = (uint64_t)g << 4;
        uint32_t T;
        if (i0 + 1 >= dense_lim) T = 0;
        else if (dense_lim + i0 <= 0xFFFFFFFFull) T = std::min<uint32_t>(256u, (uint32_t)(dense_lim + i0) / (uint32_t)(i0 + 1));
        else T = block_threshold(i0, dense_lim);
        lut[g] = (uint16_t)T;
    }
    __syncthreads();
    // wave index in a scalar register: stream numbers and offsets[] loads below are wave-uniform
    // (scalar loads, counted by lgkmcnt -- never waited for together with the deferred key gather)
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    // per wave: stash [kRing][64] x 16 B | FIFO kQCap x u16 | last-writer table k x (u32 | u64)
    constexpr size_t qbytes = kQueueBytes, sbytes = kStashBytes;
    const size_t tbytes = (size_t)k * 8;
    unsigned char* base = lds + kLutBytes + (size_t)wave * (sbytes + qbytes + tbytes);
    void* tab = base + sbytes + qbytes;
    const Wave W{(u32x4*)base, (uint16_t*)(base + sbytes), tab, lut, lane, k,
                 k0, k1, dense_lim, std::min<uint32_t>(std::max<uint32_t>(fifo_cap, 128u), kQCap)};
    const int64_t wave_stride = (int64_t)gridDim.x * kWaves;
    int64_t s = (int64_t)blockIdx.x * kWaves + wave;
    int64_t off = 0, end = 0;
    if (s < S) {
        off = offsets[s];
        end = offsets[s + 1];
    }
    if (k <= 64) {
        // Each stream's winner key is gathered at its end and stored TWO streams later, so every
        // wave keeps two streams' gathers in flight (one was measured short of the memory
        // concurrency the random-line rate needs: ~57 lines x 6k waves x 2 / 9 us of in-flight time).
        // The stream loop is unrolled by two so stream t's key lives in register set t & 1 and no
        // register copy of a load in flight exists (no s_waitcnt beyond the one for the store's data).
        KeyT* po[2] = {nullptr, nullptr};
        KeyT pv[2] = {0, 0};
        bool pok[2] = {false, false};
        const __attribute__((address_space(4))) int64_t* co =
            (const __attribute__((address_space(4))) int64_t*)offsets;
        auto one = [&](int u) {
            off = ((int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off)) |
                  ((int64_t)__builtin_amdgcn_readfirstlane((int)(off >> 32)) << 32);
            end = ((int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)end)) |
                  ((int64_t)__builtin_amdgcn_readfirstlane((int)(end >> 32)) << 32);
            const int64_t len = end - off;
            const int64_t s_pf = std::min<int64_t>(s + wave_stride, S - 1);
            // scalar loads (constant address space: offsets[] is read-only here), so that no
            // vmcnt wait for them drains the gathers in flight
            const int64_t off_next = co[s_pf], end_next = co[s_pf + 1];
            const uint64_t stream = stream_base + (uint64_t)s;
            KeyT* o = out + s * (int64_t)k;
            const int64_t at = len < kSmallLen ? k2_stream<KeyT, true, true>(W, keys, off, len, stream, o)
                                               : k2_stream<KeyT, false, true>(W, keys, off, len, stream, o);
            // the gather of stream s - 2*wave_stride (slot u) has had two streams of work to land:
            // after it this wave issued at least two vector-memory ops (the counts store and slot
            // 1-u's gather; the po store too once both slots are live), so vmcnt(2) covers it
            // without waiting for slot 1-u's gather. The loads are asm so that the compiler's own
            // waits (which cannot count past a load it does not see) stay conservative.
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(pv[u]));
            if (po[u] && lane < k) po[u][lane] = pok[u] ? pv[u] : (KeyT)0;
            if (lane == 0) counts[s] = len < (int64_t)k ? len : (int64_t)k;
            po[u] = o;
            pok[u] = at >= 0;  // else an empty slot: the load below reads a valid dummy word
            const KeyT* src = pok[u] ? keys + off + at : (const KeyT*)offsets;
            if constexpr (sizeof(KeyT) == 8)
                asm volatile("global_load_dwordx2 %0, %1, off" : "=&v"(pv[u]) : "v"(src));
            else
                asm volatile("global_load_dword %0, %1, off" : "=&v"(pv[u]) : "v"(src));
            off = off_next;
            end = end_next;
            s += wave_stride;
        };
        for (; s + wave_stride < S;) {  // two streams a trip (wave-uniform), no exit between them
            one(0);
            one(1);
        }
        if (s < S) one(0);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(pv[0]), "+v"(pv[1]));
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (po[u] && lane < k) po[u][lane] = pok[u] ? pv[u] : (KeyT)0;
        return;
    }
    for (; s < S; s += wave_stride) {
        // wave-uniform stream bounds (scalar registers: uniform control flow below)
        off = ((int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)off)) |
              ((int64_t)__builtin_amdgcn_readfirstlane((int)(off >> 32)) << 32);
        end = ((int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)end)) |
              ((int64_t)__builtin_amdgcn_readfirstlane((int)(end >> 32)) << 32);
        const int64_t len = end - off;
        const int64_t s_next = s + wave_stride;
        // prefetch, in flight during this stream's work; unconditional (clamped index), so the
        // loop-top wait for it is vmcnt(1) -- it does not also wait for the deferred gather below
        const int64_t s_pf = std::min<int64_t>(s_next, S - 1);
        const int64_t off_next = offsets[s_pf], end_next = offsets[s_pf + 1];
        const uint64_t stream = stream_base + (uint64_t)s;
        KeyT* o = out + s * (int64_t)k;
        if (len < kSmallLen) {
            k2_stream<KeyT, true, false>(W, keys, off, len, stream, o);
        } else {
            k2_stream<KeyT, false, false>(W, keys, off, len, stream, o);
        }
        if (lane == 0) counts[s] = len < (int64_t)k ? len : (int64_t)k;
        off = off_next;
        end = end_next;
    }
}

// ---- large k: one WORKGROUP per stream ------------------------------------------------------------
// Per wave, k2_segmented keeps a k-slot table in LDS: above k ~ 512 the tables cap a CU at one or two
// workgroups (k = 4096: 150 KB, one wave per SIMD) and above k = 4416 they no longer fit at all --
// round 4's global per-wave tables then paid global atomics and a 1 GiB zero fill per call (3.7 ms
// for 4096 x 2^17 at k = 8192).  Here the NW waves of a workgroup share ONE stream and ONE table:
// wave w takes the stream's 64-block iterations w, w + NW, w + 2 NW, ... (interleaved, so the
// candidate-rich dense head is spread over the waves), each with its own stash ring and FIFO, and all
// resolve into the workgroup's table -- in LDS while k * sizeof(TabT) fits beside the waves' rings,
// else the workgroup's slice of a global scratch table that stays zero between streams (the gather
// takes every entry back with an atomic exchange).  TabT = u32 when every stream index fits 32 bits.
constexpr int kWavesWG = 8;
constexpr uint32_t kWGMinK = 512;  // smaller k keep one wave per stream (C3: k = 64)

__host__ __device__ inline size_t lds_bytes_wg(uint32_t k, size_t tab_entry, bool GT) {
    return kLutBytes + (size_t)kWavesWG * (kStashBytes + kQueueBytes) + (GT ? 0 : (size_t)k * tab_entry);
}

template <typename TabT, bool SMALL, bool GT>
__device__ __forceinline__ void k2_part(const Wave& W, TabT* tab, int64_t len, uint64_t stream, uint32_t wave) {
    using IdxT = typename std::conditional<SMALL, uint32_t, uint64_t>::type;
    constexpr uint32_t QC = kQCap, RG = kRing;
    constexpr uint32_t STEP = 64u * kWavesWG;  // blocks between this wave's iterations
    const uint32_t lane = W.lane, k = W.k;
    const uint32_t s0 = (uint32_t)stream, s1 = (uint32_t)(stream >> 32);
    const DrawKey dk{W.k0, W.k1, s0, s1};
    const IdxT n_groups = (IdxT)(((uint64_t)len + 15) >> 4);
    uint32_t head = 0, tail = 0;
    IdxT gb = (IdxT)(((k >> 4) & ~63u) + 64u * wave);
    uint32_t ring = 0;
    IdxT slot_gb[RG] = {};  // first block of the iteration each ring slot holds (wave-uniform)

    auto resolve_round = [&](uint32_t nvalid) {
        __builtin_amdgcn_wave_barrier();
        const bool valid = lane < nvalid;
        const uint32_t ent = valid ? W.q[(head + lane) & (QC - 1)] : 0u;
        const uint32_t e = ent & 15u, r = ent >> 10;
        const u32x4 w = W.stash[ent >> 4];
        IdxT g0 = slot_gb[0];
#pragma unroll
        for (uint32_t q = 1; q < RG; ++q) g0 = r == q ? slot_gb[q] : g0;
        const IdxT i = ((g0 + (IdxT)((ent >> 4) & 63u)) << 4) + (IdxT)e;
        const uint32_t b = level0_byte(w, e);
        const IdxT g1 = i >> 1;
        u32x4 w1;
        if constexpr (SMALL) w1 = philox4x32_10_uniform_hi((uint32_t)g1, kDomainLevel1, s0, s1, W.k0, W.k1);
        else w1 = philox4x32_10((uint32_t)g1, (uint32_t)((uint64_t)g1 >> 32) | kDomainLevel1, s0, s1, W.k0, W.k1);
        asm volatile("" : "+v"(w1.x), "+v"(w1.y), "+v"(w1.z), "+v"(w1.w));
        const bool odd = (i & 1) != 0;
        const uint64_t j = draw_j(b, odd ? w1.z : w1.x, odd ? w1.w : w1.y, (uint64_t)i + 1, SMALL);
        if (valid && j < k) atomicMax(&tab[(uint32_t)j], (TabT)i);
        head += nvalid;
        __builtin_amdgcn_wave_barrier();
    };

    // the dense head [k, hend) by index pairs, as k2_stream (each wave takes its iterations' share)
    uint64_t hx = 4ull * k;
    if (hx - k >= 128) hx = k + ((hx - k) & ~(uint64_t)127);
    const IdxT hend = (IdxT)std::min<uint64_t>((uint64_t)len, hx);
    const IdxT flo = std::max<IdxT>((IdxT)k, hend);
    for (; gb < n_groups; gb += STEP, ring = (ring + 1) & (RG - 1)) {
        if (tail != head && ((uint32_t)__builtin_amdgcn_readfirstlane((int)W.q[head & (QC - 1)]) >> 10) == ring) {
            while (tail != head) resolve_round(std::min<uint32_t>(64u, tail - head));
        }
        slot_gb[0] = ring == 0 ? gb : slot_gb[0];
#pragma unroll
        for (uint32_t q = 1; q < RG; ++q) slot_gb[q] = ring == q ? gb : slot_gb[q];
        const IdxT g = gb + lane;
        const bool valid = g < n_groups;
        u32x4 w;
        if constexpr (SMALL) w = philox4x32_10_uniform_hi((uint32_t)g, 0u, s0, s1, W.k0, W.k1);
        else w = level0(dk, (uint64_t)g);
        const uint64_t i0 = (uint64_t)g << 4;
        const uint32_t T = g < kLut ? (uint32_t)W.lut[(uint32_t)g] : block_threshold(i0, W.dense_lim);
        const uint32_t Tmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)T);
        uint32_t mask = valid ? (Tmax <= 16u ? mask_for_small(w, T) : mask_for(w, T)) : 0u;
        const bool clip = ((uint64_t)gb << 4) < (uint64_t)flo || (((uint64_t)gb + 64) << 4) > (uint64_t)len;
        if (clip) mask &= clip16(i0, (uint64_t)flo, (uint64_t)len);
        W.stash[ring * 64 + lane] = w;
        if (((uint64_t)gb << 4) < (uint64_t)hend) {  // this iteration holds head indices (uniform)
            __builtin_amdgcn_wave_barrier();
            const IdxT ia = std::max<IdxT>((IdxT)k & ~(IdxT)1, gb << 4);
            const IdxT ib = std::min<IdxT>(hend, (gb + 64) << 4);
            for (IdxT p0 = ia; p0 < ib; p0 += 128) {
                const IdxT i = p0 + 2 * lane;  // even
                const u32x4 wl = W.stash[ring * 64 + (uint32_t)((i >> 4) - gb)];
                uint32_t b0, b1;
                level0_byte_pair(wl, (uint32_t)i & 15u, b0, b1);
                const IdxT g1 = i >> 1;
                u32x4 w1;
                if constexpr (SMALL) w1 = philox4x32_10_uniform_hi((uint32_t)g1, kDomainLevel1, s0, s1, W.k0, W.k1);
                else w1 = philox4x32_10((uint32_t)g1, (uint32_t)((uint64_t)g1 >> 32) | kDomainLevel1, s0, s1, W.k0, W.k1);
                asm volatile("" : "+v"(w1.x), "+v"(w1.y), "+v"(w1.z), "+v"(w1.w));
                const uint64_t j0 = draw_j(b0, w1.x, w1.y, (uint64_t)i + 1, SMALL);
                const uint64_t j1 = draw_j(b1, w1.z, w1.w, (uint64_t)i + 2, SMALL);
                if (i < ib && i >= (IdxT)k && j0 < k) atomicMax(&tab[(uint32_t)j0], (TabT)i);
                if (i + 1 < ib && i + 1 >= (IdxT)k && j1 < k) atomicMax(&tab[(uint32_t)j1], (TabT)(i + 1));
            }
            __builtin_amdgcn_wave_barrier();
        }
        const uint32_t cnt = (uint32_t)__popc(mask);
        const uint32_t incl = wave_incl_scan(cnt);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t tag = (ring << 10) | (lane << 4);
        if (tail - head + tot <= W.fifo_cap) {
            uint32_t pos = tail + incl - cnt;
            while (mask) {
                const uint32_t e = __builtin_ctz(mask);
                mask &= mask - 1;
                W.q[pos & (QC - 1)] = (uint16_t)(tag | e);
                ++pos;
            }
            tail += tot;
        } else {  // denser than the FIFO: one candidate per lane per round, resolved 64 at a time
            for (;;) {
                const bool has = mask != 0;
                const unsigned long long bal = __builtin_amdgcn_ballot_w64(has);
                if (!bal) break;
                if (has) {
                    const uint32_t e = __builtin_ctz(mask);
                    mask &= mask - 1;
                    const uint32_t pos = tail + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    W.q[pos & (QC - 1)] = (uint16_t)(tag | e);
                }
                tail += (uint32_t)__popcll(bal);
                if (tail - head >= 64) resolve_round(64u);
            }
        }
        while (tail - head >= 64) resolve_round(64u);
    }
    while (tail != head) resolve_round(std::min<uint32_t>(64u, tail - head));
    __builtin_amdgcn_wave_barrier();
}

template <typename KeyT, typename TabT, bool GT>
__global__ __launch_bounds__(64 * kWavesWG) void k2_segmented_wg(const KeyT* __restrict__ keys,
                                                                 const int64_t* __restrict__ offsets, int64_t S,
                                                                 uint32_t k, uint32_t k0, uint32_t k1,
                                                                 uint64_t stream_base, KeyT* __restrict__ out,
                                                                 int64_t* __restrict__ counts, uint32_t fifo_cap,
                                                                 TabT* __restrict__ gtab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    uint16_t* lut = (uint16_t*)lds;
    const uint64_t dense_lim = 256ull * k;
    for (uint32_t g = threadIdx.x; g < kLut; g += blockDim.x) {
        const uint64_t i0 = (uint64_t)g << 4;
        uint32_t T;
        if (i0 + 1 >= dense_lim) T = 0;
        else if (dense_lim + i0 <= 0xFFFFFFFFull) T = std::min<uint32_t>(256u, (uint32_t)(dense_lim + i0) / (uint32_t)(i0 + 1));
        else T = block_threshold(i0, dense_lim);
        lut[g] = (uint16_t)T;
    }
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    unsigned char* base = lds + kLutBytes + (size_t)wave * (kStashBytes + kQueueBytes);
    TabT* tab = GT ? gtab + (size_t)blockIdx.x * k
                   : (TabT*)(lds + kLutBytes + (size_t)kWavesWG * (kStashBytes + kQueueBytes));
    const Wave W{(u32x4*)base, (uint16_t*)(base + kStashBytes), nullptr, lut, lane, k,
                 k0, k1, dense_lim, std::min<uint32_t>(std::max<uint32_t>(fifo_cap, 128u), kQCap)};
    const uint32_t nthr = 64u * kWavesWG;
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t off = offsets[s], len = offsets[s + 1] - off;
        if constexpr (!GT)
            for (uint32_t j = threadIdx.x; j < k; j += nthr) tab[j] = 0;
        __syncthreads();  // the table is zero (GT: the previous stream's gather left it so)
        const uint64_t stream = stream_base + (uint64_t)s;
        if (len < kSmallLen) k2_part<TabT, true, GT>(W, tab, len, stream, wave);
        else k2_part<TabT, false, GT>(W, tab, len, stream, wave);
        if constexpr (GT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this wave's table atomics
        __syncthreads();
        if constexpr (GT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every wave's, before the gather
        KeyT* o = out + s * (int64_t)k;
        for (uint32_t j = threadIdx.x; j < k; j += nthr) {
            TabT wi;
            if constexpr (GT) wi = __hip_atomic_exchange(&tab[j], (TabT)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else wi = tab[j];
            o[j] = wi ? keys[off + (int64_t)wi] : ((int64_t)j < len ? keys[off + j] : (KeyT)0);
        }
        if (threadIdx.x == 0) counts[s] = len < (int64_t)k ? len : (int64_t)k;
        __syncthreads();  // the gather has read the table before the next stream zeroes it
    }
}

}  // namespace k2
}  // namespace rsv
