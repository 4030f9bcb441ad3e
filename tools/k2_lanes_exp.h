// k2_lanes_exp.h -- EXPERIMENT (not product): K2 with one stream per lane, timed by tools/micro_k2.hip
// against the product's wave-per-stream kernel (rsv_k2.h).  Kept for the record of DESIGN.md 5.3:
// identical results, slower on MI355X (PMC at C3: 1143 VALU per stream, 6.0 cycles per VALU
// instruction; the forward-scan form with an LDS last-writer table: 862 VALU per stream but 7.5
// cycles per instruction at 2 waves per SIMD, LDS-bound occupancy).
#pragma once
#include "../reservoir_amd/csrc/rsv_k2.h"

namespace rsv {
namespace k2 {

// ---- lane-per-stream form (k <= 64, streams of at most 2^16 elements) ---------------------------
// A wave takes 64 consecutive streams, one per lane, and walks their level-0 blocks in lockstep
// (block g of every stream at once): the block threshold is wave-uniform (scalar), and candidates
// stay in their lane -- no prefix sums, no FIFO of byte references, no ballot-serialised appends.
//
// Each stream is scanned BACKWARD (last block first, highest index first within a block): the
// winner of slot j is the largest i with j_i = j, i.e. the FIRST hit of the backward scan, so a
// 64-bit `filled` mask per lane replaces the last-writer table, and a candidate whose possible
// slots [floor(b (i+1) / 256), floor(((b+1)(i+1) - 1) / 256)] are all filled already can be
// dropped without its level-1 draw.  Late in the scan (the dense head, i < 256) most slots are
// taken: at C3 ~128 of a stream's ~273 candidates need the level-1 draw (simulated).  A hit
// stores the winner's index straight into the output row; the keys are gathered at the end.
//
// Level 0 pushes each block with a candidate (its words + a (g, mask) word) into the lane's own
// LDS ring; the level-1 draws run in rounds: every lane first skips to its next candidate that
// survives the filled test, then the lanes holding one evaluate it together.  A round is taken
// while at least kRoundMin lanes have work or some lane's ring is full.
//
// Philox with the stream in counter word 2 and the other words wave-uniform: M1 * s0 is a lane
// constant, and so are the first outputs it feeds.  Level 0 (c0 = g uniform, c1 = 0): rounds 0
// and 1 take 2 VALU in all (34 per call instead of 37); level 1 (c0 = i/2 per lane, c1 = the
// level-1 domain): 37 instead of 40.
constexpr uint32_t kLaneKMax = 64;
constexpr int64_t kLaneMaxLen = 1 << 16;  // 16-bit winner indices
#ifndef RSV_K2_LANE_CAP
#define RSV_K2_LANE_CAP 8
#endif
#ifndef RSV_K2_WAVES2
#define RSV_K2_WAVES2 2
#endif
#ifndef RSV_K2_ROUND_MIN
#define RSV_K2_ROUND_MIN 48
#endif
constexpr uint32_t kLaneCap = RSV_K2_LANE_CAP;  // ring records per lane
constexpr uint32_t kRoundMin = RSV_K2_ROUND_MIN;
constexpr int kWaves2 = RSV_K2_WAVES2;          // waves per workgroup

__host__ __device__ inline size_t lane_wave_bytes(uint32_t k) {
    const size_t lanes = (size_t)kLaneCap * 64 * 20;
    const size_t per_stream = kStashBytes + kQueueBytes + (size_t)k * 8;  // the fallback (k2_stream)
    return ((lanes > per_stream ? lanes : per_stream) + 15) & ~(size_t)15;
}

__host__ __device__ inline size_t lds_bytes2(uint32_t k) { return kLutBytes + (size_t)kWaves2 * lane_wave_bytes(k); }

struct LaneConst {
    uint32_t A0, B0, P0h, P0l;  // level 0
    uint32_t A1, P1h, P1l;      // level 1
};

__device__ __forceinline__ LaneConst lane_const(uint32_t s0, uint32_t k0) {
    LaneConst c;
    const uint64_t m1s0 = (uint64_t)kPhiloxM1 * s0;
    c.B0 = (uint32_t)m1s0;
    c.A0 = (uint32_t)(m1s0 >> 32) ^ k0;  // round-0 output word 0 with c1 = 0
    const uint64_t p0 = (uint64_t)kPhiloxM0 * c.A0;
    c.P0h = (uint32_t)(p0 >> 32);
    c.P0l = (uint32_t)p0;
    c.A1 = c.A0 ^ kDomainLevel1;  // ... with c1 = the level-1 domain bit
    const uint64_t p1 = (uint64_t)kPhiloxM0 * c.A1;
    c.P1h = (uint32_t)(p1 >> 32);
    c.P1l = (uint32_t)p1;
    return c;
}

// rounds 2..9 of Philox4x32-10 from state (x0, x1, x2, x3); round 2's x1 may be scalar (`s1x`)
__device__ __forceinline__ u32x4 philox_rounds_from2(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3,
                                                      uint32_t k0, uint32_t k1, bool x1_scalar) {
    {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * x0;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * x2;
        const uint32_t t = x1 ^ (k0 + 2u * kPhiloxW0);
        const uint32_t n0 = x1_scalar ? (uint32_t)(p1 >> 32) ^ t : xor3_key((uint32_t)(p1 >> 32), x1, k0 + 2u * kPhiloxW0);
        const uint32_t n2 = xor3_key((uint32_t)(p0 >> 32), x3, k1 + 2u * kPhiloxW1);
        x0 = n0;
        x1 = (uint32_t)p1;
        x2 = n2;
        x3 = (uint32_t)p0;
    }
#pragma unroll
    for (int r = 3; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * x0;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * x2;
        const uint32_t n0 = xor3_key((uint32_t)(p1 >> 32), x1, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t n2 = xor3_key((uint32_t)(p0 >> 32), x3, k1 + (uint32_t)r * kPhiloxW1);
        x0 = n0;
        x1 = (uint32_t)p1;
        x2 = n2;
        x3 = (uint32_t)p0;
    }
    return {x0, x1, x2, x3};
}

// level 0: counter (g, 0, s0, s1), g and s1 wave-uniform, s0 = the lane's stream
__device__ __forceinline__ u32x4 level0_lane(uint32_t g, uint32_t s1, const LaneConst& c, uint32_t k0, uint32_t k1) {
    const uint64_t p0u = (uint64_t)kPhiloxM0 * g;                    // scalar
    const uint32_t n2u = (uint32_t)(p0u >> 32) ^ s1 ^ k1;            // scalar
    const uint32_t c3u = (uint32_t)p0u;                              // scalar
    const uint64_t p1u = (uint64_t)kPhiloxM1 * n2u;                  // scalar (round 1, word 2)
    // the scalar halves of round 1's xors, pinned to SGPRs so each leaves one v_xor
    const uint32_t t0 = (uint32_t)(p1u >> 32) ^ (k0 + kPhiloxW0), t2 = c3u ^ (k1 + kPhiloxW1);
    const uint32_t x0 = c.B0 ^ t0;
    const uint32_t x2 = c.P0h ^ t2;
    return philox_rounds_from2(x0, (uint32_t)p1u, x2, c.P0l, k0, k1, true);
}

// level 1: counter (g1, domain, s0, s1), g1 per lane, s1 wave-uniform
__device__ __forceinline__ u32x4 level1_lane(uint32_t g1, uint32_t s1, const LaneConst& c, uint32_t k0, uint32_t k1) {
    const uint64_t p0 = (uint64_t)kPhiloxM0 * g1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ (s1 ^ k1);
    const uint64_t p1 = (uint64_t)kPhiloxM1 * n2;  // round 1 (word 0's product is the constant P1)
    const uint32_t x0 = xor3_key((uint32_t)(p1 >> 32), c.B0, k0 + kPhiloxW0);
    const uint32_t x2 = xor3_key(c.P1h, (uint32_t)p0, k1 + kPhiloxW1);
    return philox_rounds_from2(x0, (uint32_t)p1, x2, c.P1l, k0, k1, false);
}

// b_e < M + 1 for the 16 bytes of a block, M wave-uniform in [0, 254]: the borrow chain over the
// planes up to M's top bit; every higher plane must be zero, so they are OR'ed in.
template <int NB>
__device__ __forceinline__ uint32_t le_mask_nb(const u32x4& w, uint32_t M) {
    const uint32_t words[4] = {w.x, w.y, w.z, w.w};
    uint32_t br = 0;
#pragma unroll
    for (int p = 0; p < NB; ++p) {
        const uint32_t plane = (p & 1) ? (words[p >> 1] >> 16) : words[p >> 1];
        const uint32_t mm = (uint32_t)((int32_t)(M << (31 - p)) >> 31);
        br = __builtin_amdgcn_bitop3_b32(plane, br, mm, 0xD4);
    }
    uint32_t hi = 0;
#pragma unroll
    for (int p = NB; p < 8; ++p) {
        if ((p & 1) && p > NB) continue;  // the odd plane rides with its word below
        hi |= (p & 1) ? (words[p >> 1] >> 16) : words[p >> 1];
    }
    if (NB < 8) hi |= hi >> 16;  // the odd planes of the OR'ed words
    return ~(br | hi) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t le_mask(const u32x4& w, uint32_t M) {
    if (M >= 255) return 0xFFFFu;
    switch (32 - __builtin_clz(M | 1) - (M == 0)) {  // M's bit length (0 for M = 0)
    case 0: return le_mask_nb<0>(w, M);
    case 1: return le_mask_nb<1>(w, M);
    case 2: return le_mask_nb<2>(w, M);
    case 3: return le_mask_nb<3>(w, M);
    case 4: return le_mask_nb<4>(w, M);
    case 5: return le_mask_nb<5>(w, M);
    case 6: return le_mask_nb<6>(w, M);
    case 7: return le_mask_nb<7>(w, M);
    default: return le_mask_nb<8>(w, M);
    }
}

// inclusive wave max (unsigned)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) { return ~wave_max_u32(~x); }

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63);
}

// The wave's 64 streams, one per lane (len <= 2^16, k <= 64, stream words 1 wave-uniform).
// `o` = out + s_first * k; lanes past S have len = 0.
template <typename KeyT>
__device__ __forceinline__ void k2_lanes(unsigned char* wl, const KeyT* __restrict__ keys, int64_t off, uint32_t len,
                                         uint32_t maxlen, uint32_t minlen, uint32_t s0, uint32_t s1, uint32_t k,
                                         uint32_t k0, uint32_t k1, int64_t n_streams, KeyT* __restrict__ o) {
    const uint32_t lane = threadIdx.x & 63;
    u32x4* ring_w = (u32x4*)wl;                              // [kLaneCap][64]
    uint32_t* ring_m = (uint32_t*)(wl + kLaneCap * 64 * 16);  // [kLaneCap][64]: (g << 16) | mask
    KeyT* orow = o + (int64_t)lane * k;                       // this lane's output row (winner indices first)

    const LaneConst c = lane_const(s0, k0);
    const uint32_t dlim_m1 = 256u * k - 1u;
    const uint32_t ng = (maxlen + 15) >> 4;
    const uint32_t g_end = k >> 4;                            // first block holding an index >= k
    uint64_t filled = k >= 64 ? 0ull : ~0ull << k;            // slots >= k never take a hit
    uint32_t head = 0, tail = 0, cur_mask = 0, cur_g = 0;
    u32x4 cw{0, 0, 0, 0};
    uint32_t M = 0;  // block threshold b <= M, rising as the scan moves toward the head

    // one round: every lane skips to its next live candidate, then the live lanes draw level 1
    auto round = [&]() {
        bool live = false;
        uint32_t li = 0, lb = 0;
        for (;;) {
            const bool want = !live && (cur_mask | (head ^ tail)) != 0;
            if (!__builtin_amdgcn_ballot_w64(want)) break;
            if (want) {
                if (cur_mask == 0) {
                    const uint32_t at = (head & (kLaneCap - 1)) * 64 + lane;
                    cw = ring_w[at];
                    const uint32_t m = ring_m[at];
                    cur_mask = m & 0xFFFFu;
                    cur_g = m >> 16;
                    ++head;
                }
                const uint32_t e = 31 - __builtin_clz(cur_mask);  // highest index first
                cur_mask ^= 1u << e;
                const uint32_t i = (cur_g << 4) | e;
                const uint32_t b = level0_byte(cw, e);
                const uint32_t x = b * (i + 1);  // < 2^24
                const uint32_t jlo = x >> 8;
                if (jlo < k) {
                    const uint32_t w = ((x + i) >> 8) - jlo;        // slots jlo .. jlo + w (w <= 16)
                    const uint32_t free = (uint32_t)(~filled >> jlo);
                    live = (free & ((2u << w) - 1u)) != 0;
                    li = i;
                    lb = b;
                }
            }
        }
        if (live) {
            const u32x4 w1 = level1_lane(li >> 1, s1, c, k0, k1);
            const uint64_t L = (li & 1) ? (((uint64_t)w1.z << 32) | w1.w) : (((uint64_t)w1.x << 32) | w1.y);
            const uint32_t j = (uint32_t)draw_j(lb, (uint32_t)(L >> 32), (uint32_t)L, (uint64_t)li + 1, true);
            if (j < k && !((filled >> j) & 1ull)) {  // the first hit of the backward scan wins
                filled |= 1ull << j;
                orow[j] = (KeyT)li;
            }
        }
    };

    // one level-0 block of every lane's stream; CLIP: the block straddles index k or some stream's end
    auto block = [&](uint32_t g, auto clip) {
        const uint32_t i0 = g << 4;
        // scalar, <= 255 steps per wave in all (the empty asm keeps the compiler from turning the
        // search into a VALU one)
        while (M < 255 && (M + 1) * (i0 + 1) <= dlim_m1) {
            ++M;
            asm volatile("" : "+s"(M));
        }
        const u32x4 w = level0_lane(g, s1, c, k0, k1);
        uint32_t mask = le_mask(w, M);
        if constexpr (decltype(clip)::value) {
            if (i0 < k) mask &= (0xFFFFu << (k - i0)) & 0xFFFFu;
            mask &= len > i0 ? (0xFFFFu >> (16 - std::min<uint32_t>(16u, len - i0))) : 0u;
        }
        if (mask) {
            const uint32_t at = (tail & (kLaneCap - 1)) * 64 + lane;
            ring_w[at] = w;
            ring_m[at] = (g << 16) | mask;
            ++tail;
        }
        for (;;) {
            const uint32_t pend = tail - head;
            const uint32_t busy = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64((pend | cur_mask) != 0));
            const bool full = __builtin_amdgcn_ballot_w64(pend >= kLaneCap) != 0;
            if (!full && busy < kRoundMin) break;
            round();
        }
    };
    // blocks [g_end, ng), last first: those ending past some stream's end, then the clean middle,
    // then the block straddling index k
    const uint32_t g_mid_hi = std::max(g_end, std::min(minlen >> 4, ng));   // blocks below end within every stream
    const uint32_t g_mid_lo = std::min((k + 15) >> 4, g_mid_hi);             // blocks from here start at or past k
    uint32_t g = ng;
    for (; g > g_mid_hi; --g) block(g - 1, std::true_type());
    for (; g > g_mid_lo; --g) block(g - 1, std::false_type());
    for (; g > g_end; --g) block(g - 1, std::true_type());
    while (__builtin_amdgcn_ballot_w64((cur_mask | (head ^ tail)) != 0)) round();

    // winners' keys: one stream per step, lane j = slot j (coalesced), 8 streams' loads in flight;
    // a slot without a hit keeps its first element (j < len)
    const uint32_t nst = (uint32_t)std::min<int64_t>(64, n_streams);
    const uint32_t fl = (uint32_t)filled, fh = (uint32_t)(filled >> 32);
    for (uint32_t t0 = 0; t0 < nst; t0 += 8) {
        int64_t idx[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t t = t0 + u;
            idx[u] = -1;
            if (t < nst && lane < k) {
                const uint32_t lt = (uint32_t)__builtin_amdgcn_readlane((int)len, (int)t);
                const uint64_t ft = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)fl, (int)t) |
                                    ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)fh, (int)t) << 32);
                if ((ft >> lane) & 1ull) idx[u] = (int64_t)o[(int64_t)t * k + lane];
                else if (lane < lt) idx[u] = lane;
            }
        }
        KeyT v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t t = t0 + u;
            v[u] = 0;
            if (t < nst && lane < k && idx[u] >= 0) {
                const int64_t ot = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off, (int)t) |
                                   ((int64_t)__builtin_amdgcn_readlane((int)(off >> 32), (int)t) << 32);
                v[u] = keys[ot + idx[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t t = t0 + u;
            if (t < nst && lane < k) o[(int64_t)t * k + lane] = v[u];
        }
    }
}

// K2, second form: per wave 64 consecutive streams; lane-per-stream when they qualify (k <= 64,
// every stream <= 2^16 elements, lengths within 2x of the longest on average), else each stream
// through k2_stream (wave-per-stream) in turn.
template <typename KeyT>
__global__ __launch_bounds__(64 * kWaves2) void k2_segmented2(const KeyT* __restrict__ keys,
                                                              const int64_t* __restrict__ offsets, int64_t S,
                                                              uint32_t k, uint32_t k0, uint32_t k1,
                                                              uint64_t stream_base, KeyT* __restrict__ out,
                                                              int64_t* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    uint16_t* lut = (uint16_t*)lds;
    const uint64_t dense_lim = 256ull * k;
    for (uint32_t g = threadIdx.x; g < kLut; g += blockDim.x) lut[g] = (uint16_t)block_threshold((uint64_t)g << 4, dense_lim);
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned char* wl = lds + kLutBytes + (size_t)wave * lane_wave_bytes(k);
    const int64_t n_groups = (S + 63) >> 6;
    for (int64_t wg = (int64_t)blockIdx.x * kWaves2 + wave; wg < n_groups; wg += (int64_t)gridDim.x * kWaves2) {
        const int64_t s_first = wg << 6;
        const int64_t s = s_first + lane;
        int64_t off = 0, len = 0;
        if (s < S) {
            off = offsets[s];
            len = offsets[s + 1] - off;
        }
        const int64_t n_st = std::min<int64_t>(64, S - s_first);
        const uint32_t lenc = (uint32_t)std::min<int64_t>(len, kLaneMaxLen + 1);
        const uint32_t maxlen = wave_max_u32(lenc);
        const uint32_t minlen = wave_min_u32(lane < n_st ? lenc : 0xFFFFFFFFu);
        const uint32_t sumlen = wave_sum_u32(lenc);
        const uint64_t st_first = stream_base + (uint64_t)s_first, st_last = st_first + (uint64_t)(n_st - 1);
        const bool lanes_ok = k <= kLaneKMax && maxlen <= kLaneMaxLen && (st_first >> 32) == (st_last >> 32) &&
                              2ull * sumlen >= (uint64_t)n_st * maxlen;
        if (lanes_ok) {
            const uint64_t st = stream_base + (uint64_t)s;
            k2_lanes<KeyT>(wl, keys, off, lane < n_st ? lenc : 0u, maxlen, minlen, (uint32_t)st,
                           (uint32_t)(st_first >> 32), k, k0, k1, n_st, out + s_first * (int64_t)k);
        } else {
            const Wave W{(u32x4*)wl, (uint16_t*)(wl + kStashBytes), wl + kStashBytes + kQueueBytes, lut, lane, k,
                         k0, k1, dense_lim, kQCap};
            for (int64_t t = 0; t < n_st; ++t) {
                const int64_t ot = offsets[s_first + t];
                const int64_t lt = offsets[s_first + t + 1] - ot;
                const int64_t o_t = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ot) |
                                    ((int64_t)__builtin_amdgcn_readfirstlane((int)(ot >> 32)) << 32);
                const int64_t l_t = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lt) |
                                    ((int64_t)__builtin_amdgcn_readfirstlane((int)(lt >> 32)) << 32);
                KeyT* o = out + (s_first + t) * (int64_t)k;
                if (l_t < kSmallLen)
                    k2_stream<KeyT, 0, true, false>(W, keys, o_t, l_t, stream_base + (uint64_t)(s_first + t), o);
                else
                    k2_stream<KeyT, 0, false, false>(W, keys, o_t, l_t, stream_base + (uint64_t)(s_first + t), o);
            }
        }
        if (s < S) counts[s] = len < (int64_t)k ? len : (int64_t)k;
    }
}

}  // namespace k2
}  // namespace rsv
