// k1_dev_bodies.h -- development K1 loop bodies kept for A/B timing in tools/micro_k1.hip and
// tools/micro_k1o.hip (NOT product code: the product K1 is rsv_scan.h k1_body_q).  Moved out of the
// product header in rounds 4 and 5.  Each was the product body in an earlier round (DESIGN.md 5
// decision 1):
//   k1_body       per-iteration block pushes (round 1)
//   k1_body_bits  deferred pushes, one bit per block (round 2)
//   k1_body_z     the zero-byte fold carried in the queue (round 2-3)
//   k1_body_p     pair entries, window bits pushed in ballot rounds (rounds 3-4)
#pragma once
#include "../reservoir_amd/csrc/rsv_scan.h"

#ifndef RSV_K1P_COUNT
#define RSV_K1P_COUNT(i, v)  // development counters (tools/micro_k1o.hip)
#endif

namespace rsv {
// Push the U blocks of one iteration (has[u]: block g_begin + off[u] holds a candidate) with one
// wave-uniform branch; whenever 64 blocks wait, all lanes resolve one each.  The queue holds
// < 64 waiting + 64 U pushed entries.
template <int U, class Hit>
__device__ __forceinline__ void push_blocks(const bool (&has)[U], const uint32_t (&off)[U], uint32_t* q,
                                            uint32_t& qn, uint64_t* cq, uint32_t& cqn, uint32_t lane,
                                            const DrawKey& dk, uint64_t g_begin, uint64_t lo, uint64_t hi,
                                            uint64_t dense_lim, uint32_t k, Hit& hit) {
    unsigned long long bal[U], any = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        bal[u] = __ballot(has[u]);
        any |= bal[u];
    }
    if (any == 0) return;
    const unsigned long long lt = lanemask_lt64();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (has[u]) q[qn + __popcll(bal[u] & lt)] = off[u];
        qn += (uint32_t)__popcll(bal[u]);
    }
    while (qn >= 64) {
        qn -= 64;
        __builtin_amdgcn_wave_barrier();
        resolve_block(dk, true, g_begin + q[qn + lane], lo, hi, dense_lim, k, cq, cqn, lane, hit);
        __builtin_amdgcn_wave_barrier();
    }
}

template <class Hit>
__device__ __forceinline__ void drain_blocks(const uint32_t* q, uint32_t qn, uint64_t* cq, uint32_t& cqn,
                                             uint32_t lane, const DrawKey& dk, uint64_t g_begin, uint64_t lo,
                                             uint64_t hi, uint64_t dense_lim, uint32_t k, Hit& hit) {
    __builtin_amdgcn_wave_barrier();
    const bool valid = lane < qn;
    resolve_block(dk, valid, g_begin + (valid ? q[lane] : 0u), lo, hi, dense_lim, k, cq, cqn, lane, hit);
    drain_queue(dk, cq, cqn, lane, k, hit);
}

// K1 main loop, per-iteration pushes (the product launches k1_body_bits below; this form stays as
// the A/B reference of tools/micro_k1.hip): grid-stride over level-0 blocks (16 indices each), U blocks per lane per
// iteration; wave-uniform so the queue can run full-wave level-1 evaluations.  Hits (k ln(n/k) of
// them) go straight to global atomicMax on the k-slot winner table: ~14k atomics per 1e9 indices
// at k = 1024.  `q` = this wave's block queue (>= 63 + 64 U entries), `cq` its candidate queue
// (kQueue entries).
template <int U>
__device__ __forceinline__ void k1_body(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                        uint64_t n_groups, unsigned long long* __restrict__ win, uint32_t* q,
                                        uint64_t* cq) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t qn = 0, cqn = 0;
    auto hit = [&](uint32_t j, uint64_t i) { atomicMax(&win[j], (unsigned long long)i); };
    const uint64_t dense_lim = 256ull * k;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
    for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U; base < n_groups;
         base += stride) {
        u32x4 w[U];
        uint32_t off[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            off[u] = (uint32_t)(base + u * 64 + lane);  // n_groups < 2^32 per launch (host splits)
            w[u] = level0(dk, g_begin + off[u]);
        }
        bool has[U];
#pragma unroll
        for (int u = 0; u < U; ++u)  // dense region (index < 256k): any block may hit
            has[u] = (off[u] < n_groups) &  // bitwise: no short-circuit branches
                     (((((g_begin + off[u]) << 4) + 1) < dense_lim) | any_zero_byte(w[u]));
        push_blocks<U>(has, off, q, qn, cq, cqn, lane, dk, g_begin, lo, hi, dense_lim, k, hit);
    }
    drain_blocks(q, qn, cq, cqn, lane, dk, g_begin, lo, hi, dense_lim, k, hit);
}

// ---- K1 with deferred pushes -------------------------------------------------------------------
// The per-iteration push above runs on ~every iteration (some lane of the wave nearly always holds
// a candidate block) and cost ~28 us per 1e9 indices.  Here each lane only ORs one bit per block
// into a register mask; every W = 32 / U iterations the wave pushes the set bits in rounds -- each
// round every lane with bits left pushes its lowest one (ballot + prefix count), so a round is one
// wave-uniform step and the queue needs room for just one round (64) beyond a partial batch.
// The window's nb bits are shifted in oldest first (bits = bits * 2 + has: one v_lshl_or per block),
// so bit b is window block idx = nb - 1 - b, the block at offset base0 + (idx / U) * stride +
// (idx % U) * 64 + lane (all 32-bit: offsets < 2^31 per launch, stride * W < 2^32).
template <int U, class Hit>
__device__ __forceinline__ void push_bits(uint32_t bits, uint32_t nb, uint32_t base0, uint32_t stride, uint32_t* q,
                                          uint32_t& qn, uint64_t* cq, uint32_t& cqn, uint32_t lane, const DrawKey& dk,
                                          uint64_t g_begin, uint64_t lo, uint64_t hi, uint64_t dense_lim, uint32_t k,
                                          Hit& hit) {
    const unsigned long long lt = lanemask_lt64();
    while (__any(bits != 0)) {
        const bool has = bits != 0;
        const unsigned long long bal = __ballot(has);
        if (has) {
            const uint32_t idx = nb - 1 - __builtin_ctz(bits);
            bits &= bits - 1;
            q[qn + __popcll(bal & lt)] = base0 + (idx / U) * stride + (idx % U) * 64u + lane;
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= 64) {
            qn -= 64;
            __builtin_amdgcn_wave_barrier();
            resolve_block(dk, true, g_begin + q[qn + lane], lo, hi, dense_lim, k, cq, cqn, lane, hit);
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int U>
__device__ __forceinline__ void k1_body_bits(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi,
                                             uint64_t g_begin, uint64_t n_groups,
                                             unsigned long long* __restrict__ win, uint32_t* q, uint64_t* cq) {
    constexpr int W = 32 / U;  // iterations per push window (one bit per block)
    const uint32_t lane = threadIdx.x & 63;
    uint32_t qn = 0, cqn = 0;
    auto hit = [&](uint32_t j, uint64_t i) { atomicMax(&win[j], (unsigned long long)i); };
    const uint64_t dense_lim = 256ull * k;
    const uint32_t ng = (uint32_t)n_groups;  // < 2^31 per launch (host splits)
    // first offset whose block lies wholly in the sparse region (16 g + 1 >= 256 k): from there on
    // a block holds a candidate iff one of its 16 level-0 bytes is zero
    const uint64_t g_sparse = (dense_lim + 14) >> 4;
    const uint32_t off_sparse = g_sparse <= g_begin ? 0u : (uint32_t)std::min<uint64_t>(g_sparse - g_begin, ng);
    const uint32_t stride = gridDim.x * blockDim.x * U;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    // per-lane level-0 counter kept in VGPRs and stepped by `stride` (rebuilding it from a
    // scalar base every iteration made the compiler pad SALU->VALU hazards with 15 s_nop).  The
    // launch never crosses a multiple of 2^32 blocks (launch_k1_last_writer splits there), so the
    // counter's high word is one scalar for the whole launch: Philox round 0's first output and
    // round 1's first product are then wave-uniform and leave the VALU (19 -> 18 v_mad_u64_u32 and
    // 20 -> 19 v_bitop3 per block); only the low word is carried per lane.
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g_begin >> 32));
    uint32_t gl = (uint32_t)g_begin + base + lane;
    while (base < ng) {  // wave-uniform
        const uint32_t base0 = base;
        uint32_t bits = 0, nb = 0;
        for (int t = 0; t < W && base < ng; ++t, base += stride, gl += stride, nb += U) {
            u32x4 w[U];
            // block u's counter is gl + 64 u: the addend rides in the first product (no v_add)
#pragma unroll
            for (int u = 0; u < U; ++u)
                w[u] = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
            if (base >= off_sparse && base + U * 64 <= ng) {  // steady state: zero-byte test only
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    // some b_e == 0 <=> the 16-bit OR of the planes' halves is not all ones
                    const uint32_t x = w[u].x | w[u].y | w[u].z | w[u].w;
                    uint32_t y;
                    // (s_nop 0: the gfx950 SDWA wait state, see fold_pair in rsv_scan.h)
                    asm("v_or_b32_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                        "s_nop 0"
                        : "=v"(y) : "v"(x));
                    const bool has = (uint16_t)y != 0xFFFFu;
                    bits = bits + bits + (uint32_t)has;
                }
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t off = base + u * 64 + lane;
                    const bool has =
                        (off < ng) & (((((g_begin + off) << 4) + 1) < dense_lim) | any_zero_byte(w[u]));
                    bits = (bits << 1) | (uint32_t)has;
                }
            }
        }
        push_bits<U>(bits, nb, base0, stride, q, qn, cq, cqn, lane, dk, g_begin, lo, hi, dense_lim, k, hit);
    }
    drain_blocks(q, qn, cq, cqn, lane, dk, g_begin, lo, hi, dense_lim, k, hit);
}

// ---- K1 with the zero-byte mask carried in the queue (k1_body_z) -------------------------------
// k1_body_bits pushes a block's OFFSET, and the resolve recomputes its level-0 Philox to find the
// candidate bytes.  In the sparse region (i + 1 >= 256 k) a candidate is exactly a zero byte, so
// the 16-bit fold of the block's planes (y: bit e clear <=> b_e == 0) says everything the resolve
// needs: the main loop leaves y in an LDS window beside the bit, the push packs it into the queue
// entry, and the resolve goes straight to the level-1 draw with b = 0 -- no level-0 recompute, no
// byte extraction.  Dense-region blocks (i < 256 k) carry y = 0 (all bytes zero is impossible for
// a real block: probability 2^-128) and take the recomputing resolve.

constexpr uint32_t kK1ZWin = 20;  // blocks per lane per window (W x U); 16..32 within 2 us, 20 best (r02ad)

template <int U, int WIN = kK1ZWin>
__device__ __forceinline__ void k1_body_z(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                          uint64_t n_groups, unsigned long long* __restrict__ win, uint64_t* q,
                                          uint16_t* wy, uint32_t* tab, uint64_t* cq) {
    static_assert(WIN % U == 0 && WIN <= 32, "the window's bits fit one 32-bit mask");
    constexpr int W = WIN / U;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t qn = 0, cqn = 0;
    auto hit = [&](uint32_t j, uint64_t i) { atomicMax(&win[j], (unsigned long long)i); };
    const uint64_t dense_lim = 256ull * k;
    const uint32_t ng = (uint32_t)n_groups;  // < 2^31 per launch (host splits)
    const uint64_t g_sparse = (dense_lim + 14) >> 4;
    const uint32_t off_sparse = g_sparse <= g_begin ? 0u : (uint32_t)std::min<uint64_t>(g_sparse - g_begin, ng);
    const uint32_t stride = gridDim.x * blockDim.x * U;
    const uint32_t c1u = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(lo >> 33) | kDomainLevel1));
    const bool hi_uniform = (lo >> 33) == ((hi - 1) >> 33);
    const bool pre_ok = hi <= (1ull << 40);
    const uint64_t k_hi = (uint64_t)k << 32;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g_begin >> 32));
    uint32_t gl = (uint32_t)g_begin + base + lane;
    uint16_t* wyl = wy + lane;
    // window row b holds slot s = WIN-1-b: block base0 + (s / U) stride + (s % U) 64 + lane
    if (lane < WIN) tab[lane] = ((WIN - 1 - lane) / U) * stride + ((WIN - 1 - lane) % U) * 64u;
    __builtin_amdgcn_wave_barrier();
    // the steady branch holds blocks wholly inside [lo, hi) and the sparse region
    const uint32_t off_steady =
        __builtin_amdgcn_readfirstlane((int)std::max<uint32_t>(off_sparse, (lo & 15) ? 1u : 0u));
    const uint32_t ng_steady = __builtin_amdgcn_readfirstlane((int)(ng - ((hi & 15) ? 1u : 0u)));

    // all lanes take a queue entry (valid lanes only): its first zero byte gets the level-1 draw
    // here; a block with more (~3 % of blocks) goes back on the block queue with that byte masked
    // (y |= its bit), to be met again.  Clipped indices (outside [lo, hi)) were folded into y by
    // the main loop, so no entry needs a clip.
    auto resolve = [&](bool valid, uint64_t ent) {
        const uint32_t off = (uint32_t)ent, y = (uint32_t)(ent >> 32);
        const uint64_t g = g_begin + off, i0 = g << 4;
        const bool dense = valid && y == 0;
        if (__builtin_amdgcn_ballot_w64(dense)) resolve_block(dk, dense, g, lo, hi, dense_lim, k, cq, cqn, lane, hit);
        const uint32_t zm = (valid && !dense) ? (~y & 0xFFFFu) : 0u;
        uint32_t rest = 0;
        if (zm) {
            const uint32_t e = __builtin_ctz(zm);
            rest = zm & (zm - 1);
            const uint64_t i = i0 + e;
            const u32x4 w = level1_b0_words(dk, i, hi_uniform, c1u);
            const uint32_t Lh = (i & 1) ? w.z : w.x;
            // j >= floor((Lh >> 8) (i + 1) / 2^32) (the top 24 of L >> 8's 56 bits): when that
            // already reaches k the candidate loses (all but ~256 k / i of them); exact otherwise.
            // Needs (Lh >> 8) (i + 1) < 2^64: i < 2^40 for the whole launch (pre_ok, uniform).
            const bool maybe = !pre_ok || (uint64_t)(Lh >> 8) * (i + 1) < k_hi;
            if (maybe) {
                const uint64_t L = ((uint64_t)Lh << 32) | ((i & 1) ? w.w : w.y);
                const uint64_t j = __umul64hi(L >> 8, i + 1);
                if (j < k) hit((uint32_t)j, i);
            }
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(rest != 0);
        if (bal) {
            if (rest) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                q[qn + pos] = (uint64_t)off | ((uint64_t)(~rest & 0xFFFFu) << 32);
            }
            qn += (uint32_t)__popcll(bal);
        }
    };

    while (base < ng) {  // wave-uniform
        const uint32_t base0 = base;
        uint32_t bits = 0, nb = 0;
        if (base0 >= off_steady && (uint64_t)base0 + (uint64_t)(W - 1) * stride + U * 64 <= ng_steady) {
            // a whole window of steady iterations, unrolled: the window slot is an immediate LDS
            // offset, and the bit is shifted in by the compare's carry (v_cmp + v_addc: bits = 2 bits
            // + has) -- 5 VALU per block beside the Philox and one counter add per iteration
#pragma unroll
            for (int t = 0; t < W; ++t) {
                u32x4 w[U];
                const uint32_t gt = gl + t * stride;
#pragma unroll
                for (int u = 0; u < U; ++u)
                    w[u] = philox4x32_10_uniform_hi(gt, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t y = fold16(w[u]);
                    asm("v_cmp_ne_u32_e32 vcc, 0xffff, %1\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                        : "+v"(bits)
                        : "v"(y)
                        : "vcc");
                    wyl[(WIN - 1 - (t * U + u)) * 64] = (uint16_t)y;
                }
            }
            base += W * stride;
            gl += W * stride;
            nb = W * U;
        } else {  // a partial window (first, last, or where the dense / clipped blocks lie)
            for (int t = 0; t < W && base < ng; ++t, base += stride, gl += stride, nb += U) {
                u32x4 w[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    w[u] = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
                if (base >= off_steady && base + U * 64 <= ng_steady) {  // steady state: zero-byte test only
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t y = fold16(w[u]);
                        bits = bits + bits + (uint32_t)((uint16_t)y != 0xFFFFu);
                        wyl[(WIN - 1 - (t * U + u)) * 64] = (uint16_t)y;
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t off = base + u * 64 + lane;
                        const uint64_t i0 = (g_begin + off) << 4;
                        const bool dense = i0 + 1 < dense_lim;
                        // indices outside [lo, hi) count as nonzero bytes (never candidates)
                        const uint32_t y = dense ? 0u : (fold16(w[u]) | (~clip_mask16(i0, lo, hi) & 0xFFFFu));
                        const bool has = (off < ng) & (dense | ((uint16_t)y != 0xFFFFu));
                        bits = bits + bits + (uint32_t)has;
                        wyl[(WIN - 1 - (t * U + u)) * 64] = (uint16_t)y;
                    }
                }
            }
        }
        // push the window's marked blocks: each round every lane with bits left pushes its lowest.
        // Left-aligned, bit b is slot WIN-1-b: its fold is wy row b, its offset lbase + tab[b].
        bits <<= WIN - nb;
        const uint32_t lbase = base0 + lane;
        __builtin_amdgcn_wave_barrier();
        for (;;) {
            const bool has = bits != 0;
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(has);
            if (!bal) break;
            const uint32_t b = __builtin_ctz(bits | (1u << (WIN - 1)));  // (any row for a lane with none)
            bits &= bits - 1;
            const uint32_t off = lbase + tab[b];
            const uint32_t y = wyl[b * 64];
            RSV_K1P_COUNT(6, __popcll(bal));
            if (has) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                q[qn + pos] = (uint64_t)off | ((uint64_t)y << 32);
            }
            qn += (uint32_t)__popcll(bal);
            while (qn >= 64) {  // a resolve may append (blocks with more zero bytes)
                qn -= 64;
                __builtin_amdgcn_wave_barrier();
                const uint64_t ent = q[qn + lane];
                __builtin_amdgcn_wave_barrier();
                resolve(true, ent);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    while (qn > 0) {  // the last partial rounds (appends shrink geometrically)
        __builtin_amdgcn_wave_barrier();
        const uint32_t nv = std::min<uint32_t>(qn, 64u);
        qn -= nv;
        const bool valid = lane < nv;
        const uint64_t ent = valid ? q[qn + lane] : 0ull;
        __builtin_amdgcn_wave_barrier();
        resolve(valid, ent);
    }
    __builtin_amdgcn_wave_barrier();
    drain_queue(dk, cq, cqn, lane, k, hit);
}

// ---- K1 with pair entries (k1_body_p, rounds 3-4) ----------------------------------------------------------
// As k1_body_z (round 3; now tools/k1_dev_bodies.h), but a lane's two blocks of an iteration (offsets o and o + 64) share one window bit
// and one queue entry: the 32-bit fold z holds block o's 16-bit fold in its low half and block
// o + 64's in its high half (bit e clear <=> byte e & 15 of block o + 64 (e >> 4) is zero), built
// by two SDWA ops straight into the halves, and one compare marks the pair -- 4 VALU ops per block
// beside the Philox instead of 5, and half the window stores.  An entry's zero bytes are resolved
// one at a time as before.  A pair with a dense-region (or out-of-range-partner) half -- z half 0,
// impossible for a real sparse block (2^-128) -- takes the recomputing resolve for both blocks.
constexpr uint32_t kK1PWin = 10;  // iterations (pairs per lane) per window

template <int W = kK1PWin>
__device__ __forceinline__ void k1_body_p(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                          uint64_t n_groups, unsigned long long* __restrict__ win, uint64_t* q,
                                          uint32_t* wz, uint32_t* tab, uint64_t* cq) {
    static_assert(W <= 32, "the window's bits fit one 32-bit mask");
    constexpr int U = 2;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t qn = 0, cqn = 0;
    auto hit = [&](uint32_t j, uint64_t i) { atomicMax(&win[j], (unsigned long long)i); };
    const uint64_t dense_lim = 256ull * k;
    const uint32_t ng = (uint32_t)n_groups;  // < 2^31 per launch (host splits)
    const uint64_t g_sparse = (dense_lim + 14) >> 4;
    const uint32_t off_sparse = g_sparse <= g_begin ? 0u : (uint32_t)std::min<uint64_t>(g_sparse - g_begin, ng);
    const uint32_t stride = gridDim.x * blockDim.x * U;
    const uint32_t c1u = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(lo >> 33) | kDomainLevel1));
    const bool hi_uniform = (lo >> 33) == ((hi - 1) >> 33);
    const bool pre_ok = hi <= (1ull << 40);
    const uint64_t k_hi = (uint64_t)k << 32;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g_begin >> 32));
    uint32_t gl = (uint32_t)g_begin + base + lane;
    uint32_t* wzl = wz + lane;
    // window row b holds iteration W-1-b: pair base0 + (W-1-b) stride + lane (and + 64)
    if (lane < W) tab[lane] = (W - 1 - lane) * stride;
    __builtin_amdgcn_wave_barrier();
    const uint32_t off_steady =
        __builtin_amdgcn_readfirstlane((int)std::max<uint32_t>(off_sparse, (lo & 15) ? 1u : 0u));
    const uint32_t ng_steady = __builtin_amdgcn_readfirstlane((int)(ng - ((hi & 15) ? 1u : 0u)));

    auto resolve = [&](bool valid, uint64_t ent) {
        const uint32_t off = (uint32_t)ent, z = (uint32_t)(ent >> 32);
        const bool dense = valid && ((z & 0xFFFFu) == 0 || (z >> 16) == 0);
        RSV_K1P_COUNT(0, 1);
        RSV_K1P_COUNT(1, __popcll(__builtin_amdgcn_ballot_w64(valid)));
        if (__builtin_amdgcn_ballot_w64(dense)) {
            RSV_K1P_COUNT(2, 1);
            resolve_block(dk, dense, g_begin + off, lo, hi, dense_lim, k, cq, cqn, lane, hit);
            resolve_block(dk, dense && off + 64 < ng, g_begin + off + 64, lo, hi, dense_lim, k, cq, cqn, lane, hit);
        }
        const uint32_t zm = (valid && !dense) ? ~z : 0u;
        uint32_t rest = 0;
        if (zm) {
            const uint32_t e = __builtin_ctz(zm);
            rest = zm & (zm - 1);
            const uint64_t i = ((g_begin + off + ((e >> 4) << 6)) << 4) + (e & 15u);
            const u32x4 w = level1_b0_words(dk, i, hi_uniform, c1u);
            const uint32_t Lh = (i & 1) ? w.z : w.x;
            const bool maybe = !pre_ok || (uint64_t)(Lh >> 8) * (i + 1) < k_hi;
            if (maybe) {
                const uint64_t L = ((uint64_t)Lh << 32) | ((i & 1) ? w.w : w.y);
                const uint64_t j = __umul64hi(L >> 8, i + 1);
                if (j < k) hit((uint32_t)j, i);
            }
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(rest != 0);
        if (bal) {
            if (rest) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                q[qn + pos] = (uint64_t)off | ((uint64_t)~rest << 32);
            }
            qn += (uint32_t)__popcll(bal);
        }
    };

    while (base < ng) {  // wave-uniform
        const uint32_t base0 = base;
        uint32_t bits = 0, nb = 0;
        if (base0 >= off_steady && (uint64_t)base0 + (uint64_t)(W - 1) * stride + U * 64 <= ng_steady) {
#pragma unroll
            for (int t = 0; t < W; ++t) {
                const uint32_t gt = gl + t * stride;
                u32x4 w0, w1;
                philox4x32_10_uniform_hi_x2(gt, ghi, dk.s0, dk.s1, dk.k0, dk.k1, w0, w1);
                // fold_pair and the mark in ONE asm block (the hazard recognizer pads an s_nop
                // between adjacent inline-asm blocks; the two below are the SDWA wait states)
                const uint32_t xa = w0.x | w0.y | w0.z | w0.w, xb = w1.x | w1.y | w1.z | w1.w;
                uint32_t z;
                asm("v_or_b32_sdwa %0, %2, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                    "s_nop 0\n\t"
                    "v_or_b32_sdwa %0, %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                    "s_nop 0\n\t"
                    "v_cmp_ne_u32_e32 vcc, -1, %0\n\t"
                    "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
                    : "=&v"(z), "+v"(bits)
                    : "v"(xa), "v"(xb)
                    : "vcc");
                wzl[(W - 1 - t) * 64] = z;
            }
            base += W * stride;
            gl += W * stride;
            nb = W;
        } else {  // a partial window (first, last, or where the dense / clipped blocks lie)
            for (int t = 0; t < W && base < ng; ++t, base += stride, gl += stride, ++nb) {
                u32x4 w[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    w[u] = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
                uint32_t z;
                bool has;
                if (base >= off_steady && base + U * 64 <= ng_steady) {
                    z = fold_pair(w[0], w[1]);
                    has = z != 0xFFFFFFFFu;
                } else {
                    uint32_t y[U];
                    bool h[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t off = base + u * 64 + lane;
                        const uint64_t i0 = (g_begin + off) << 4;
                        const bool dense = i0 + 1 < dense_lim;
                        // indices outside [lo, hi) count as nonzero bytes (never candidates); a
                        // block past the launch is no candidate and not dense
                        y[u] = off >= ng ? 0xFFFFu
                                         : dense ? 0u : (fold16(w[u]) | (~clip_mask16(i0, lo, hi) & 0xFFFFu));
                        h[u] = (off < ng) & (dense | ((uint16_t)y[u] != 0xFFFFu));
                    }
                    z = (y[0] & 0xFFFFu) | (y[1] << 16);
                    has = h[0] | h[1];
                }
                bits = bits + bits + (uint32_t)has;
                wzl[(W - 1 - t) * 64] = z;
            }
        }
        // push the window's marked pairs: each round every lane with bits left pushes its lowest.
        // Left-aligned, bit b is row b: its fold is wz row b, its offset lbase + tab[b].
        bits <<= W - nb;
        const uint32_t lbase = base0 + lane;
        __builtin_amdgcn_wave_barrier();
        RSV_K1P_COUNT(3, 1);
        for (;;) {
            const bool has = bits != 0;
            const unsigned long long bal = __builtin_amdgcn_ballot_w64(has);
            if (!bal) break;
            RSV_K1P_COUNT(4, 1);
            RSV_K1P_COUNT(5, __popcll(bal));
            const uint32_t b = __builtin_ctz(bits | (1u << (W - 1)));  // (any row for a lane with none)
            bits &= bits - 1;
            const uint32_t off = lbase + tab[b];
            const uint32_t z = wzl[b * 64];
            if (has) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                q[qn + pos] = (uint64_t)off | ((uint64_t)z << 32);
            }
            qn += (uint32_t)__popcll(bal);
            while (qn >= 64) {  // a resolve may append (pairs with more zero bytes)
                qn -= 64;
                __builtin_amdgcn_wave_barrier();
                const uint64_t ent = q[qn + lane];
                __builtin_amdgcn_wave_barrier();
                resolve(true, ent);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    while (qn > 0) {  // the last partial rounds (appends shrink geometrically)
        __builtin_amdgcn_wave_barrier();
        const uint32_t nv = std::min<uint32_t>(qn, 64u);
        qn -= nv;
        const bool valid = lane < nv;
        const uint64_t ent = valid ? q[qn + lane] : 0ull;
        __builtin_amdgcn_wave_barrier();
        resolve(valid, ent);
    }
    __builtin_amdgcn_wave_barrier();
    drain_queue(dk, cq, cqn, lane, k, hit);
}

// ---- the round-5 k1_body_q (each wave resolves its own leftovers) with a cost probe: SKIP_TAIL
// leaves out the final partial rounds (WRONG winners; tools/micro_k1o t) -----------------------------
template <int W = 12, bool FAST = false, bool SKIP_TAIL = false>
__device__ __forceinline__ void k1_body_q_dev(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                          uint64_t n_groups, unsigned long long* __restrict__ win, uint64_t* q,
                                          uint64_t* cq) {
    static_assert(W % 2 == 0, "half windows");
    constexpr int U = 2;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t qn = 0, cqn = 0;
    auto hit = [&](uint32_t j, uint64_t i) { atomicMax(&win[j], (unsigned long long)i); };
    const uint64_t dense_lim = 256ull * k;
    const uint32_t ng = (uint32_t)n_groups;  // < 2^31 per launch (host splits)
    const uint64_t g_sparse = (dense_lim + 14) >> 4;
    const uint32_t off_sparse = g_sparse <= g_begin ? 0u : (uint32_t)std::min<uint64_t>(g_sparse - g_begin, ng);
    const uint32_t stride = gridDim.x * blockDim.x * U;
    const uint32_t c1u = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(lo >> 33) | kDomainLevel1));
    const bool hi_uniform = (lo >> 33) == ((hi - 1) >> 33);
    const bool pre_ok = hi <= (1ull << 40);
    const uint64_t k_hi = (uint64_t)k << 32;
    const uint32_t g0 = (uint32_t)g_begin;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g_begin >> 32));
    uint32_t gl = g0 + base + lane;
    const uint32_t off_steady =
        __builtin_amdgcn_readfirstlane((int)std::max<uint32_t>(off_sparse, (lo & 15) ? 1u : 0u));
    const uint32_t ng_steady = __builtin_amdgcn_readfirstlane((int)(ng - ((hi & 15) ? 1u : 0u)));

    // one queue entry per lane (valid lanes): its pair's first zero byte by level 1; the pair's other
    // zero bytes go back to the queue; a dense / clipped pair (a z half 0) recomputes both blocks
    auto resolve = [&](bool valid, uint64_t ent) {
        const uint32_t gt = (uint32_t)ent, off = gt - g0, z = (uint32_t)(ent >> 32);
        const bool dense = valid && ((z & 0xFFFFu) == 0 || (z >> 16) == 0);
        if (__builtin_amdgcn_ballot_w64(dense)) {
            resolve_block(dk, dense, g_begin + off, lo, hi, dense_lim, k, cq, cqn, lane, hit);
            resolve_block(dk, dense && off + 64 < ng, g_begin + off + 64, lo, hi, dense_lim, k, cq, cqn, lane, hit);
        }
        const uint32_t zm = (valid && !dense) ? ~z : 0u;
        uint32_t rest = 0;
        if (zm) {
            const uint32_t e = __builtin_ctz(zm);
            rest = zm & (zm - 1);
            if constexpr (FAST) {
                // the zero byte's block ghi:bl (bl = gt or gt + 64: never crosses the launch's
                // 2^32-block span); level-1 counter i >> 1 = ghi:bl:(e & 15) >> 1, low word below
                const uint32_t bl = gt + ((e & 16u) << 2);
                const uint32_t g1lo = (bl << 3) | ((e & 15u) >> 1);
                const u32x4 w = philox4x32_10_uniform_hi(g1lo, c1u, dk.s0, dk.s1, dk.k0, dk.k1);
                const uint64_t i = ((((uint64_t)ghi << 32) | bl) << 4) | (e & 15u);
                const bool odd = e & 1u;
                const uint32_t Lh = odd ? w.z : w.x;
                if ((uint64_t)(Lh >> 8) * (i + 1) < k_hi) {
                    const uint64_t L = ((uint64_t)Lh << 32) | (odd ? w.w : w.y);
                    const uint64_t j = __umul64hi(L >> 8, i + 1);
                    if (j < k) hit((uint32_t)j, i);
                }
            } else {
                const uint64_t i = ((g_begin + off + ((e >> 4) << 6)) << 4) + (e & 15u);
                const u32x4 w = level1_b0_words(dk, i, hi_uniform, c1u);
                const uint32_t Lh = (i & 1) ? w.z : w.x;
                const bool maybe = !pre_ok || (uint64_t)(Lh >> 8) * (i + 1) < k_hi;
                if (maybe) {
                    const uint64_t L = ((uint64_t)Lh << 32) | ((i & 1) ? w.w : w.y);
                    const uint64_t j = __umul64hi(L >> 8, i + 1);
                    if (j < k) hit((uint32_t)j, i);
                }
            }
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(rest != 0);
        if (bal) {
            if (rest) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                q[qn + pos] = (uint64_t)(uint32_t)ent | ((uint64_t)~rest << 32);
            }
            qn += (uint32_t)__popcll(bal);
        }
    };
    auto rounds = [&]() {
        while (qn >= 64) {  // a resolve may append (pairs with more zero bytes)
            qn -= 64;
            __builtin_amdgcn_wave_barrier();
            const uint64_t ent = q[qn + lane];
            __builtin_amdgcn_wave_barrier();
            resolve(true, ent);
            __builtin_amdgcn_wave_barrier();
        }
    };
    // append this lane's pair (counter word gt, fold z) when has; wave-uniform call
    auto append = [&](bool has, uint32_t gt, uint32_t z) {
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(has);
        if (has) {
            const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            q[qn + pos] = (uint64_t)gt | ((uint64_t)z << 32);
        }
        qn += (uint32_t)__popcll(bal);
    };

    // the wave's queue base as a scalar (LDS addresses are 32-bit), so an append's address is one
    // v_lshl_add of the lane's slot onto base + 8 qn
    const uint32_t q_s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)q);
    while (base < ng) {  // wave-uniform
        if (base >= off_steady && (uint64_t)base + (uint64_t)(W - 1) * stride + U * 64 <= ng_steady) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int t = 0; t < W / 2; ++t) {
                    const uint32_t gt = gl + t * stride;
                    u32x4 w0, w1;
                    philox4x32_10_uniform_hi_x2(gt, ghi, dk.s0, dk.s1, dk.k0, dk.k1, w0, w1);
                    // the pair fold (with the gfx950 SDWA wait states, fold_pair) and its mark as a
                    // lane mask in one asm block
                    const uint32_t xa = w0.x | w0.y | w0.z | w0.w, xb = w1.x | w1.y | w1.z | w1.w;
                    uint32_t z;
                    unsigned long long m;
                    asm("v_or_b32_sdwa %0, %2, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                        "s_nop 0\n\t"
                        "v_or_b32_sdwa %0, %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                        "s_nop 0\n\t"
                        "v_cmp_ne_u32_e64 %1, -1, %0"
                        : "=&v"(z), "=s"(m)
                        : "v"(xa), "v"(xb));
                    const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    // the marked lanes store (exec = m inside the asm, restored before it ends; one
                    // wave's LDS operations complete in order, so the rounds' reads see the entries)
                    const uint32_t sb = q_s + 8u * qn;
                    const uint64_t ent = (uint64_t)gt | ((uint64_t)z << 32);
                    unsigned long long sv;
                    uint32_t addr;
                    asm volatile("v_lshl_add_u32 %1, %2, 3, %3\n\t"
                                 "s_mov_b64 %0, exec\n\t"
                                 "s_mov_b64 exec, %4\n\t"
                                 "ds_write_b64 %1, %5\n\t"
                                 "s_mov_b64 exec, %0"
                                 : "=&s"(sv), "=&v"(addr)
                                 : "v"(pos), "s"(sb), "s"(m), "v"(ent)
                                 : "memory");
                    qn += (uint32_t)__popcll(m);
                }
                gl += (W / 2) * stride;
                __builtin_amdgcn_wave_barrier();
                rounds();
            }
            base += W * stride;
        } else {  // a partial window (first, last, or where the dense / clipped blocks lie)
            for (int t = 0; t < W && base < ng; ++t, base += stride, gl += stride) {
                u32x4 w[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    w[u] = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
                uint32_t z;
                bool has;
                if (base >= off_steady && base + U * 64 <= ng_steady) {
                    z = fold_pair(w[0], w[1]);
                    has = z != 0xFFFFFFFFu;
                } else {
                    uint32_t y[U];
                    bool hb[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t off = base + u * 64 + lane;
                        const uint64_t i0 = (g_begin + off) << 4;
                        const bool dense = i0 + 1 < dense_lim;
                        // indices outside [lo, hi) count as nonzero bytes (never candidates); a
                        // block past the launch is no candidate and not dense
                        y[u] = off >= ng ? 0xFFFFu
                                         : dense ? 0u : (fold16(w[u]) | (~clip_mask16(i0, lo, hi) & 0xFFFFu));
                        hb[u] = (off < ng) & (dense | ((uint16_t)y[u] != 0xFFFFu));
                    }
                    z = (y[0] & 0xFFFFu) | (y[1] << 16);
                    has = hb[0] | hb[1];
                }
                append(has, gl, z);
                __builtin_amdgcn_wave_barrier();
                rounds();
            }
        }
    }
    if (SKIP_TAIL) return;  // cost probe: WRONG winners
    while (qn > 0) {  // the last partial rounds (appends shrink geometrically)
        __builtin_amdgcn_wave_barrier();
        const uint32_t nv = std::min<uint32_t>(qn, 64u);
        qn -= nv;
        const bool valid = lane < nv;
        const uint64_t ent = valid ? q[qn + lane] : 0ull;
        __builtin_amdgcn_wave_barrier();
        resolve(valid, ent);
    }
    __builtin_amdgcn_wave_barrier();
    drain_queue(dk, cq, cqn, lane, k, hit);
}

// ---- k1_body_q over a static two-group schedule (round 5 probe; the product took it, rsv_scan.h).  The launch's half windows (units
// of W/2 iterations, 768 contiguous blocks) go to waves in order: the first W1 waves take A units
// each, the rest B each -- so the first generation of resident workgroups can run long (fewer
// waves, fewer final partial rounds: 4.4 us of the 5086-workgroup launch) while the last
// generation stays short (the launch's end waits for the last workgroups).  A first try claimed
// units dynamically from one global counter: 1.05 ms per launch -- ~87 k same-address atomics
// serialise at ~12 ns each (profiles/r05/micro_k1o_dyn_claims.jsonl). ---------------------------------
template <int W = 12, bool FAST = false>
__device__ __forceinline__ void k1_body_q_sched(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                              uint64_t n_groups, unsigned long long* __restrict__ win, uint64_t* q,
                                              uint64_t* cq, uint32_t W1, uint32_t A, uint32_t B) {
    static_assert(W % 2 == 0, "half windows");
    constexpr int U = 2;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t qn = 0, cqn = 0;
    auto hit = [&](uint32_t j, uint64_t i) { atomicMax(&win[j], (unsigned long long)i); };
    const uint64_t dense_lim = 256ull * k;
    const uint32_t ng = (uint32_t)n_groups;  // < 2^31 per launch (host splits)
    const uint64_t g_sparse = (dense_lim + 14) >> 4;
    const uint32_t off_sparse = g_sparse <= g_begin ? 0u : (uint32_t)std::min<uint64_t>(g_sparse - g_begin, ng);
    const uint32_t stride = gridDim.x * blockDim.x * U;
    const uint32_t c1u = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(lo >> 33) | kDomainLevel1));
    const bool hi_uniform = (lo >> 33) == ((hi - 1) >> 33);
    const bool pre_ok = hi <= (1ull << 40);
    const uint64_t k_hi = (uint64_t)k << 32;
    const uint32_t g0 = (uint32_t)g_begin;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g_begin >> 32));
    uint32_t gl = g0 + base + lane;
    const uint32_t off_steady =
        __builtin_amdgcn_readfirstlane((int)std::max<uint32_t>(off_sparse, (lo & 15) ? 1u : 0u));
    const uint32_t ng_steady = __builtin_amdgcn_readfirstlane((int)(ng - ((hi & 15) ? 1u : 0u)));

    // one queue entry per lane (valid lanes): its pair's first zero byte by level 1; the pair's other
    // zero bytes go back to the queue; a dense / clipped pair (a z half 0) recomputes both blocks
    auto resolve = [&](bool valid, uint64_t ent) {
        const uint32_t gt = (uint32_t)ent, off = gt - g0, z = (uint32_t)(ent >> 32);
        const bool dense = valid && ((z & 0xFFFFu) == 0 || (z >> 16) == 0);
        if (__builtin_amdgcn_ballot_w64(dense)) {
            resolve_block(dk, dense, g_begin + off, lo, hi, dense_lim, k, cq, cqn, lane, hit);
            resolve_block(dk, dense && off + 64 < ng, g_begin + off + 64, lo, hi, dense_lim, k, cq, cqn, lane, hit);
        }
        const uint32_t zm = (valid && !dense) ? ~z : 0u;
        uint32_t rest = 0;
        if (zm) {
            const uint32_t e = __builtin_ctz(zm);
            rest = zm & (zm - 1);
            if constexpr (FAST) {
                // the zero byte's block ghi:bl (bl = gt or gt + 64: never crosses the launch's
                // 2^32-block span); level-1 counter i >> 1 = ghi:bl:(e & 15) >> 1, low word below
                const uint32_t bl = gt + ((e & 16u) << 2);
                const uint32_t g1lo = (bl << 3) | ((e & 15u) >> 1);
                const u32x4 w = philox4x32_10_uniform_hi(g1lo, c1u, dk.s0, dk.s1, dk.k0, dk.k1);
                const uint64_t i = ((((uint64_t)ghi << 32) | bl) << 4) | (e & 15u);
                const bool odd = e & 1u;
                const uint32_t Lh = odd ? w.z : w.x;
                if ((uint64_t)(Lh >> 8) * (i + 1) < k_hi) {
                    const uint64_t L = ((uint64_t)Lh << 32) | (odd ? w.w : w.y);
                    const uint64_t j = __umul64hi(L >> 8, i + 1);
                    if (j < k) hit((uint32_t)j, i);
                }
            } else {
                const uint64_t i = ((g_begin + off + ((e >> 4) << 6)) << 4) + (e & 15u);
                const u32x4 w = level1_b0_words(dk, i, hi_uniform, c1u);
                const uint32_t Lh = (i & 1) ? w.z : w.x;
                const bool maybe = !pre_ok || (uint64_t)(Lh >> 8) * (i + 1) < k_hi;
                if (maybe) {
                    const uint64_t L = ((uint64_t)Lh << 32) | ((i & 1) ? w.w : w.y);
                    const uint64_t j = __umul64hi(L >> 8, i + 1);
                    if (j < k) hit((uint32_t)j, i);
                }
            }
        }
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(rest != 0);
        if (bal) {
            if (rest) {
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                q[qn + pos] = (uint64_t)(uint32_t)ent | ((uint64_t)~rest << 32);
            }
            qn += (uint32_t)__popcll(bal);
        }
    };
    auto rounds = [&]() {
        while (qn >= 64) {  // a resolve may append (pairs with more zero bytes)
            qn -= 64;
            __builtin_amdgcn_wave_barrier();
            const uint64_t ent = q[qn + lane];
            __builtin_amdgcn_wave_barrier();
            resolve(true, ent);
            __builtin_amdgcn_wave_barrier();
        }
    };
    // append this lane's pair (counter word gt, fold z) when has; wave-uniform call
    auto append = [&](bool has, uint32_t gt, uint32_t z) {
        const unsigned long long bal = __builtin_amdgcn_ballot_w64(has);
        if (has) {
            const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            q[qn + pos] = (uint64_t)gt | ((uint64_t)z << 32);
        }
        qn += (uint32_t)__popcll(bal);
    };

    // the wave's queue base as a scalar (LDS addresses are 32-bit), so an append's address is one
    // v_lshl_add of the lane's slot onto base + 8 qn
    const uint32_t q_s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)q);
    constexpr uint32_t UB = (W / 2) * U * 64;
    const uint32_t units = (ng + UB - 1) / UB;
    (void)base;
    (void)stride;
    // strided within each group (unit j * group_waves + wave): the launch's first units -- the dense
    // region, many times a sparse unit's work -- go one per wave to the first-dispatched waves
    const uint32_t wg = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t nB = gridDim.x * (blockDim.x >> 6) - W1;
    const bool ga = wg < W1;
    const uint32_t cnt = ga ? A : B, u_step = ga ? W1 : nB, u_first = ga ? wg : W1 * A + (wg - W1);
    for (uint32_t j = 0; j < cnt; ++j) {  // wave-uniform
        const uint32_t u = u_first + j * u_step;
        if (u >= units) break;
        uint32_t ub = u * UB;
        gl = g0 + ub + lane;
        if (ub >= off_steady && ub + UB <= ng_steady) {
#pragma unroll
            for (int t = 0; t < W / 2; ++t) {
                const uint32_t gt = gl + t * (U * 64);
                u32x4 w0, w1;
                philox4x32_10_uniform_hi_x2(gt, ghi, dk.s0, dk.s1, dk.k0, dk.k1, w0, w1);
                const uint32_t xa = w0.x | w0.y | w0.z | w0.w, xb = w1.x | w1.y | w1.z | w1.w;
                uint32_t z;
                unsigned long long m;
                asm("v_or_b32_sdwa %0, %2, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                    "s_nop 0\n\t"
                    "v_or_b32_sdwa %0, %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
                    "s_nop 0\n\t"
                    "v_cmp_ne_u32_e64 %1, -1, %0"
                    : "=&v"(z), "=s"(m)
                    : "v"(xa), "v"(xb));
                const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                const uint32_t sb = q_s + 8u * qn;
                const uint64_t ent = (uint64_t)gt | ((uint64_t)z << 32);
                unsigned long long sv;
                uint32_t addr;
                asm volatile("v_lshl_add_u32 %1, %2, 3, %3\n\t"
                             "s_mov_b64 %0, exec\n\t"
                             "s_mov_b64 exec, %4\n\t"
                             "ds_write_b64 %1, %5\n\t"
                             "s_mov_b64 exec, %0"
                             : "=&s"(sv), "=&v"(addr)
                             : "v"(pos), "s"(sb), "s"(m), "v"(ent)
                             : "memory");
                qn += (uint32_t)__popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
            rounds();
        } else {  // a unit holding the dense / clipped blocks or the launch's end
            for (int t = 0; t < W / 2 && ub < ng; ++t, ub += U * 64, gl += U * 64) {
                u32x4 w[U];
#pragma unroll
                for (int v = 0; v < U; ++v)
                    w[v] = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * v));
                uint32_t y[U];
                bool hb[U];
#pragma unroll
                for (int v = 0; v < U; ++v) {
                    const uint32_t off = ub + v * 64 + lane;
                    const uint64_t i0 = (g_begin + off) << 4;
                    const bool dense = i0 + 1 < dense_lim;
                    y[v] = off >= ng ? 0xFFFFu
                                     : dense ? 0u : (fold16(w[v]) | (~clip_mask16(i0, lo, hi) & 0xFFFFu));
                    hb[v] = (off < ng) & (dense | ((uint16_t)y[v] != 0xFFFFu));
                }
                const uint32_t z = (y[0] & 0xFFFFu) | (y[1] << 16);
                append(hb[0] | hb[1], gl, z);
                __builtin_amdgcn_wave_barrier();
                rounds();
            }
        }
    }
    while (qn > 0) {  // the last partial rounds (appends shrink geometrically)
        __builtin_amdgcn_wave_barrier();
        const uint32_t nv = std::min<uint32_t>(qn, 64u);
        qn -= nv;
        const bool valid = lane < nv;
        const uint64_t ent = valid ? q[qn + lane] : 0ull;
        __builtin_amdgcn_wave_barrier();
        resolve(valid, ent);
    }
    __builtin_amdgcn_wave_barrier();
    drain_queue(dk, cq, cqn, lane, k, hit);
}

}  // namespace rsv
