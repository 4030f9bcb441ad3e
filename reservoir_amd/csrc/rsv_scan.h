// rsv_scan.h -- the level-0 scan shared by K1 (one stream) and K2 (segmented): evaluate the 16-
// index level-0 Philox blocks, and push the ~1/256 candidate indices through a per-wave LDS queue
// so the level-1 Philox (exact j) always runs with all 64 lanes busy.
//
// Without the queue the candidates are evaluated where they are found: almost every wave
// iteration holds one (64 lanes x 16 indices / 256), so the whole wave pays a second Philox for a
// single active lane -- measured 383 us vs ~120 us for the level-0 work alone at 1e9 indices.
#pragma once
#include <algorithm>

#include "rsv_device.h"

namespace rsv {

constexpr uint32_t kQueue = 128;  // per-wave LDS entries: < 64 waiting + one round of <= 64 pushes
constexpr uint64_t kIndexMask = (1ull << 56) - 1;  // queue entry = (b_i << 56) | i

__device__ __forceinline__ unsigned long long lanemask_lt64() {
    const uint32_t lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

__device__ __forceinline__ uint32_t clip_mask16(uint64_t i0, uint64_t lo, uint64_t hi) {
    uint32_t m = 0xFFFFu;
    if (i0 < lo) m = (lo - i0 >= 16) ? 0u : ((0xFFFFu << (uint32_t)(lo - i0)) & 0xFFFFu);
    if (i0 + 16 > hi) m &= (hi <= i0) ? 0u : (0xFFFFu >> (uint32_t)(16 - (hi - i0)));
    return m;
}

// Candidate mask of one level-0 block: bit e set if b_{i0+e} * (i0+e+1) < 256k may hold (a
// necessary condition for j < k).  Beyond index 256k-1 this is exactly "b == 0" (1 in 256).  In
// the dense region (K2's whole 4096-element streams at k = 64) the bit-sliced test "b < T" with
// the block's threshold T = ceil(256k / (i0+1)) gives a superset for the block's 16 indices (exact
// for the first); the level-1 draw decides every candidate exactly.
__device__ __forceinline__ uint32_t candidate_mask16(const u32x4& w, uint64_t i0, uint64_t dense_lim) {
    if (i0 + 1 >= dense_lim) return zero_byte_mask16(w);
    // T = ceil(dense_lim / (i0+1)): the fp32 estimate is within a few units; correct it exactly
    const float Tf = __fdividef((float)dense_lim, (float)(i0 + 1));
    if (Tf > 300.0f) return 0xFFFFu;  // T > 256: every byte qualifies
    // Tf <= 300: its error is far below one unit, so one step each way makes T exact
    uint32_t T = (uint32_t)Tf;
    if ((uint64_t)T * (i0 + 1) < dense_lim) ++T;
    if (T > 0 && (uint64_t)(T - 1) * (i0 + 1) >= dense_lim) --T;
    return lt_mask16(w, T > 256u ? 256u : T);
}

// Evaluate queue entry q[pos] (level 1) and report a hit (j < k) to `hit(j, i)`.
template <class Hit>
__device__ __forceinline__ void resolve_entry(const DrawKey& dk, uint64_t e, uint32_t k, Hit& hit) {
    const uint64_t i = e & kIndexMask;
    const uint64_t j = exact_j(dk, i, (uint32_t)(e >> 56));
    if (j < k) hit((uint32_t)j, i);
}

// Push this lane's candidates (mask over the block starting at i0) into the wave queue; whenever
// 64 entries wait, all lanes resolve one each.  Must be called by the whole wave (uniform flow).
template <class Hit>
__device__ __forceinline__ void enqueue_block(const DrawKey& dk, const u32x4& w, uint64_t i0,
                                              uint32_t mask, uint64_t* q, uint32_t& qn,
                                              uint32_t lane, uint32_t k, Hit& hit) {
    while (__any(mask != 0)) {
        const bool has = mask != 0;
        const unsigned long long bal = __ballot(has);
        if (has) {
            const uint32_t e = __builtin_ctz(mask);
            mask &= mask - 1;
            q[qn + __popcll(bal & lanemask_lt64())] = ((uint64_t)level0_byte(w, e) << 56) | (i0 + e);
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= 64) {
            qn -= 64;
            __builtin_amdgcn_wave_barrier();
            resolve_entry(dk, q[qn + lane], k, hit);
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <class Hit>
__device__ __forceinline__ void drain_queue(const DrawKey& dk, const uint64_t* q, uint32_t& qn,
                                            uint32_t lane, uint32_t k, Hit& hit) {
    __builtin_amdgcn_wave_barrier();
    if (lane < qn) resolve_entry(dk, q[lane], k, hit);
    qn = 0;
    __builtin_amdgcn_wave_barrier();
}

// ---- block queue (K1): a wave iteration pushes the OFFSETS of level-0 blocks that hold a candidate
// In K1's sparse region (index >= 256k) a block holds a candidate only if one of its 16 bytes is
// zero (6% of blocks, but ~98% of wave iterations see at least one), so whatever is done per
// pushed block is paid by the whole wave nearly every iteration.  The iteration therefore only
// tests "any zero byte" and pushes a 32-bit block offset; at drain time the wave recomputes the
// level-0 block (one Philox per 64 pushed blocks per lane), decodes it and runs the level-1 draws,
// 64 blocks at once.  (Pushing the raw 24-B block instead cost 28 us per 1e9 indices.)

// Resolve queued block g (valid lanes only; the call is wave-uniform): the block's FIRST candidate
// is evaluated in place by every lane at once; further candidates of the same block (about 3 % of
// sparse blocks -- but 86 % of 64-block drains hold one) go to the per-candidate queue `cq`, so a
// lone second candidate does not cost the whole wave another level-1 Philox.
template <class Hit>
__device__ __forceinline__ void resolve_block(const DrawKey& dk, bool valid, uint64_t g, uint64_t lo,
                                              uint64_t hi, uint64_t dense_lim, uint32_t k, uint64_t* cq,
                                              uint32_t& cqn, uint32_t lane, Hit& hit) {
    const u32x4 w = level0(dk, g);
    const uint64_t i0 = g << 4;
    uint32_t mask = valid ? candidate_mask16(w, i0, dense_lim) : 0u;
    if (i0 < lo || i0 + 16 > hi) mask &= clip_mask16(i0, lo, hi);
    if (mask) {
        const uint32_t e = __builtin_ctz(mask);
        mask &= mask - 1;
        const uint64_t j = exact_j(dk, i0 + e, level0_byte(w, e));
        if (j < k) hit((uint32_t)j, i0 + e);
    }
    enqueue_block(dk, w, i0, mask, cq, cqn, lane, k, hit);
}

// the 16-bit OR of a block's plane halves: bit e clear <=> b_e == 0 (one SDWA op for the fold; the
// wait state after it keeps a reader right behind from the gfx950 SDWA hazard, see fold_pair)
__device__ __forceinline__ uint32_t fold16(const u32x4& w) {
    const uint32_t x = w.x | w.y | w.z | w.w;
    uint32_t y;
    asm("v_or_b32_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "s_nop 0"
        : "=v"(y)
        : "v"(x));
    return y;
}

// level-1 draw of a sparse-region candidate (b = 0): j = floor((L >> 8) (i + 1) / 2^64).
// The level-1 Philox words of index i (L = words x:y for even i, z:w for odd).  hi_uniform (wave-
// uniform): the counter's high word (i / 2^33) is the same for the whole launch.
__device__ __forceinline__ u32x4 level1_b0_words(const DrawKey& dk, uint64_t i, bool hi_uniform, uint32_t c1u) {
    const uint64_t g1 = i >> 1;
    if (hi_uniform) return philox4x32_10_uniform_hi((uint32_t)g1, c1u, dk.s0, dk.s1, dk.k0, dk.k1);
    return philox4x32_10((uint32_t)g1, (uint32_t)(g1 >> 32) | kDomainLevel1, dk.s0, dk.s1, dk.k0, dk.k1);
}

// z = fold16(a) | fold16(b) << 16.  The wait states are part of the block: on gfx950 a VALU op
// reading a register right after an SDWA op wrote part of it reads the OLD value (tools/micro_k1o
// fold_check: 21 % wrong without them, none with one s_nop 0 each).
__device__ __forceinline__ uint32_t fold_pair(const u32x4& a, const u32x4& b) {
    const uint32_t xa = a.x | a.y | a.z | a.w, xb = b.x | b.y | b.z | b.w;
    uint32_t z;
    asm("v_or_b32_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "s_nop 0\n\t"
        "v_or_b32_sdwa %0, %2, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "s_nop 0"
        : "=&v"(z)
        : "v"(xa), "v"(xb));
    return z;
}

// ---- K1 with direct appends (k1_body_q, round 5) -----------------------------------------------
// k1_body_p marks a window's pairs in a per-lane bit mask and pushes them afterwards in ballot
// rounds (one entry per lane per round: ~5 rounds of ~14 VALU per 12-iteration window, the max
// over 64 lanes of a Binomial(12, 0.118)).  Here every iteration appends its marked pairs at once:
// the compare's lane mask IS the ballot, so an append is two mbcnt + one address op under that
// mask, and the window keeps no fold rows or offset table.  The entry carries the pair's Philox
// counter word gt (the launch never crosses a 2^32-block boundary, so the block is ghi:gt) and its
// fold.  The queue holds < 64 waiting entries + half a window of appends (k1q_cap): the rounds run
// after each half window.  The steady append takes no branch (the store runs under exec = the mark
// inside one asm block), so the unrolled window stays one basic block for the scheduler.
template <int W>
constexpr uint32_t k1q_cap() { return 64u * (1u + W / 2); }
// waves per K1 workgroup (256 threads): the pooled tail's per-wave queue count
constexpr uint32_t kQueueWaves = 4;

// FAST (launch-uniform, the kernel picks): the level-1 counter's high word is uniform over the
// launch and every index is below 2^40 -- the resolve then forms the counter's low word with
// 32-bit ops from the entry's counter word instead of the general 64-bit index arithmetic.
//
// Two work layouts (launch-uniform): A == 0 -- grid-stride over whole windows (every wave the same
// number of iterations); A > 0 -- a static two-group schedule of half windows (units of W/2
// iterations over 768 contiguous blocks): the first W1 waves take A units each, the rest B each,
// strided within each group (unit j * group_waves + wave, so the launch's first units -- the dense
// region, many times a sparse unit's work -- go one per wave to the first-dispatched waves).  The
// first generation of resident workgroups then runs long (fewer waves: every wave ends on one or two
// partial resolve rounds, 4.4 us of an 83 us launch at 20 k waves -- tools/micro_k1o t), the last
// stays short (the launch's end waits on the last workgroups): tools/micro_k1o s, 1e9 draws:
// 81.7-81.8 us at (6144, 10, 2) vs 83.0-83.2 for the grid-stride launch (profiles/r05/).
template <int W = 12, bool FAST = false>
__device__ __forceinline__ void k1_body_q(const DrawKey& dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                          uint64_t n_groups, unsigned long long* __restrict__ win, uint64_t* q,
                                          uint64_t* cq, uint32_t W1 = 0, uint32_t A = 0, uint32_t B = 0,
                                          uint32_t* pool = nullptr) {
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
    const uint64_t k_hi = (uint64_t)k << 32, k_24 = (uint64_t)k << 24;
    int32_t dpend = 0;  // dense entries appended and not yet resolved (wave-uniform)
    const uint32_t g0 = (uint32_t)g_begin;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g_begin >> 32));
    uint32_t gl = g0 + base + lane;
    const uint32_t off_steady =
        __builtin_amdgcn_readfirstlane((int)std::max<uint32_t>(off_sparse, (lo & 15) ? 1u : 0u));
    const uint32_t ng_steady = __builtin_amdgcn_readfirstlane((int)(ng - ((hi & 15) ? 1u : 0u)));

    // one queue entry per lane (valid lanes): its pair's first zero byte by level 1; the pair's other
    // zero bytes go back to the queue; a dense / clipped pair (a z half 0) recomputes both blocks.  An
    // entry's low word is lo(M0 gt) (what the steady pair's round 0 already holds), so gt = lo M0^-1.
    auto resolve = [&](bool valid, uint64_t ent) {
        const uint32_t gt = (uint32_t)ent * kPhiloxM0Inv, off = gt - g0, z = (uint32_t)(ent >> 32);
        // every queued entry holds a zero byte or a dense half (its fold is never all ones): a full
        // round (valid) needs no zm != 0 test
        __builtin_assume(!valid || z != 0xFFFFFFFFu);
        // the dense test only while a partial iteration's dense entries are pending (the steady
        // loop appends none: a steady pair with a zero fold half would need 16 zero bytes in a
        // block, and resolving it as sparse is exact there anyway)
        bool dense = false;
        if (dpend > 0) {  // wave-uniform
            dense = valid && ((z & 0xFFFFu) == 0 || (z >> 16) == 0);
            const unsigned long long db = __builtin_amdgcn_ballot_w64(dense);
            if (db) {
                resolve_block(dk, dense, g_begin + off, lo, hi, dense_lim, k, cq, cqn, lane, hit);
                resolve_block(dk, dense && off + 64 < ng, g_begin + off + 64, lo, hi, dense_lim, k, cq, cqn, lane, hit);
                dpend -= std::min<int32_t>(dpend, (int32_t)__popcll(db));
            }
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
                const bool odd = e & 1u;
                const uint32_t Lh = odd ? w.z : w.x;
                // a superset of j < k on 32-bit operands, the 64-bit index formed only behind it:
                // i >> 8 = ghi:bl >> 4 (i < 2^40) and i + 1 >= (i >> 8) << 8, so (Lh >> 8)(i + 1) <
                // k 2^32 (itself implied by j < k) implies (Lh >> 8)(i >> 8) < k 2^24.  With the
                // dense test above skipped: 81.5-82.1 -> 80.6-81.0 us (profiles/r05/micro_k1o_trim.jsonl)
                const uint32_t i8 = (ghi << 28) | (bl >> 4);
                if ((uint64_t)(Lh >> 8) * i8 < k_24) {
                    const uint64_t i = ((((uint64_t)ghi << 32) | bl) << 4) | (e & 15u);
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
    // M0 in a VGPR, opaque to the compiler (philox4x32_10_uniform_hi_x2_at)
    uint32_t m0v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(m0v) : "s"(kPhiloxM0));
    // one steady iteration: the pair at counter word gl + d (d wave-uniform), its fold and mark
    // appended (see below); the entry's low word is lo(M0 (gl + d))
    auto steady = [&](uint32_t d) {
        u32x4 w0, w1;
        uint32_t glo;
        philox4x32_10_uniform_hi_x2_at(gl, m0v, (uint64_t)kPhiloxM0 * d, ghi, dk.s0, dk.s1, dk.k0, dk.k1, w0, w1, glo);
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
        const uint64_t ent = (uint64_t)glo | ((uint64_t)z << 32);
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
    };
    // one iteration of a partial window (the first, the last, or where dense / clipped blocks lie) at
    // block offset b (wave-uniform) and counter word gl
    auto partial = [&](uint32_t b) {
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            w[u] = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
        uint32_t z;
        bool has;
        if (b >= off_steady && b + U * 64 <= ng_steady) {
            z = fold_pair(w[0], w[1]);
            has = z != 0xFFFFFFFFu;
        } else {
            uint32_t y[U];
            bool hb[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t off = b + u * 64 + lane;
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
        dpend += (int32_t)__popcll(__builtin_amdgcn_ballot_w64(has && ((z & 0xFFFFu) == 0 || (z >> 16) == 0)));
        append(has, gl * kPhiloxM0, z);
        __builtin_amdgcn_wave_barrier();
        rounds();
    };
    if (A > 0) {
        constexpr uint32_t UB = (W / 2) * U * 64;
        const uint32_t units = (ng + UB - 1) / UB;
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
                for (int t = 0; t < W / 2; ++t) steady(t * (U * 64));
                __builtin_amdgcn_wave_barrier();
                rounds();
            } else {  // a unit holding dense / clipped blocks or the launch's end
                for (int t = 0; t < W / 2 && ub < ng; ++t, ub += U * 64, gl += U * 64) partial(ub);
            }
        }
        base = ng;  // the grid-stride loop below has nothing left
    }
    while (base < ng) {  // wave-uniform
        if (base >= off_steady && (uint64_t)base + (uint64_t)(W - 1) * stride + U * 64 <= ng_steady) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int t = 0; t < W / 2; ++t) steady(t * stride);
                gl += (W / 2) * stride;
                __builtin_amdgcn_wave_barrier();
                rounds();
            }
            base += W * stride;
        } else {  // a partial window (first, last, or where the dense / clipped blocks lie)
            for (int t = 0; t < W && base < ng; ++t, base += stride, gl += stride) {
                partial(base);
            }
        }
    }
    if (pool) {
        // The workgroup's leftovers pooled (every wave holds < 64, and a pooled round's rests <= 64):
        // round w of the waves' queues taken end to end goes to wave w, so a workgroup runs
        // ceil(sum / 64) tail rounds at once instead of one or two per wave (each a whole wave's
        // level-1 Philox however few lanes it holds); the rests they append are pooled again.  `pool`
        // (LDS, one word per wave): the wave's count, bit 31 = it has dense entries pending (an entry
        // may move to a wave without any, which then runs the dense test -- exact either way).
        // Needs every wave of the workgroup here (k1_body_q is called workgroup-wide).  Measured
        // (tools/micro_k1o o, profiles/r06/micro_k1o_tail_ab.jsonl): fewer VALU but no faster -- 81.2-81.5
        // vs 80.7-81.2 us per 1e9 draws (the barriers hold each workgroup to its slowest wave), so the
        // product kernels pass no pool and keep the per-wave tail below.
        constexpr uint32_t cap = k1q_cap<W>(), NW = kQueueWaves;
        const uint32_t wv = threadIdx.x >> 6;
        const uint64_t* q0 = q - (size_t)wv * cap;
        for (;;) {
            if (lane == 0) pool[wv] = qn | (dpend > 0 ? 0x80000000u : 0u);
            __syncthreads();
            uint32_t c[NW], T = 0, anyd = 0;
#pragma unroll
            for (uint32_t v = 0; v < NW; ++v) {
                const uint32_t pv = (uint32_t)__builtin_amdgcn_readfirstlane((int)pool[v]);
                c[v] = pv & 0x7FFFFFFFu;
                anyd |= pv >> 31;
                T += c[v];
            }
            if (T == 0) break;  // workgroup-uniform
            uint32_t o = 64u * wv + lane, src = 0;
            const bool valid = o < T;
#pragma unroll
            for (uint32_t v = 0; v + 1 < NW; ++v)
                if (src == v && o >= c[v]) {
                    o -= c[v];
                    src = v + 1;
                }
            const uint64_t ent = valid ? q0[(size_t)src * cap + o] : 0ull;
            __syncthreads();  // every read done before a wave appends to its own queue again
            qn = 0;
            dpend = anyd ? (1 << 30) : 0;
            if (64u * wv < T) resolve(valid, ent);  // wave-uniform
        }
    } else {
        while (qn > 0) {  // the last partial rounds (appends shrink geometrically)
            __builtin_amdgcn_wave_barrier();
            const uint32_t nv = std::min<uint32_t>(qn, 64u);
            qn -= nv;
            const bool valid = lane < nv;
            const uint64_t ent = valid ? q[qn + lane] : 0ull;
            __builtin_amdgcn_wave_barrier();
            resolve(valid, ent);
        }
    }
    __builtin_amdgcn_wave_barrier();
    drain_queue(dk, cq, cqn, lane, k, hit);
}

}  // namespace rsv
