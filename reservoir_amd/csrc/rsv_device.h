// rsv_device.h -- device helpers shared by the gfx950 kernels: Philox4x32-10, draw format R2,
// and the scrambled hash of Sampler.distinct.
//
// Draw format R2 (DESIGN.md "Draw format"): for element index i of Philox stream s under key
// (seed), U_i is a 64-bit uniform assembled from two counter-based Philox4x32-10 calls:
//   level 0: ctr = (g0, g0>>32, s, s>>32), g0 = i >> 4   -> 128 bits shared by 16 indices, read
//            as 8 bit-planes of 16 bits (plane p = bits [16 (p&1), 16 (p&1) + 16) of word p>>1);
//            b_i = the byte whose bit p is bit (i & 15) of plane p -- the top byte of U_i
//   level 1: ctr = (g1, (g1>>32) | 1<<31, s, s>>32), g1 = i >> 1 -> two 64-bit words;
//            L_i = word (i & 1) = (w[2(i&1)] << 32) | w[2(i&1)+1]
//   U_i = (b_i << 56) | (L_i >> 8),  j_i = floor(U_i * (i+1) / 2^64)   (uniform on [0, i])
// Element i >= k replaces slot j_i iff j_i < k (Algorithm R).  Since U_i >= b_i * 2^56, a
// necessary condition for j_i < k is b_i * (i+1) < 256 k; the kernels test that on level-0
// bits only and evaluate level 1 for the ~1/256 candidates that pass.  The bit-sliced layout makes
// the sparse-region test "some b_i of the block is 0" one OR over the four words and a fold of
// the two 16-bit halves (5 VALU ops for 16 indices; per-byte SWAR took 11).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsv {

struct u32x4 {
    uint32_t x, y, z, w;
};

constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;
constexpr uint32_t kDomainLevel1 = 0x80000000u;

// three-input xor in one VALU op (gfx950 has no v_xor3_b32; v_bitop3_b32 with truth table 0x96).
// The builtin, not inline asm: the hazard recognizer pads every inline-asm block with an s_nop
// (13 per K1 iteration of two blocks, ~14 % of its issue slots), and the scheduler cannot move it.
__device__ __forceinline__ uint32_t xor3_key(uint32_t a, uint32_t b, uint32_t key) {
    return __builtin_amdgcn_bitop3_b32(a, b, key, 0x96);
}

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11).  k0/k1 are wave-uniform (kernel args), so
// the key schedule stays in SGPRs; each round is two v_mad_u64_u32 and two v_bitop3 (xor3).
__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c0;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * c2;
        const uint32_t n0 = xor3_key((uint32_t)(p1 >> 32), c1, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t n2 = xor3_key((uint32_t)(p0 >> 32), c3, k1 + (uint32_t)r * kPhiloxW1);
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    return {c0, c1, c2, c3};
}

// The same function when counter words 1..3 are wave-uniform (c0 per lane): round 0's first output
// and round 1's first product are then scalar (SALU, hoisted out of any loop over c0), and round
// 1's xors take one scalar operand each -- 18 v_mad_u64_u32 + 1 v_bitop3 + 2 v_xor per call
// instead of 19 + 20 (the asm xor3 forces VGPR operands, so the uniform part must stay in C).
// `add0` = kPhiloxM0 * d for counter c0 + d (d wave-uniform): the addend of the first product's
// v_mad_u64_u32, so a lane evaluating the blocks at c0 and c0 + 64 needs no v_add for the second.
__device__ __forceinline__ u32x4 philox4x32_10_uniform_hi(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                          uint32_t k0, uint32_t k1, uint64_t add0 = 0) {
    // round 0
    const uint64_t p1u = (uint64_t)kPhiloxM1 * c2;                  // scalar
    const uint32_t n0u = (uint32_t)(p1u >> 32) ^ c1 ^ k0;           // scalar
    const uint64_t p0 = (uint64_t)kPhiloxM0 * c0 + add0;            // vector: M0 (c0 + d) mod 2^64
    // c3 ^ k1 on the scalar unit: a v_bitop3 with two scalar operands costs a v_mov first
    uint32_t d2 = (uint32_t)(p0 >> 32) ^ (c3 ^ k1);
    const uint32_t d1u = (uint32_t)p1u;                             // scalar
    uint32_t d3 = (uint32_t)p0;                                     // vector
    // round 1
    const uint64_t q0u = (uint64_t)kPhiloxM0 * n0u;                 // scalar
    const uint64_t q1 = (uint64_t)kPhiloxM1 * d2;                   // vector
    uint32_t c0v = (uint32_t)(q1 >> 32) ^ (d1u ^ (k0 + kPhiloxW0));  // one scalar operand
    uint32_t c2v = d3 ^ ((uint32_t)(q0u >> 32) ^ (k1 + kPhiloxW1));  // one scalar operand
    uint32_t c1v = (uint32_t)q1;
    uint32_t c3v = (uint32_t)q0u;  // scalar until round 2 (its product's operand is c2v)
    {  // round 2: c3v and the key are both scalar (one v_xor, no v_mov)
        const uint64_t p0r = (uint64_t)kPhiloxM0 * c0v;
        const uint64_t p1r = (uint64_t)kPhiloxM1 * c2v;
        const uint32_t n0 = xor3_key((uint32_t)(p1r >> 32), c1v, k0 + 2u * kPhiloxW0);
        const uint32_t n2 = (uint32_t)(p0r >> 32) ^ (c3v ^ (k1 + 2u * kPhiloxW1));
        c0v = n0;
        c1v = (uint32_t)p1r;
        c2v = n2;
        c3v = (uint32_t)p0r;
    }
#pragma unroll
    for (int r = 3; r < 10; ++r) {
        const uint64_t p0r = (uint64_t)kPhiloxM0 * c0v;
        const uint64_t p1r = (uint64_t)kPhiloxM1 * c2v;
        const uint32_t n0 = xor3_key((uint32_t)(p1r >> 32), c1v, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t n2 = xor3_key((uint32_t)(p0r >> 32), c3v, k1 + (uint32_t)r * kPhiloxW1);
        c0v = n0;
        c1v = (uint32_t)p1r;
        c2v = n2;
        c3v = (uint32_t)p0r;
    }
    return {c0v, c1v, c2v, c3v};
}

// Two philox4x32_10_uniform_hi calls (counters c0 and c0 + 64, same uniform words) with their
// rounds interleaved in the source, so the two dependent chains issue alternately (a lone chain
// leaves every other issue slot of the wave waiting on its previous round: K1 measured 89 -> 125 us
// when the scheduler emitted the second call after the first).
__device__ __forceinline__ void philox4x32_10_uniform_hi_x2(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                            uint32_t k0, uint32_t k1, u32x4& a, u32x4& b) {
    const uint64_t p1u = (uint64_t)kPhiloxM1 * c2;
    const uint32_t n0u = (uint32_t)(p1u >> 32) ^ c1 ^ k0;
    const uint64_t pa = (uint64_t)kPhiloxM0 * c0;
    const uint64_t pb = (uint64_t)kPhiloxM0 * c0 + (uint64_t)kPhiloxM0 * 64u;
    const uint32_t da2 = xor3_key((uint32_t)(pa >> 32), c3, k1), db2 = xor3_key((uint32_t)(pb >> 32), c3, k1);
    const uint32_t d1u = (uint32_t)p1u;
    const uint32_t da3 = (uint32_t)pa, db3 = (uint32_t)pb;
    const uint64_t q0u = (uint64_t)kPhiloxM0 * n0u;
    const uint64_t qa = (uint64_t)kPhiloxM1 * da2, qb = (uint64_t)kPhiloxM1 * db2;
    uint32_t a0 = (uint32_t)(qa >> 32) ^ (d1u ^ (k0 + kPhiloxW0)), b0 = (uint32_t)(qb >> 32) ^ (d1u ^ (k0 + kPhiloxW0));
    uint32_t a2 = da3 ^ ((uint32_t)(q0u >> 32) ^ (k1 + kPhiloxW1)), b2 = db3 ^ ((uint32_t)(q0u >> 32) ^ (k1 + kPhiloxW1));
    uint32_t a1 = (uint32_t)qa, b1 = (uint32_t)qb;
    uint32_t a3 = (uint32_t)q0u, b3 = (uint32_t)q0u;
#pragma unroll
    for (int r = 2; r < 10; ++r) {
        const uint64_t pa0 = (uint64_t)kPhiloxM0 * a0, pb0 = (uint64_t)kPhiloxM0 * b0;
        const uint64_t pa1 = (uint64_t)kPhiloxM1 * a2, pb1 = (uint64_t)kPhiloxM1 * b2;
        const uint32_t na0 = xor3_key((uint32_t)(pa1 >> 32), a1, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t nb0 = xor3_key((uint32_t)(pb1 >> 32), b1, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t na2 = xor3_key((uint32_t)(pa0 >> 32), a3, k1 + (uint32_t)r * kPhiloxW1);
        const uint32_t nb2 = xor3_key((uint32_t)(pb0 >> 32), b3, k1 + (uint32_t)r * kPhiloxW1);
        a0 = na0;
        b0 = nb0;
        a1 = (uint32_t)pa1;
        b1 = (uint32_t)pb1;
        a2 = na2;
        b2 = nb2;
        a3 = (uint32_t)pa0;
        b3 = (uint32_t)pb0;
    }
    a = {a0, a1, a2, a3};
    b = {b0, b1, b2, b3};
}

// M0^-1 mod 2^32: K1's queue entries carry lo(M0 c0) (the round-0 product a pair already holds)
// instead of the counter word c0 itself, recovered as lo * M0^-1
constexpr uint32_t kPhiloxM0Inv = 0x991A7CDBu;
static_assert((uint32_t)(kPhiloxM0 * kPhiloxM0Inv) == 1u, "M0 inverse");

// philox4x32_10_uniform_hi_x2 at counters c0 = gl + d and gl + d + 64 (d wave-uniform, no 2^32 wrap),
// given m0v = M0 in a VGPR: each round-0 product is then one v_mad_u64_u32 m0v * gl + M0 (d [+ 64])
// with the wave-uniform addend in SGPRs (a VOP3 reads one scalar operand), so the pair's counter word
// needs no v_add.  lo_a = lo(M0 (gl + d)), the entry word K1 queues.
__device__ __forceinline__ void philox4x32_10_uniform_hi_x2_at(uint32_t gl, uint32_t m0v, uint64_t offa,
                                                               uint32_t c1, uint32_t c2, uint32_t c3,
                                                               uint32_t k0, uint32_t k1, u32x4& a, u32x4& b,
                                                               uint32_t& lo_a) {
    const uint64_t p1u = (uint64_t)kPhiloxM1 * c2;
    const uint32_t n0u = (uint32_t)(p1u >> 32) ^ c1 ^ k0;
    const uint64_t pa = (uint64_t)m0v * gl + offa;
    const uint64_t pb = (uint64_t)m0v * gl + (offa + (uint64_t)kPhiloxM0 * 64u);
    lo_a = (uint32_t)pa;
    const uint32_t c3k = c3 ^ k1;  // scalar (see philox4x32_10_uniform_hi)
    const uint32_t da2 = (uint32_t)(pa >> 32) ^ c3k, db2 = (uint32_t)(pb >> 32) ^ c3k;
    const uint32_t d1u = (uint32_t)p1u;
    const uint32_t da3 = (uint32_t)pa, db3 = (uint32_t)pb;
    const uint64_t q0u = (uint64_t)kPhiloxM0 * n0u;
    const uint64_t qa = (uint64_t)kPhiloxM1 * da2, qb = (uint64_t)kPhiloxM1 * db2;
    uint32_t a0 = (uint32_t)(qa >> 32) ^ (d1u ^ (k0 + kPhiloxW0)), b0 = (uint32_t)(qb >> 32) ^ (d1u ^ (k0 + kPhiloxW0));
    uint32_t a2 = da3 ^ ((uint32_t)(q0u >> 32) ^ (k1 + kPhiloxW1)), b2 = db3 ^ ((uint32_t)(q0u >> 32) ^ (k1 + kPhiloxW1));
    uint32_t a1 = (uint32_t)qa, b1 = (uint32_t)qb;
    uint32_t a3 = (uint32_t)q0u, b3 = (uint32_t)q0u;
    {  // round 2: a3 = b3 and the key are scalar
        const uint64_t pa0 = (uint64_t)kPhiloxM0 * a0, pb0 = (uint64_t)kPhiloxM0 * b0;
        const uint64_t pa1 = (uint64_t)kPhiloxM1 * a2, pb1 = (uint64_t)kPhiloxM1 * b2;
        const uint32_t na0 = xor3_key((uint32_t)(pa1 >> 32), a1, k0 + 2u * kPhiloxW0);
        const uint32_t nb0 = xor3_key((uint32_t)(pb1 >> 32), b1, k0 + 2u * kPhiloxW0);
        const uint32_t s3 = (uint32_t)q0u ^ (k1 + 2u * kPhiloxW1);
        const uint32_t na2 = (uint32_t)(pa0 >> 32) ^ s3, nb2 = (uint32_t)(pb0 >> 32) ^ s3;
        a0 = na0;
        b0 = nb0;
        a1 = (uint32_t)pa1;
        b1 = (uint32_t)pb1;
        a2 = na2;
        b2 = nb2;
        a3 = (uint32_t)pa0;
        b3 = (uint32_t)pb0;
    }
#pragma unroll
    for (int r = 3; r < 10; ++r) {
        const uint64_t pa0 = (uint64_t)kPhiloxM0 * a0, pb0 = (uint64_t)kPhiloxM0 * b0;
        const uint64_t pa1 = (uint64_t)kPhiloxM1 * a2, pb1 = (uint64_t)kPhiloxM1 * b2;
        const uint32_t na0 = xor3_key((uint32_t)(pa1 >> 32), a1, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t nb0 = xor3_key((uint32_t)(pb1 >> 32), b1, k0 + (uint32_t)r * kPhiloxW0);
        const uint32_t na2 = xor3_key((uint32_t)(pa0 >> 32), a3, k1 + (uint32_t)r * kPhiloxW1);
        const uint32_t nb2 = xor3_key((uint32_t)(pb0 >> 32), b3, k1 + (uint32_t)r * kPhiloxW1);
        a0 = na0;
        b0 = nb0;
        a1 = (uint32_t)pa1;
        b1 = (uint32_t)pb1;
        a2 = na2;
        b2 = nb2;
        a3 = (uint32_t)pa0;
        b3 = (uint32_t)pb0;
    }
    a = {a0, a1, a2, a3};
    b = {b0, b1, b2, b3};
}

struct DrawKey {
    uint32_t k0, k1;  // Philox key = seed
    uint32_t s0, s1;  // Philox stream words (counter words 2, 3)
};

__device__ __forceinline__ u32x4 level0(const DrawKey& dk, uint64_t g0) {
    return philox4x32_10((uint32_t)g0, (uint32_t)(g0 >> 32), dk.s0, dk.s1, dk.k0, dk.k1);
}

__device__ __forceinline__ uint32_t word_of(const u32x4& w, uint32_t q) {
    return q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
}

// b_e (e = 0..15) of a level-0 block: bit e of each of the 8 planes
__device__ __forceinline__ uint32_t level0_byte(const u32x4& w, uint32_t e) {
    // planes 2q (bit 0 after the shift) and 2q+1 (bit 16) of word q, interleaved into bits 2q, 2q+1
    const uint32_t u = ((w.x >> e) & 0x10001u) | (((w.y >> e) & 0x10001u) << 2) |
                       (((w.z >> e) & 0x10001u) << 4) | (((w.w >> e) & 0x10001u) << 6);
    return (u & 0x55u) | ((u >> 15) & 0xAAu);
}

// exact j_i given b_i (level-1 evaluated here)
__device__ __forceinline__ uint64_t exact_j(const DrawKey& dk, uint64_t i, uint32_t b) {
    const uint64_t g1 = i >> 1;
    const u32x4 w =
        philox4x32_10((uint32_t)g1, (uint32_t)(g1 >> 32) | kDomainLevel1, dk.s0, dk.s1, dk.k0, dk.k1);
    const uint64_t L = (i & 1) ? (((uint64_t)w.z << 32) | w.w) : (((uint64_t)w.x << 32) | w.y);
    const uint64_t U = ((uint64_t)b << 56) | (L >> 8);
    return __umul64hi(U, i + 1);
}

// OR of the 8 planes folded onto bits 0..15 and 16..31 alike: bit e clear <=> b_e == 0
__device__ __forceinline__ uint32_t planes_or(const u32x4& w) {
    const uint32_t x = w.x | w.y | w.z | w.w;
    return x | __builtin_amdgcn_alignbit(x, x, 16);  // x | rotate(x, 16)
}

// 16-bit mask of the zero bytes b_e == 0 of a level-0 block (exact)
__device__ __forceinline__ uint32_t zero_byte_mask16(const u32x4& w) { return ~planes_or(w) & 0xFFFFu; }

// true iff some b_e of the block is zero (the sparse-region candidate test)
__device__ __forceinline__ bool any_zero_byte(const u32x4& w) { return planes_or(w) != 0xFFFFFFFFu; }

// 16-bit mask of b_e < T (T in [0, 256]): bit-sliced compare, most significant plane first
__device__ __forceinline__ uint32_t lt_mask16(const u32x4& w, uint32_t T) {
    if (T >= 256u) return 0xFFFFu;
    uint32_t lt = 0, eq = 0xFFFFu;
#pragma unroll
    for (int p = 7; p >= 0; --p) {
        const uint32_t plane = (word_of(w, (uint32_t)p >> 1) >> (16 * (p & 1))) & 0xFFFFu;
        const uint32_t tm = 0u - ((T >> p) & 1u);  // all ones where T has bit p
        lt |= eq & ~plane & tm;
        eq &= ~(plane ^ tm);
    }
    return lt & 0xFFFFu;
}

// ---------------------------------------------------------------------------------------------
// Sampler.distinct scrambled hash (Sampler.scala:396) with scala.util.hashing.byteswap64
// (scala-library 2.13.6: v * 0x9e3779b97f4a7c15, reverse bytes, * 0x9e3779b97f4a7c15).
__host__ __device__ __forceinline__ uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }

__host__ __device__ __forceinline__ int64_t byteswap64(int64_t v) {
    uint64_t hc = (uint64_t)v * 0x9e3779b97f4a7c15ULL;
    hc = bswap64(hc);
    return (int64_t)(hc * 0x9e3779b97f4a7c15ULL);
}

__host__ __device__ __forceinline__ int64_t scramble(int64_t r0, int64_t r1, int64_t hashed) {
    return byteswap64(r1 ^ byteswap64(r0 ^ hashed));
}

enum HashKind : int { kHashIdentity = 1, kHashJavaLong = 2, kHashJavaInt = 3, kHashPrecomputed = 4, kHashUuid = 5 };

// java.util.UUID.hashCode (JDK: hilo = mostSigBits ^ leastSigBits; (int)(hilo >> 32) ^ (int) hilo),
// widened like `.toLong`, of a 16-byte key laid out [mostSigBits | leastSigBits], little-endian Longs
__host__ __device__ __forceinline__ int64_t uuid_hash_code(uint64_t msb, uint64_t lsb) {
    const uint64_t hilo = msb ^ lsb;
    return (int64_t)(int32_t)((uint32_t)(hilo >> 32) ^ (uint32_t)hilo);
}

// where a wide-key distinct sampler's hash comes from (rsv_wide.hip)
enum WideSrc : int { kWideSrcHashes = 0, kWideSrcUuid = 1 };

template <typename KeyT, int HASH>
__host__ __device__ __forceinline__ int64_t hash_of(KeyT key) {
    if constexpr (HASH == kHashJavaLong) {
        const uint64_t v = (uint64_t)(int64_t)key;
        return (int64_t)(int32_t)(uint32_t)(v ^ (v >> 32));
    } else if constexpr (HASH == kHashJavaInt) {
        return (int64_t)(int32_t)key;
    } else {
        return (int64_t)key;  // identity (Int keys widen with sign, like Int.toLong)
    }
}

// lane ^ s exchange (wave64) without the LDS crossbar (ds_bpermute: an LDS round trip on the sort networks'
// dependent chains): quad_perm DPP for s = 1, 2, two row shifts for 4, row_ror for 8, the gfx950
// permlane16/32 swaps for 16, 32.  s folds to a constant once the networks are unrolled.
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v, int s) {
    switch (s) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    case 4: {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xF, 0xF, false);  // row_shl:4 (i + 4)
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, false);  // row_shr:4 (i - 4)
        return (threadIdx.x & 4) ? dn : up;
    }
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    }
    case 32: {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
    default: return (uint32_t)__shfl_xor((int)v, s);
    }
}

template <typename T>
__device__ __forceinline__ T xor_any(T v, int s) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t x = (uint64_t)v;
        const uint32_t lo = xor_lane32((uint32_t)x, s), hi = xor_lane32((uint32_t)(x >> 32), s);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)xor_lane32((uint32_t)v, s);
    }
}

// End of a one-workgroup host publication: every wave waits for its own stores, the workgroup
// barrier orders them before lane 0, and lane 0 alone runs the system-scope release (L2 write-back)
// and stores the flag.  (A __threadfence_system() in every wave cost ~4 us more per publication.)
__device__ __forceinline__ void publish_flag(uint32_t* flag, uint32_t gen) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace rsv
