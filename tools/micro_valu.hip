// micro_valu.hip -- issue cost of the VALU instructions that make up Philox4x32-10 on gfx950, and
// the cost of one whole level-0 Philox call as K1 evaluates it (development tool, not product).
//
// Every wave of a full chip (256 CUs x 32 waves, i.e. 8 waves on each SIMD) issues a long run of
// independent instructions of one kind; s_memtime (shader-clock ticks, MI355X_MICROARCH.md) around
// the run gives cycles per wave (s_memrealtime, 100 MHz, beside it gives the clock the run had), and
//     cycles per wave-instruction on one SIMD = median wave cycles / (instructions per wave x 8).
// The result is clock-independent (DVFS moves wall time, not these cycles).  bench.py's VALU
// roofline prices a Philox call with these costs (profiles/r02/valu_costs.json).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro_valu.hip -o tools/micro_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "../reservoir_amd/csrc/rsv_device.h"

using namespace rsv;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

constexpr int kWavesPerSimd = 8;
constexpr int kBlocksPerCu = 8;  // 8 x 4 waves = 32 waves per CU

// 8 instructions of kind OP to 8 different destinations, inputs a, b (vector) and s (scalar)
template <int OP>
__device__ __forceinline__ void burst(uint32_t (&d)[8], uint64_t (&q)[8], uint32_t a, uint32_t b, uint32_t s) {
#define ONE(i)                                                                                              \
    if constexpr (OP == 0) {                                                                                \
        uint64_t c;                                                                                         \
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(q[i]), "=s"(c) : "v"(a), "s"(s));             \
    } else if constexpr (OP == 1) {                                                                         \
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d[i]) : "v"(a), "v"(b), "s"(s));      \
    } else if constexpr (OP == 2) {                                                                         \
        asm volatile("v_xor_b32 %0, %1, %2" : "=v"(d[i]) : "s"(s), "v"(a));                                 \
    } else if constexpr (OP == 3) {                                                                         \
        asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(d[i]) : "v"(a), "s"(s));                              \
    } else if constexpr (OP == 4) {                                                                         \
        asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(d[i]) : "v"(a), "s"(s));                              \
    } else if constexpr (OP == 5) {                                                                         \
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(d[i]) : "s"(s), "v"(a));                                 \
    } else if constexpr (OP == 6) {                                                                         \
        asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(d[i]) : "v"(a), "v"(b), "s"(s));                     \
    } else if constexpr (OP == 7) {                                                                         \
        const uint64_t ab = ((uint64_t)b << 32) | a;                                                        \
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(q[i]) : "v"(ab), "v"(ab), "v"(ab));               \
    }
    ONE(0) ONE(1) ONE(2) ONE(3) ONE(4) ONE(5) ONE(6) ONE(7)
#undef ONE
}

template <int OP>
__global__ __launch_bounds__(256) void op_rate(uint64_t* cyc, uint32_t* sink, uint32_t s, int iters) {
    uint32_t d[8];
    uint64_t q[8];
    const uint32_t a = threadIdx.x * 0x9E3779B9u, b = a ^ s;
    __builtin_amdgcn_s_barrier();
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        burst<OP>(d, q, a + it, b, s);
        burst<OP>(d, q, a + it, b, s);
        burst<OP>(d, q, a + it, b, s);
        burst<OP>(d, q, a + it, b, s);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= d[i] ^ (uint32_t)q[i];
    if (r == 0x1234567u) sink[0] = r;
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        cyc[2 * w] = t1 - t0;
        cyc[2 * w + 1] = r1 - r0;
    }
}

// K1's level-0 call (counter words 1..3 wave-uniform), two chains per lane as in K1
__global__ __launch_bounds__(256) void philox_rate(uint64_t* cyc, uint32_t* sink, uint32_t s, int iters) {
    const DrawKey dk{0xC0FFEEu, s, 0x5A5Au, 0};
    uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x, acc = 0;
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
    __builtin_amdgcn_s_barrier();
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it, gl += 1u << 21) {
        const u32x4 w0 = philox4x32_10_uniform_hi(gl, ghi, dk.s0, dk.s1, dk.k0, dk.k1);
        const u32x4 w1 = philox4x32_10_uniform_hi(gl + 64, ghi, dk.s0, dk.s1, dk.k0, dk.k1);
        acc ^= w0.x ^ w0.y ^ w0.z ^ w0.w ^ w1.x ^ w1.y ^ w1.z ^ w1.w;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (acc == 0x1234567u) sink[0] = acc;
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        cyc[2 * w] = t1 - t0;
        cyc[2 * w + 1] = r1 - r0;
    }
}

// the full (non-uniform) Philox4x32-10 of the level-1 draws
__global__ __launch_bounds__(256) void philox_full_rate(uint64_t* cyc, uint32_t* sink, uint32_t s, int iters) {
    uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x, acc = 0;
    __builtin_amdgcn_s_barrier();
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it, gl += 1u << 21) {
        const u32x4 w0 = philox4x32_10(gl, gl ^ 0x80000000u, s, gl >> 7, 0xC0FFEEu, s);
        const u32x4 w1 = philox4x32_10(gl + 64, gl ^ 0x80000001u, s, gl >> 7, 0xC0FFEEu, s);
        acc ^= w0.x ^ w0.y ^ w0.z ^ w0.w ^ w1.x ^ w1.y ^ w1.z ^ w1.w;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (acc == 0x1234567u) sink[0] = acc;
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        cyc[2 * w] = t1 - t0;
        cyc[2 * w + 1] = r1 - r0;
    }
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * kBlocksPerCu, waves = grid * 4;
    uint64_t* cyc;
    uint32_t* sink;
    CK(hipMalloc(&cyc, (size_t)waves * 16));
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint64_t> h(2 * (size_t)waves);
    // per row: cycles per wave-instruction per SIMD two ways -- from each wave's own s_memtime span
    // (a LOWER bound: the 8 waves of a SIMD do not all overlap for the whole span, dispatch staggers
    // their starts) and from the launch's wall time at the in-kernel clock (an UPPER bound: includes
    // the dispatch ramp); a long run (16x the iterations) brings the two together
    auto run = [&](auto kern, const char* name, double per_iter, int iters) -> int {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, cyc, sink, 7u, iters);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, cyc, sink, 7u, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(h.data(), cyc, (size_t)waves * 16, hipMemcpyDeviceToHost));
        std::vector<uint64_t> s(waves), r(waves);
        for (int w = 0; w < waves; ++w) s[w] = h[2 * w], r[w] = h[2 * w + 1];
        std::sort(s.begin(), s.end());
        std::sort(r.begin(), r.end());
        const double med = (double)s[s.size() / 2], rmed = (double)r[r.size() / 2];
        const double ghz = med / rmed * 0.1;  // shader clock during the run (guide: memtime / memrealtime x 100 MHz)
        const double per_simd = per_iter * iters * kWavesPerSimd;
        const double cpi = med / per_simd, wall_cpi = ms * 1e6 * ghz / per_simd;
        printf("{\"op\": \"%s\", \"iters\": %d, \"cycles_per_wave_instr_per_simd_wave_span\": %.3f, "
               "\"cycles_per_wave_instr_per_simd_wall\": %.3f, \"median_wave_cycles\": %.0f, \"wall_ms\": %.4f, "
               "\"clock_GHz\": %.3f, \"wall_ns_per_wave_instr_per_simd\": %.3f}\n",
               name, iters, cpi, wall_cpi, med, ms, ghz, ms * 1e6 / per_simd);
        return 0;
    };
    const double burst_instr = 4.0 * 8;
    // the clock ramps under sustained load: ~1 s of back-to-back launches before the first row
    for (int rep = 0; rep < 2000; ++rep) hipLaunchKernelGGL(op_rate<2>, dim3(grid), dim3(256), 0, 0, cyc, sink, 7u, 1024);
    CK(hipDeviceSynchronize());
    for (int it : {1024, 16384}) if (run(op_rate<0>, "v_mad_u64_u32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(op_rate<1>, "v_bitop3_b32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(op_rate<2>, "v_xor_b32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(op_rate<3>, "v_mul_hi_u32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(op_rate<4>, "v_mul_lo_u32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(op_rate<5>, "v_add_u32", burst_instr, it)) return 1;
    // the guide's fp32 FMA figure (2 cycles per wave64 instruction on a SIMD) against the 32-bit
    // integer ops above: reconciles the 4-cycle issue model bench.py's VALU roofline prices with
    for (int it : {1024, 16384}) if (run(op_rate<6>, "v_fma_f32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(op_rate<7>, "v_pk_fma_f32", burst_instr, it)) return 1;
    for (int it : {1024, 16384}) if (run(philox_rate, "philox4x32_10_uniform_hi (per call)", 2.0, it)) return 1;
    for (int it : {1024, 16384}) if (run(philox_full_rate, "philox4x32_10 (per call)", 2.0, it)) return 1;
    return 0;
}
