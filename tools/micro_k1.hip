// micro_k1.hip -- instruction-rate and K1-variant microbenchmarks (development tool, not product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include tools/micro_k1.hip -o tools/micro_k1
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "../reservoir_amd/csrc/rsv_device.h"
#include "k1_dev_bodies.h"

using namespace rsv;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

// ---- op-rate kernels: 8 independent chains, ITER iterations ---------------------------------
template <int OP>
__global__ __launch_bounds__(256) void op_rate(uint32_t* out, uint32_t seed, int iters) {
    uint32_t a[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) a[c] = threadIdx.x * 7 + c + seed;
    const uint32_t m = 0xD2511F53u ^ seed;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (OP == 0) {  // v_mad_u64_u32 (64-bit product, both halves used)
                uint64_t p = (uint64_t)a[c] * m;
                a[c] = (uint32_t)p ^ (uint32_t)(p >> 32);
            } else if constexpr (OP == 1) {  // v_mul_hi_u32 only
                a[c] = __umulhi(a[c], m) + c;
            } else if constexpr (OP == 2) {  // v_mul_lo_u32 only
                a[c] = a[c] * m + c;
            } else if constexpr (OP == 3) {  // xor / add (full-rate reference)
                a[c] = (a[c] ^ m) + c;
            } else if constexpr (OP == 4) {  // 24-bit mul
                a[c] = __umul24(a[c], m) + c;
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) r ^= a[c];
    if (r == 0x12345678u) out[0] = r;
}

// ---- K1 variants over an index range ---------------------------------------------------------
// V0: level 0 only (Philox + zero-byte pre-test), count blocks with a candidate
__global__ __launch_bounds__(256) void k1_level0_only(DrawKey dk, uint64_t n_groups, unsigned long long* cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t c = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups; g += stride) {
        const u32x4 w = level0(dk, g + (1ull << 20));
        c += any_zero_byte(w);
    }
    if (c == 0xFFFFFFFFu) atomicAdd(cnt, c);
}

// V1: philox only, no test at all
__global__ __launch_bounds__(256) void philox_only(DrawKey dk, uint64_t n_groups, unsigned long long* cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t c = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups; g += stride) {
        const u32x4 w = level0(dk, g);
        c ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    if (c == 0x12345u) atomicAdd(cnt, c);
}

// V2: the product's level-0 loop (uniform-hi Philox, U blocks per lane, the bit-window test) with
// the pushes removed: the cost of everything but the candidate handling
template <int U>
__global__ __launch_bounds__(256) void k1_l0_bits_only(DrawKey dk, uint64_t n_groups, unsigned long long* cnt) {
    const uint32_t ng = (uint32_t)n_groups;
    const uint32_t stride = gridDim.x * blockDim.x * U;
    uint32_t base = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * U);
    uint32_t gl = base + (threadIdx.x & 63);
    uint32_t acc = 0;
    while (base < ng) {
        uint32_t bits = 0;
        for (int t = 0; t < 32 / U && base < ng; ++t, base += stride, gl += stride) {
            u32x4 w[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                w[u] = philox4x32_10_uniform_hi(gl, 0u, dk.s0, dk.s1, dk.k0, dk.k1, (uint64_t)kPhiloxM0 * (64u * u));
#pragma unroll
            for (int u = 0; u < U; ++u) bits = (bits << 1) | (uint32_t)any_zero_byte(w[u]);
        }
        acc ^= bits;
    }
    if (acc == 0x12345u) atomicAdd(cnt, acc);
}

template <int U>
__global__ __launch_bounds__(256) void k1_var(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                              uint64_t n_groups, unsigned long long* win) {
    __shared__ uint32_t qs[4][63 + 64 * U + 1];
    __shared__ uint64_t cqs[4][kQueue];
    k1_body<U>(dk, k, lo, hi, g_begin, n_groups, win, qs[threadIdx.x >> 6], cqs[threadIdx.x >> 6]);
}

template <int U>
__global__ __launch_bounds__(256) void k1_var_bits(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                                   uint64_t n_groups, unsigned long long* win) {
    __shared__ uint32_t qs[4][63 + 64 + 1];
    __shared__ uint64_t cqs[4][kQueue];
    k1_body_bits<U>(dk, k, lo, hi, g_begin, n_groups, win, qs[threadIdx.x >> 6], cqs[threadIdx.x >> 6]);
}

template <int U>
__global__ __launch_bounds__(256) void k1_var_z(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                                uint64_t n_groups, unsigned long long* win) {
    __shared__ uint64_t qs[4][128];
    __shared__ uint16_t wys[4][kK1ZWin * 64];
    __shared__ uint32_t tabs[4][kK1ZWin];
    __shared__ uint64_t cqs[4][kQueue];
    k1_body_z<U>(dk, k, lo, hi, g_begin, n_groups, win, qs[threadIdx.x >> 6], wys[threadIdx.x >> 6],
                 tabs[threadIdx.x >> 6], cqs[threadIdx.x >> 6]);
}

template <int U, int WIN>
__global__ __launch_bounds__(256) void k1_var_zw(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                                 uint64_t n_groups, unsigned long long* win) {
    __shared__ uint64_t qs[4][128];
    __shared__ uint16_t wys[4][WIN * 64];
    __shared__ uint32_t tabs[4][WIN];
    __shared__ uint64_t cqs[4][kQueue];
    k1_body_z<U, WIN>(dk, k, lo, hi, g_begin, n_groups, win, qs[threadIdx.x >> 6], wys[threadIdx.x >> 6],
                      tabs[threadIdx.x >> 6], cqs[threadIdx.x >> 6]);
}

int main(int argc, char** argv) {
    uint32_t* d;
    CK(hipMalloc(&d, 64));
    unsigned long long* cnt;
    CK(hipMalloc(&cnt, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = 256 * 8, iters = 4096;
    const double ops = (double)blocks * 256 * iters * 8;
    auto time_op = [&](auto kern, const char* name) -> int {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u, iters);
        }
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        // lane-ops per second and per CU per clock at 2.4 GHz
        printf("%-28s %8.3f ms  %8.2f Tlane-op/s  %6.1f lane-op/clk/CU@2.4GHz\n", name, ms, ops / ms / 1e9,
               ops / (ms * 1e-3) / 256 / 2.4e9);
        return 0;
    };
    time_op(op_rate<0>, "mad_u64_u32 (+xor)");
    time_op(op_rate<1>, "mul_hi_u32 (+add)");
    time_op(op_rate<2>, "mul_lo_u32 (+add)");
    time_op(op_rate<3>, "xor+add");
    time_op(op_rate<4>, "mul_u32_u24 (+add)");

    const uint64_t n_groups = 1000000000ull / 16;
    DrawKey dk{0xC0FFEE, 0, 0x5A5A, 0};
    auto time_k = [&](auto kern, const char* name, int grid) -> int {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, n_groups, cnt);
        CK(hipEventRecord(e0));
        for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, n_groups, cnt);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s grid %6d  %8.1f us per 1e9 indices  (%.1f G philox/s)\n", name, grid, ms / 5 * 1e3,
               n_groups / (ms / 5 * 1e-3) / 1e9);
        return 0;
    };
    for (int grid : {1024, 2048, 4096, 8192}) time_k(philox_only, "philox_only", grid);
    for (int grid : {2048, 8192}) time_k(k1_level0_only, "level0+zero-test", grid);
    unsigned long long* win;
    CK(hipMalloc(&win, 1024 * 8));
    CK(hipMemset(win, 0, 1024 * 8));
    [[maybe_unused]] auto time_v = [&](auto kern, const char* name, int grid, int unroll) -> int {
        const uint64_t lo = 1024, hi = 1000000000ull;
        for (int rep = 0; rep < 2; ++rep)
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, 1024u, lo, hi, 0ull, n_groups, win);
        CK(hipEventRecord(e0));
        for (int rep = 0; rep < 5; ++rep)
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, 1024u, lo, hi, 0ull, n_groups, win);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, 1024u, lo, hi, 0ull, n_groups, win);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms1;
        CK(hipEventElapsedTime(&ms1, e0, e1));
        printf("%-28s grid %6d unroll %d  %8.1f us per 1e9 indices (single launch %.1f)\n", name, grid, unroll,
               ms / 5 * 1e3, ms1 * 1e3);
        return 0;
    };
    if (argc > 1 && argv[1][0] == 'p') {  // one launch of each variant, for rocprofv3 --pmc passes
        hipLaunchKernelGGL(philox_only, dim3(8192), dim3(256), 0, 0, dk, n_groups, cnt);
        hipLaunchKernelGGL(k1_level0_only, dim3(8192), dim3(256), 0, 0, dk, n_groups, cnt);
        hipLaunchKernelGGL(k1_var<2>, dim3(4096), dim3(256), 0, 0, dk, 1024u, 1024ull, 1000000000ull, 0ull,
                           n_groups, win);
        hipLaunchKernelGGL(k1_var_bits<2>, dim3(4096), dim3(256), 0, 0, dk, 1024u, 1024ull, 1000000000ull, 0ull,
                           n_groups, win);
        hipLaunchKernelGGL(k1_l0_bits_only<2>, dim3(4096), dim3(256), 0, 0, dk, n_groups, cnt);
        hipLaunchKernelGGL(k1_var_z<2>, dim3(4096), dim3(256), 0, 0, dk, 1024u, 1024ull, 1000000000ull, 0ull,
                           n_groups, win);
        CK(hipDeviceSynchronize());
        return 0;
    }
    if (argc > 1) {  // A/B: per-iteration pushes vs deferred bit-mask pushes (+ identical winners)
        std::vector<unsigned long long> ref(1024), got(1024);
        auto run_once = [&](auto kern, int grid, std::vector<unsigned long long>& out) -> int {
            CK(hipMemset(win, 0, 1024 * 8));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, 1024u, 1024ull, 1000000000ull, 0ull, n_groups,
                               win);
            CK(hipMemcpy(out.data(), win, 1024 * 8, hipMemcpyDeviceToHost));
            return 0;
        };
        if (run_once(k1_var<2>, 8192, ref)) return 1;
        if (argv[1][0] == 'z') {  // window x grid sweep of the zero-mask body (LDS sets the occupancy)
            const bool fine = argv[1][1] == 'f';  // 'zf': finer grid steps, two passes
            for (int pass = 0; pass < (fine ? 2 : 1); ++pass)
                for (int g : fine ? std::vector<int>{2560, 2816, 3072, 3328, 3584, 4096}
                                  : std::vector<int>{1536, 2048, 2560, 3072, 4096}) {
                    time_v(k1_var_zw<2, 32>, "k1 z win32", g, 2);
                    time_v(k1_var_zw<2, 16>, "k1 z win16", g, 2);
                    time_v(k1_var_zw<2, 24>, "k1 z win24", g, 2);
                    time_v(k1_var_zw<2, 20>, "k1 z win20", g, 2);
                }
            for (auto* kern : {k1_var_zw<2, 16>, k1_var_zw<2, 24>}) {
                if (run_once(kern, 2048, got)) return 1;
                printf("  winners identical: %s\n", ref == got ? "yes" : "NO");
            }
            return 0;
        }
        if (argv[1][0] == 'g') {  // grid sweep of the product body
            for (int g : {1536, 2048, 2560, 3072, 3584, 4096, 5120, 6144, 8192, 12288})
                time_v(k1_var_bits<2>, "k1 bit-mask push", g, 2);
            return 0;
        }
        for (int grid : {4096, 8192}) {
            time_v(k1_var_z<2>, "k1 zero-mask queue", grid / 2, 2);
            if (run_once(k1_var_z<2>, grid / 2, got)) return 1;
            printf("  winners identical (z): %s\n", ref == got ? "yes" : "NO");
            time_v(k1_var<2>, "k1 per-iteration push", grid / 2, 2);
            time_v(k1_var_bits<1>, "k1 bit-mask push", grid, 1);
            time_v(k1_var_bits<2>, "k1 bit-mask push", grid / 2, 2);
            if (run_once(k1_var_bits<2>, grid / 2, got)) return 1;
            printf("  winners identical: %s\n", ref == got ? "yes" : "NO");
            if (run_once(k1_var_bits<1>, grid, got)) return 1;
            printf("  winners identical (U=1): %s\n", ref == got ? "yes" : "NO");
        }
        return 0;
    }
    for (int grid : {4096, 8192, 16384}) {
        time_v(k1_var<1>, "k1 product body", grid / 1, 1);
        time_v(k1_var<2>, "k1 product body", grid / 2, 2);
        time_v(k1_var<4>, "k1 product body", grid / 4, 4);
    }

    return 0;
}
