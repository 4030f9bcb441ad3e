// micro_k1o.hip -- K1 A/B (development tool, not product): the round-3 body k1_body_z
// compiled with the default register allocation (.sgpr_count 100 -> 6 workgroups of 256 per CU,
// MI355X_MICROARCH.md "Residency") and with amdgpu_num_sgpr limits that admit 8, over a grid sweep.
// Every variant's winner table is checked against the default's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include tools/micro_k1o.hip -o tools/micro_k1o
//        (+ -DK1O_DEBUG -o tools/micro_k1o_dbg: per-launch counters, mode 'd')
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

__device__ unsigned long long g_dbg[8];
#ifdef K1O_DEBUG  // counters (mode 'd'); the timing build leaves them out
#define RSV_K1P_COUNT(i, v) \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_dbg[i], (unsigned long long)(v))
#endif
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

struct K1Lds {
    uint64_t q[4][128];
    uint16_t wy[4][kK1ZWin * 64];
    uint32_t tab[4][kK1ZWin];
    uint64_t cq[4][kQueue];
};

#define KDEF(NAME, ATTR)                                                                                  \
    __global__ __launch_bounds__(256) ATTR void NAME(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi,     \
                                                     uint64_t g_begin, uint64_t n_groups,                 \
                                                     unsigned long long* __restrict__ win) {              \
        __shared__ K1Lds L;                                                                               \
        const int w = threadIdx.x >> 6;                                                                   \
        k1_body_z<2>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.wy[w], L.tab[w], L.cq[w]);          \
    }
KDEF(k1_base, )
KDEF(k1_s80, __attribute__((amdgpu_num_sgpr(80))))
KDEF(k1_s72, __attribute__((amdgpu_num_sgpr(72))))

// pair entries (k1_body_p), W iterations per window
template <int W>
struct K1PLds {
    uint64_t q[4][128];
    uint32_t wz[4][W * 64];
    uint32_t tab[4][W];
    uint64_t cq[4][kQueue];
};
template <int W>
__global__ __launch_bounds__(256) void k1_pair(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                               uint64_t n_groups, unsigned long long* __restrict__ win) {
    __shared__ K1PLds<W> L;
    const int w = threadIdx.x >> 6;
    k1_body_p<W>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.wz[w], L.tab[w], L.cq[w]);
}

// direct appends (k1_body_q), W iterations per window
template <int W>
struct K1QLds {
    uint64_t q[4][k1q_cap<W>()];
    uint64_t cq[4][kQueue];
    uint32_t pool[4];
};
template <int W, bool FAST = false>
__global__ __launch_bounds__(256) void k1_q(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                            uint64_t n_groups, unsigned long long* __restrict__ win) {
    __shared__ K1QLds<W> L;
    const int w = threadIdx.x >> 6;
    k1_body_q<W, FAST>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w]);
}

// the product body (a copy) with the tail cost probe (tools/k1_dev_bodies.h)
template <int W, bool FAST, bool SKIP>
__global__ __launch_bounds__(256) void k1_qd(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                             uint64_t n_groups, unsigned long long* __restrict__ win) {
    __shared__ K1QLds<W> L;
    const int w = threadIdx.x >> 6;
    k1_body_q_dev<W, FAST, SKIP>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w]);
}

// a static two-group schedule of half windows (tools/k1_dev_bodies.h k1_body_q_sched)
template <int W, bool FAST>
__global__ __launch_bounds__(256) void k1_qs(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                             uint64_t n_groups, unsigned long long* __restrict__ win, uint32_t W1,
                                             uint32_t A, uint32_t B) {
    __shared__ K1QLds<W> L;
    const int w = threadIdx.x >> 6;
    k1_body_q_sched<W, FAST>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], W1, A, B);
}

// the product body over its two-group plan (round 5: A/B'd against a copy with the trimmed resolve
// rounds the product then took -- 81.5-82.1 vs 80.6-81.0 us, profiles/r05/micro_k1o_trim.jsonl)
template <int W, bool FAST, bool TRIM>
__global__ __launch_bounds__(256) void k1_qp(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                             uint64_t n_groups, unsigned long long* __restrict__ win, uint32_t W1,
                                             uint32_t A, uint32_t B) {
    __shared__ K1QLds<W> L;
    const int w = threadIdx.x >> 6;
    (void)TRIM;
    k1_body_q<W, FAST>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], W1, A, B);
}

// the product body with the workgroup-pooled tail (round 6; k1_qp keeps the per-wave tail)
template <int W, bool FAST>
__global__ __launch_bounds__(256) void k1_qpp(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                              uint64_t n_groups, unsigned long long* __restrict__ win, uint32_t W1,
                                              uint32_t A, uint32_t B) {
    __shared__ K1QLds<W> L;
    const int w = threadIdx.x >> 6;
    k1_body_q<W, FAST>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], W1, A, B, L.pool);
}

// the product body over its plan with each wave's shader clock stamped at entry and exit (a separate
// diagnostic kernel, MI355X_MICROARCH.md DVFS item 6: in the product no stamp executes): per wave
// dt = s_memtime ticks (shader cycles), dr = s_memrealtime ticks (100 MHz) -> the in-kernel clock
template <int W, bool FAST>
__global__ __launch_bounds__(256) void k1_qclk(DrawKey dk, uint32_t k, uint64_t lo, uint64_t hi, uint64_t g_begin,
                                               uint64_t n_groups, unsigned long long* __restrict__ win, uint32_t W1,
                                               uint32_t A, uint32_t B, unsigned long long* __restrict__ stamps) {
    __shared__ K1QLds<W> L;
    const int w = threadIdx.x >> 6;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    k1_body_q<W, FAST>(dk, k, lo, hi, g_begin, n_groups, win, L.q[w], L.cq[w], W1, A, B);
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) {  // vector stores
        stamps[2 * wave] = t1 - t0;
        stamps[2 * wave + 1] = r1 - r0;
    }
}

// a stand-in for a collective running beside K1 (RCCL's all-gather kernel: a few workgroups for tens
// of us): `blocks` workgroups of 256 threads that spin for `ns` nanoseconds of wall clock
__global__ __launch_bounds__(256) void occupy(uint64_t ns) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while ((__builtin_amdgcn_s_memrealtime() - t0) * 10 < ns) __builtin_amdgcn_s_sleep(2);
}

template <bool NOP>
__global__ void fold_check(const uint32_t* in, uint32_t* out) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    const uint32_t xa = in[2 * t], xb = in[2 * t + 1];
    uint32_t z, bits = 0;
    if (NOP) asm volatile("v_or_b32_sdwa %0, %2, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "s_nop 0\n\t"
        "v_or_b32_sdwa %0, %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "s_nop 0\n\t"
        "v_cmp_ne_u32_e32 vcc, -1, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
        : "=&v"(z), "+v"(bits)
        : "v"(xa), "v"(xb)
        : "vcc");
    else asm volatile("v_or_b32_sdwa %0, %2, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "v_or_b32_sdwa %0, %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1\n\t"
        "v_cmp_ne_u32_e32 vcc, -1, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
        : "=&v"(z), "+v"(bits)
        : "v"(xa), "v"(xb)
        : "vcc");
    out[2 * t] = z;
    out[2 * t + 1] = bits;
}

int main(int argc, char** argv) {
    for (int nop = 0; nop < 2; ++nop) {  // the pair fold's SDWA + mark: z = fold(xa) | fold(xb) << 16, bits = (z != ~0)
        const int N = 64 * 4096;
        std::vector<uint32_t> in(2 * N), out(2 * N);
        uint64_t st = 0x9E3779B97F4A7C15ull;
        for (int t = 0; t < 2 * N; ++t) {
            st ^= st << 13; st ^= st >> 7; st ^= st << 17;
            uint32_t v = (uint32_t)st;
            if ((st >> 40) % 3 == 0) v |= 0xFFFF0000u >> (16 * (t & 1));  // fold 0xFFFF often
            if ((st >> 44) % 5 == 0) v = 0xFFFF0000u;
            in[t] = v;
        }
        uint32_t *di, *dout;
        CK(hipMalloc(&di, 8 * N));
        CK(hipMalloc(&dout, 8 * N));
        CK(hipMemcpy(di, in.data(), 8 * N, hipMemcpyHostToDevice));
        int bad = 0;
        for (int rep = 0; rep < 20; ++rep) {
            if (nop) hipLaunchKernelGGL(fold_check<true>, dim3(N / 64), dim3(64), 0, 0, di, dout);
            else hipLaunchKernelGGL(fold_check<false>, dim3(N / 64), dim3(64), 0, 0, di, dout);
            CK(hipMemcpy(out.data(), dout, 8 * N, hipMemcpyDeviceToHost));
            for (int t = 0; t < N; ++t) {
                const uint32_t fa = (in[2 * t] | (in[2 * t] >> 16)) & 0xFFFFu, fb = (in[2 * t + 1] | (in[2 * t + 1] >> 16)) & 0xFFFFu;
                const uint32_t z = fa | (fb << 16);
                if (out[2 * t] != z || out[2 * t + 1] != (uint32_t)(z != 0xFFFFFFFFu)) ++bad;
            }
        }
        CK(hipFree(di));
        CK(hipFree(dout));
        printf("{\"fold_check_nop\": %d, \"bad\": %d, \"of\": %d}\n", nop, bad, 20 * N);
    }    const uint64_t n = 1000000000ull, lo = 1024, n_groups = (n + 15) / 16;
    const uint32_t k = 1024;
    DrawKey dk{0xC0FFEE, 0, 0x5A5A, 0};
    unsigned long long* win;
    CK(hipMalloc(&win, k * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> ref(k), got(k);
    auto run = [&](auto kern, int grid, std::vector<unsigned long long>& out) -> int {
        CK(hipMemset(win, 0, k * 8));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win);
        CK(hipMemcpy(out.data(), win, k * 8, hipMemcpyDeviceToHost));
        return 0;
    };
    auto time_v = [&](auto kern, const char* name, int grid) -> int {
        for (int rep = 0; rep < 3; ++rep)
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win);
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int rep = 0; rep < reps; ++rep)
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (run(kern, grid, got)) return 1;
        printf("{\"kernel\": \"%s\", \"grid\": %d, \"us\": %.2f, \"winners_match\": %s}\n", name, grid,
               ms / reps * 1e3, got == ref ? "true" : "false");
        return 0;
    };
    if (run(k1_base, 3072, ref)) return 1;
    // argv: passes, then grids (each pass visits every grid, in the given order)
    if (argc > 1 && argv[1][0] == 'd') {  // counters of one pair10 launch
        unsigned long long z[8] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof z));
        if (run(k1_pair<10>, 4096, got)) return 1;
        if (run(k1_base, 4096, got)) return 1;
        CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(g_dbg), sizeof z));
        printf("{\"resolves\": %llu, \"valid\": %llu, \"dense\": %llu, \"windows\": %llu, \"rounds\": %llu, "
               "\"pushed\": %llu, \"base_pushed\": %llu, \"match\": %s}\n", z[0], z[1], z[2], z[3], z[4], z[5], z[6], got == ref ? "true" : "false");
        return 0;
    }
    if (argc > 1 && (argv[1][0] == 't' || argv[1][0] == 'p')) {
        // t: the final partial rounds' cost (the body with / without them).  p (round 5, removed): the
        // workgroup's leftovers handed to its last wave -- slower, the workgroup slot stays held while
        // that wave resolves them alone (profiles/r05/micro_k1o_pool_ab.jsonl)
        for (int p = 0; p < 3; ++p)
            for (int g : {5086, 3072}) {
                if (time_v(k1_qd<12, true, false>, "q12fast_perwave", g)) return 1;
                if (time_v(k1_qd<12, true, true>, "q12fast_skiptail(wrong)", g)) return 1;
            }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'c') {  // K1 beside a concurrent occupier kernel: plan vs grid-stride
        const uint32_t W1 = 6144, A = 10, B = 2;
        const uint64_t units = (n_groups + 767) / 768, waves = W1 + (units - (uint64_t)W1 * A + 1) / 2;
        const int pgrid = (int)((waves + 3) / 4);
        hipStream_t s1, s2;
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        for (int rep = 0; rep < 3000; ++rep)
            hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(pgrid), dim3(256), 0, s1, dk, k, lo, n, 0ull, n_groups, win,
                               W1, A, B);
        CK(hipDeviceSynchronize());
        for (int occ : {0, 16, 64}) {
            for (int p = 0; p < 3; ++p)
                for (int v = 0; v < 2; ++v) {
                    float tot = 0;
                    const int reps = 20;
                    for (int rep = 0; rep < reps; ++rep) {
                        CK(hipEventRecord(e0, s1));
                        if (v == 0)
                            hipLaunchKernelGGL((k1_q<12, true>), dim3(5086), dim3(256), 0, s1, dk, k, lo, n, 0ull, n_groups, win);
                        else
                            hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(pgrid), dim3(256), 0, s1, dk, k, lo, n, 0ull,
                                               n_groups, win, W1, A, B);
                        if (occ) hipLaunchKernelGGL(occupy, dim3(occ), dim3(256), 0, s2, 30000ull);
                        CK(hipEventRecord(e1, s1));
                        CK(hipEventSynchronize(e1));
                        CK(hipStreamSynchronize(s2));
                        float ms;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        tot += ms;
                    }
                    printf("{\"occupier_blocks\": %d, \"layout\": \"%s\", \"us\": %.2f}\n", occ,
                           v ? "plan" : "grid_stride", tot / reps * 1e3);
                }
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'k') {  // K1's in-kernel clock (stamped diagnostic kernel, see k1_qclk)
        const uint32_t W1 = 6144, A = 10, B = 2;
        const uint64_t units = (n_groups + 767) / 768, waves = W1 + (units - (uint64_t)W1 * A + 1) / 2;
        const int pgrid = (int)((waves + 3) / 4);
        unsigned long long* stamps;
        CK(hipMalloc(&stamps, (size_t)pgrid * 4 * 16));
        // >= 2 s of back-to-back launches first (the clock settles under load)
        for (int rep = 0; rep < 25000; ++rep)
            hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(pgrid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win,
                               W1, A, B);
        CK(hipDeviceSynchronize());
        for (int p = 0; p < 5; ++p) {
            const int reps = 20;
            CK(hipEventRecord(e0));
            for (int rep = 0; rep < reps; ++rep)
                hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(pgrid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups,
                                   win, W1, A, B);
            CK(hipEventRecord(e1));
            hipLaunchKernelGGL((k1_qclk<12, true>), dim3(pgrid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win, W1, A,
                               B, stamps);
            CK(hipDeviceSynchronize());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<unsigned long long> st((size_t)pgrid * 4 * 2);
            CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> clk;
            for (size_t w = 0; w < st.size() / 2; ++w)
                if (st[2 * w + 1] >= 100) clk.push_back((double)st[2 * w] / (double)st[2 * w + 1] * 0.1);  // GHz
            std::sort(clk.begin(), clk.end());
            printf("{\"mode\": \"k1_in_kernel_clock\", \"launch_us\": %.2f, \"waves\": %zu, \"clock_GHz_median\": %.3f, "
                   "\"clock_GHz_p10\": %.3f, \"clock_GHz_p90\": %.3f}\n", ms / reps * 1e3, clk.size(),
                   clk[clk.size() / 2], clk[clk.size() / 10], clk[clk.size() * 9 / 10]);
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'o') {  // round 6: per-wave vs workgroup-pooled tail; argv[2..] "W1:A:B" plans
        // (the r05 schedule body k1_body_q_sched -- round-5 steady and tail -- beside them at 6144:10:2)
        const uint32_t units = (uint32_t)((n_groups + 767) / 768);
        for (int rep = 0; rep < 3000; ++rep)
            hipLaunchKernelGGL((k1_qpp<12, true>), dim3(4024), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win, 6144u,
                               10u, 2u);
        CK(hipDeviceSynchronize());
        for (int p = 0; p < 3; ++p)
            for (int a = 2; a < argc; ++a) {
                unsigned W1, A, B;
                if (sscanf(argv[a], "%u:%u:%u", &W1, &A, &B) != 3) return 2;
                const uint64_t rest = (uint64_t)units > (uint64_t)W1 * A ? units - (uint64_t)W1 * A : 0;
                const uint64_t waves = std::min<uint64_t>(W1, (units + A - 1) / A) + (rest + B - 1) / B;
                const int grid = (int)((waves + 3) / 4);
                for (int v = 0; v < 3; ++v) {
                    if (v == 2 && !(W1 == 6144 && A == 10 && B == 2)) continue;
                    auto launch = [&]() {
                        if (v == 0)
                            hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull,
                                               n_groups, win, W1, A, B);
                        else if (v == 1)
                            hipLaunchKernelGGL((k1_qpp<12, true>), dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups,
                                               win, W1, A, B);
                        else
                            hipLaunchKernelGGL((k1_qs<12, true>), dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups,
                                               win, W1, A, B);
                    };
                    for (int rep = 0; rep < 3; ++rep) launch();
                    const int reps = 20;
                    CK(hipEventRecord(e0));
                    for (int rep = 0; rep < reps; ++rep) launch();
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    CK(hipMemset(win, 0, k * 8));
                    launch();
                    CK(hipMemcpy(got.data(), win, k * 8, hipMemcpyDeviceToHost));
                    printf("{\"mode\": \"tail\", \"body\": \"%s\", \"W1\": %u, \"A\": %u, \"B\": %u, \"grid\": %d, "
                           "\"us\": %.2f, \"winners_match\": %s}\n",
                           v == 0 ? "per_wave_tail" : v == 1 ? "pooled_tail" : "r05_sched_body", W1, A, B, grid,
                           ms / reps * 1e3, got == ref ? "true" : "false");
                }
            }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'w') {  // window length under the two-group plan: W = 8 / 12 / 16
        auto plan_for = [&](uint64_t UB, uint32_t& A) {
            const uint64_t units = (n_groups + UB - 1) / UB;
            A = (uint32_t)((units * 755 / 1000 + 3072) / 6144);
            const uint64_t waves = 6144 + (units - 6144ull * A + 1) / 2;
            return (int)((waves + 3) / 4);
        };
        uint32_t A8, A12, A16;
        const int g8 = plan_for(512, A8), g12 = plan_for(768, A12), g16 = plan_for(1024, A16);
        for (int rep = 0; rep < 3000; ++rep)
            hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(g12), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win,
                               6144u, A12, 2u);
        CK(hipDeviceSynchronize());
        for (int p = 0; p < 4; ++p)
            for (int v = 0; v < 3; ++v) {
                auto launch = [&]() {
                    if (v == 0)
                        hipLaunchKernelGGL((k1_qp<8, true, false>), dim3(g8), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups,
                                           win, 6144u, A8, 2u);
                    else if (v == 1)
                        hipLaunchKernelGGL((k1_qp<12, true, false>), dim3(g12), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups,
                                           win, 6144u, A12, 2u);
                    else
                        hipLaunchKernelGGL((k1_qp<16, true, false>), dim3(g16), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups,
                                           win, 6144u, A16, 2u);
                };
                for (int rep = 0; rep < 3; ++rep) launch();
                const int reps = 20;
                CK(hipEventRecord(e0));
                for (int rep = 0; rep < reps; ++rep) launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipMemset(win, 0, k * 8));
                launch();
                CK(hipMemcpy(got.data(), win, k * 8, hipMemcpyDeviceToHost));
                printf("{\"W\": %d, \"us\": %.2f, \"winners_match\": %s}\n", v == 0 ? 8 : v == 1 ? 12 : 16,
                       ms / reps * 1e3, got == ref ? "true" : "false");
            }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'n') {  // the product's grid-stride grid vs its two-group plan over sizes
        // (replicas of rsv_elements.hip k1_grid / k1_plan); argv[2..]: draw counts
        for (int a = 2; a < argc; ++a) {
            const uint64_t nn = (uint64_t)atof(argv[a]), ng = (nn + 15) / 16 - lo / 16;
            const uint64_t per_window = 2ull * 256 * 12;
            uint64_t g;
            if (ng < per_window * 768) g = std::min<uint64_t>((ng / 2 + 255) / 256, 256 * 20);
            else {
                const uint64_t mm = std::max<uint64_t>(1, (ng + per_window * 5120 / 2) / (per_window * 5120));
                g = std::max<uint64_t>(1, ng / (per_window * mm));
            }
            const uint64_t units = (ng + 767) / 768, A = (units * 755 / 1000 + 3072) / 6144;
            const bool plan = ng >= per_window * 768 && A >= 4;
            const uint64_t waves = plan ? 6144 + (units - 6144 * A + 1) / 2 : 0;
            const int pg = plan ? (int)((waves + 3) / 4) : 0;
            std::vector<unsigned long long> r0(k), r1(k);
            float best0 = 1e9f, best1 = 1e9f;
            for (int p = 0; p < 3; ++p) {
                for (int v = 0; v < 2; ++v) {
                    if (v == 1 && !plan) continue;
                    auto launch = [&]() {
                        if (v == 0)
                            hipLaunchKernelGGL((k1_q<12, true>), dim3((unsigned)g), dim3(256), 0, 0, dk, k, lo, nn, lo / 16, ng, win);
                        else
                            hipLaunchKernelGGL((k1_qs<12, true>), dim3(pg), dim3(256), 0, 0, dk, k, lo, nn, lo / 16, ng, win,
                                               6144u, (uint32_t)A, 2u);
                    };
                    for (int rep = 0; rep < 3; ++rep) launch();
                    const int reps = 10;
                    CK(hipEventRecord(e0));
                    for (int rep = 0; rep < reps; ++rep) launch();
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    CK(hipMemset(win, 0, k * 8));
                    launch();
                    CK(hipMemcpy((v ? r1 : r0).data(), win, k * 8, hipMemcpyDeviceToHost));
                    float& b = v ? best1 : best0;
                    b = std::min(b, ms / reps * 1000.0f);
                }
            }
            printf("{\"n\": %.3g, \"grid_stride_us\": %.2f, \"grid\": %llu, \"plan_A\": %llu, \"plan_grid\": %d, \"plan_us\": %.2f, "
                   "\"winners_match\": %s}\n", (double)nn, best0, (unsigned long long)g, plan ? (unsigned long long)A : 0ull,
                   pg, plan ? best1 : 0.0f, plan ? (r0 == r1 ? "true" : "false") : "null");
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {  // static two-group schedules vs the product grid
        // argv[2..]: "W1:A:B" triples (W1 waves of A half windows, the rest B each)
        const uint32_t units = (uint32_t)((n_groups + 767) / 768);
        for (int p = 0; p < 3; ++p) {
            if (time_v(k1_q<12, true>, "q12fast", 5086)) return 1;
            for (int a = 2; a < argc; ++a) {
                unsigned W1, A, B;
                if (sscanf(argv[a], "%u:%u:%u", &W1, &A, &B) != 3) return 2;
                const uint64_t rest = (uint64_t)units > (uint64_t)W1 * A ? units - (uint64_t)W1 * A : 0;
                const uint64_t waves = std::min<uint64_t>(W1, (units + A - 1) / A) + (rest + B - 1) / B;
                const int grid = (int)((waves + 3) / 4);
                auto launch = [&]() {
                    hipLaunchKernelGGL((k1_qs<12, true>), dim3(grid), dim3(256), 0, 0, dk, k, lo, n, 0ull, n_groups, win,
                                       W1, A, B);
                };
                for (int rep = 0; rep < 3; ++rep) launch();
                const int reps = 20;
                CK(hipEventRecord(e0));
                for (int rep = 0; rep < reps; ++rep) launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipMemset(win, 0, k * 8));
                launch();
                CK(hipMemcpy(got.data(), win, k * 8, hipMemcpyDeviceToHost));
                printf("{\"kernel\": \"q12fast_sched\", \"W1\": %u, \"A\": %u, \"B\": %u, \"grid\": %d, \"us\": %.2f, "
                       "\"winners_match\": %s}\n", W1, A, B, grid, ms / reps * 1e3, got == ref ? "true" : "false");
            }
        }
        return 0;
    }
    const int passes = argc > 1 ? atoi(argv[1]) : 2;
    std::vector<int> grids;
    for (int a = 2; a < argc; ++a) grids.push_back(atoi(argv[a]));
    if (grids.empty()) grids = {2048, 3072, 4096, 6144};
    for (int p = 0; p < passes; ++p)
        for (int g : grids) {
            if (time_v(k1_base, "base", g)) return 1;
            if (time_v(k1_pair<12>, "pair12", g)) return 1;
            if (time_v(k1_q<12>, "q12", g)) return 1;
            if (time_v(k1_q<12, true>, "q12fast", g)) return 1;
        }
    return 0;
}
