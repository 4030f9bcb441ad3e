// micro_k1o.hip -- K1 occupancy A/B (development tool, not product): the product body k1_body_z
// compiled with the default register allocation (.sgpr_count 100 -> 6 workgroups of 256 per CU,
// MI355X_MICROARCH.md "Residency") and with amdgpu_num_sgpr limits that admit 8, over a grid sweep.
// Every variant's winner table is checked against the default's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include tools/micro_k1o.hip -o tools/micro_k1o
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "../reservoir_amd/csrc/rsv_device.h"
#include "../reservoir_amd/csrc/rsv_scan.h"

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

int main(int argc, char** argv) {
    const uint64_t n = 1000000000ull, lo = 1024, n_groups = (n + 15) / 16;
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
    const int passes = argc > 1 ? atoi(argv[1]) : 2;
    std::vector<int> grids;
    for (int a = 2; a < argc; ++a) grids.push_back(atoi(argv[a]));
    if (grids.empty()) grids = {2048, 3072, 4096, 6144};
    for (int p = 0; p < passes; ++p)
        for (int g : grids) {
            if (time_v(k1_base, "base", g)) return 1;
            if (time_v(k1_s80, "s80", g)) return 1;
        }
    return 0;
}
