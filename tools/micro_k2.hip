// micro_k2.hip -- K2 (segmented, rsv_k2.h) variant timing at C3's shape: 2^20 streams x 4096 keys,
// k = 64 (development tool, not product).  Variants: 0 = product kernel, 1 = no winner-key gather,
// 2 = no level-1 Philox, 8 = candidates dropped after the FIFO append, 9 = 8 + 1, 16 = the
// winner keys stored right after their gather (the product defers the store by one stream),
// 8192 = the 8-plane candidate mask for every block (the product takes 4 planes once T <= 16),
// 512 = the dense head [k, 4k) uncut (the product cuts it to whole 64-pair rounds), 16384 / 32768 =
// heads [k, 6k) / [k, 8k) (cut to whole rounds).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro_k2.hip -o tools/micro_k2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "k2_dev_variants.h"  // the round-4 kernel + cost-probe variants
#include "../reservoir_amd/csrc/rsv_k2.h"  // the product kernel (mode n: the product against variant 0)
namespace kd = rsv::k2dev;

using namespace rsv;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ void fill(int64_t* keys, int64_t n, int64_t* offs, int64_t S, int64_t L) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t z = (uint64_t)i + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        keys[i] = (int64_t)(z ^ (z >> 31));
        if (i <= S && i * L <= n) offs[i] = i * L;
    }
}

int main(int argc, char** argv) {
    const int64_t S = 1 << 20, L = 4096, n = S * L;
    const uint32_t k = 64;
    int64_t *keys, *offs, *out, *cnt;
    CK(hipMalloc(&keys, n * 8));
    CK(hipMalloc(&offs, (S + 1) * 8));
    CK(hipMalloc(&out, S * k * 8));
    CK(hipMalloc(&cnt, S * 8));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, keys, n, offs, S, L);
    CK(hipDeviceSynchronize());
    const size_t lds = kd::lds_bytes(k);
    unsigned grid = (unsigned)std::min<int64_t>(S / kd::kWaves, 256 * 128);  // the product's cap (rsv_segmented.hip)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<int64_t> ref(S * k), got(S * k);
    size_t lds_run = lds;
    auto run = [&](auto kern, const char* name, bool check) -> int {
        std::vector<float> ts;
        // the first ~20 launches run on a still-ramping clock (bench.py's ramp note): timed after them
        for (int rep = 0; rep < 45; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kd::kWaves), lds_run, 0, (const int64_t*)keys,
                               (const int64_t*)offs, S, k, 1u, 0u, 0ull, out, cnt, 0xFFFFFFFFu,
                               (unsigned long long*)nullptr);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 25) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f}\n", name, ts[ts.size() / 2], ts[0]);
        if (check) {
            CK(hipMemcpy(got.data(), out, S * k * 8, hipMemcpyDeviceToHost));
            printf("  identical to variant 0: %s\n", got == ref ? "yes" : "NO");
        }
        return 0;
    };
    // the product kernel (rsv_k2.h) through its own launch shape, timed like run()
    auto run_product = [&](const char* name) -> int {
        std::vector<float> ts;
        const size_t plds = rsv::k2::lds_bytes(k);
        const unsigned pgrid = (unsigned)std::min<int64_t>((S + rsv::k2::kWaves - 1) / rsv::k2::kWaves, 256 * 128);
        for (int rep = 0; rep < 45; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(rsv::k2::k2_segmented<int64_t>, dim3(pgrid), dim3(64 * rsv::k2::kWaves), plds, 0,
                               (const int64_t*)keys, (const int64_t*)offs, S, k, 1u, 0u, 0ull, out, cnt,
                               rsv::k2::kQCap);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 25) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"min_ms\": %.4f}\n", name, ts[ts.size() / 2], ts[0]);
        CK(hipMemcpy(got.data(), out, S * k * 8, hipMemcpyDeviceToHost));
        printf("  identical to variant 0: %s\n", got == ref ? "yes" : "NO");
        return 0;
    };
    if (run(kd::k2_segmented<int64_t, 0>, "0 wave-per-stream", false)) return 1;
    CK(hipMemcpy(ref.data(), out, S * k * 8, hipMemcpyDeviceToHost));
    if (argc > 1 && argv[1][0] == 'n') {  // the product kernel against the round-4 form (A/B/A/B)
        for (int rep = 0; rep < 2; ++rep) {
            if (run_product("product rsv_k2.h")) return 1;
            if (run(kd::k2_segmented<int64_t, 0>, "0 round-4 copy (k2_dev_variants.h)", true)) return 1;
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'o') {  // occupancy sensitivity: the product with its LDS padded
        CK(hipFuncSetAttribute((const void*)kd::k2_segmented<int64_t, 0>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        for (size_t pad : {lds, (size_t)(160 * 1024 / 3), (size_t)(160 * 1024 / 2)}) {
            lds_run = pad;
            char name[64];
            snprintf(name, sizeof name, "0 product, %zu B LDS per workgroup", pad);
            if (run(kd::k2_segmented<int64_t, 0>, name, true)) return 1;
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'l') return 0;  // the two product forms only
    if (argc > 1 && argv[1][0] == 'p') return 0;  // one variant only (rocprofv3 --pmc passes)
    if (argc > 1 && argv[1][0] == 'q') {  // occupancy: the 2048-entry FIFO (4 workgroups per CU)
        lds_run = kd::lds_bytes(k, 128);
        if (run(kd::k2_segmented<int64_t, 128>, "128 FIFO 2048 entries", true)) return 1;
        lds_run = kd::lds_bytes(k, 256);
        if (run(kd::k2_segmented<int64_t, 256>, "256 stash ring of 2 iterations", true)) return 1;
        lds_run = lds;
        if (run(kd::k2_segmented<int64_t, 0>, "0 product (again)", true)) return 1;
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'g') {  // A/B/A against the previous masks and the gather-free forms
        if (run(kd::k2_segmented<int64_t, 8192>, "8192 8-plane masks everywhere (r02 up to here)", true)) return 1;
        if (run(kd::k2_segmented<int64_t, 0>, "0 product (again)", true)) return 1;
        if (run(kd::k2_segmented<int64_t, 8193>, "8193 8-plane masks, no gather", false)) return 1;
        if (run(kd::k2_segmented<int64_t, 1>, "1 no gather", false)) return 1;
        if (run(kd::k2_segmented<int64_t, 8192>, "8192 (again)", true)) return 1;
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'c') {  // cost split of the level-0 side (no gather, no resolve)
        if (run(kd::k2_segmented<int64_t, 9>, "9 dropped + no gather", false)) return 1;
        if (run(kd::k2_segmented<int64_t, 9 | 1024>, "9 + no head", false)) return 1;
        if (run(kd::k2_segmented<int64_t, 9 | 1024 | 2048>, "9 + no head + no append", false)) return 1;
        if (run(kd::k2_segmented<int64_t, 9 | 1024 | 2048 | 4096>, "9 + no head + no append + no candidates", false)) return 1;
        if (run(kd::k2_segmented<int64_t, 1 | 1024>, "1 + no head (resolve kept)", false)) return 1;
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'G') {  // grid sweep of the product (argv[2..]: grids)
        for (int pass = 0; pass < 2; ++pass)
            for (int a = 2; a < argc; ++a) {
                grid = (unsigned)atoi(argv[a]);
                char name[64];
                snprintf(name, sizeof name, "0 product, grid %u", grid);
                if (run(kd::k2_segmented<int64_t, 0>, name, true)) return 1;
            }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'r') {  // dense head cut to whole 64-pair rounds vs uncut (A/B/A/B)
        for (int rep = 0; rep < 2; ++rep) {
            if (run(kd::k2_segmented<int64_t, 512>, "512 head [k, 4k) uncut (r02)", true)) return 1;
            if (run(kd::k2_segmented<int64_t, 0>, "0 product (again)", true)) return 1;
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'm') {  // head multiplier 4 (product) vs 6, 8 (whole rounds)
        for (int rep = 0; rep < 2; ++rep) {
            if (run(kd::k2_segmented<int64_t, 16384>, "16384 head [k, 6k) in whole rounds", true)) return 1;
            if (run(kd::k2_segmented<int64_t, 32768>, "32768 head [k, 8k) in whole rounds", true)) return 1;
            if (run(kd::k2_segmented<int64_t, 0>, "0 product (again)", true)) return 1;
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'h') {  // dense-head multiplier: 4 (product), 2, none
        if (run(kd::k2_segmented<int64_t, 32>, "32 head [k, 2k)", true)) return 1;
        if (run(kd::k2_segmented<int64_t, 64>, "64 no head (all through the FIFO)", true)) return 1;
        if (run(kd::k2_segmented<int64_t, 0>, "0 product (again)", true)) return 1;
        return 0;
    }
    if (run(kd::k2_segmented<int64_t, 1>, "1 no gather", false)) return 1;
    if (run(kd::k2_segmented<int64_t, 2>, "2 no level-1 philox", false)) return 1;
    if (run(kd::k2_segmented<int64_t, 16>, "16 gather stored at once (no deferral)", true)) return 1;
    if (run(kd::k2_segmented<int64_t, 8>, "8 candidates dropped", false)) return 1;
    if (run(kd::k2_segmented<int64_t, 9>, "9 dropped + no gather", false)) return 1;
    if (run(kd::k2_segmented<int64_t, 0>, "0 product (again)", true)) return 1;
    return 0;
}
