// micro_gather.hip -- the memory floor of K2's winner-key gather at C3's shape (development tool, not
// product): 2^20 streams x 4096 int64 keys, 64 winners per stream at uniform random positions (the
// last writer of a slot is uniform on [0, n)), one wave per stream, lane j loads keys[off + w_j] and
// stores the 64-key output row.  Prints the kernel time and the implied bytes per winner at a given
// bandwidth.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro_gather.hip -o tools/micro_gather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ void fill(int64_t* keys, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) keys[i] = (int64_t)mix(i);
}

// MODE 0: gather + store; MODE 1: store only (index as the value); MODE 2: gather with the winner
// positions sorted within the stream (same lines, ascending order)
template <int MODE>
__global__ __launch_bounds__(256) void gather(const int64_t* __restrict__ keys, int64_t S, int L,
                                              int64_t* __restrict__ out, uint64_t salt) {
    const int lane = threadIdx.x & 63;
    const int64_t wstride = (int64_t)gridDim.x * 4;
    for (int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < S; s += wstride) {
        uint32_t w = (uint32_t)(mix(((uint64_t)s << 6 | lane) ^ salt) % (uint64_t)L);
        if (MODE == 2) {  // bitonic sort of the 64 positions across the wave
            for (int size = 2; size <= 64; size <<= 1)
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    const uint32_t o = (uint32_t)__shfl_xor((int)w, stride);
                    const bool up = (lane & size) == 0, lower = (lane & stride) == 0;
                    w = (lower == up) ? min(w, o) : max(w, o);
                }
        }
        const int64_t v = MODE == 1 ? (int64_t)w : keys[s * L + w];
        out[s * 64 + lane] = v;
    }
}

// The byte basis of a random 8-B gather (does a lone 8-B load move a 64-B half-line or
// the whole 128-B line?).  Every wave loads 64 words of its stream at KNOWN line positions:
//   LINE 0: 64 distinct 128-B lines, word 0 of each                    -> 64 lines, 64 half-lines
//   LINE 1: 32 distinct lines, words 0 and 8 (both 64-B halves)         -> 32 lines, 64 half-lines
//   LINE 2: 32 distinct lines, words 0 and 1 (the same 64-B half twice) -> 32 lines, 32 half-lines
// 128-B fetches: LINE 1 costs what LINE 2 costs (and half of LINE 0); 64-B fetches: LINE 1 costs
// what LINE 0 costs.  Read with rocprofv3 --pmc TCC_EA0_RDREQ_sum (requests) and kernel time.
template <int LINE>
__global__ __launch_bounds__(256) void line_probe(const int64_t* __restrict__ keys, int64_t S, int L,
                                                  int64_t* __restrict__ out, uint64_t salt) {
    const int lane = threadIdx.x & 63;
    const int64_t wstride = (int64_t)gridDim.x * 4;
    const uint32_t lines = (uint32_t)L / 16;  // 128-B lines per stream (256 at L = 4096)
    for (int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < S; s += wstride) {
        const uint32_t base = (uint32_t)(mix((uint64_t)s ^ salt) % lines);
        uint32_t line, word;
        if (LINE == 0) {
            line = (base + 4u * lane) % lines;  // 64 distinct lines (step 4 of 256)
            word = 0;
        } else {
            line = (base + 8u * (lane >> 1)) % lines;  // 32 distinct lines, two loads each
            word = LINE == 1 ? 8u * (lane & 1) : (lane & 1);
        }
        out[s * 64 + lane] = keys[s * L + line * 16 + word];
    }
}

int main() {
    const int64_t S = 1 << 20, L = 4096, n = S * L;
    int64_t *keys, *out;
    CK(hipMalloc(&keys, n * 8));
    CK(hipMalloc(&out, S * 64 * 8));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, keys, n);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](auto kern, const char* name, unsigned grid) -> int {
        std::vector<float> ts;
        for (int rep = 0; rep < 9; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, (const int64_t*)keys, S, (int)L, out,
                               (uint64_t)rep * 0x9E3779B97F4A7C15ULL);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double ms = ts[ts.size() / 2];
        printf("{\"variant\": \"%s\", \"grid\": %u, \"median_ms\": %.4f, \"min_ms\": %.4f, "
               "\"bytes_per_winner_at_6.3TBs\": %.1f}\n",
               name, grid, ms, ts[0], ms * 1e-3 * 6.3e12 / (double)(S * 64));
        return 0;
    };
    const char* only = getenv("MICRO_GATHER_ONLY");  // "lines": the byte-basis probes alone (PMC runs)
    if (!(only && only[0] == 'l'))
        for (unsigned grid : {4096u, 16384u, 262144u}) {
            if (run(gather<0>, "gather", grid)) return 1;
            if (run(gather<2>, "gather sorted", grid)) return 1;
            if (run(gather<1>, "store only", grid)) return 1;
        }
    for (int rep = 0; rep < 2; ++rep) {
        if (run(line_probe<0>, "lines: 64 distinct 128-B lines, word 0", 16384u)) return 1;
        if (run(line_probe<1>, "lines: 32 lines x both 64-B halves", 16384u)) return 1;
        if (run(line_probe<2>, "lines: 32 lines x one 64-B half twice", 16384u)) return 1;
    }
    return 0;
}
