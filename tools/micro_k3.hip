// micro_k3.hip -- K3 filter streaming-read variants (development tool): bytes/s of a pass that
// loads 8-B keys, computes the Sampler.distinct scrambled hash and compares it with a threshold no
// key passes (the steady-state case), by unroll U, grid and load flavour.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro_k3.hip -o tools/micro_k3
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../reservoir_amd/csrc/rsv_device.h"

using namespace rsv;
typedef long long v2i64 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

template <int U, int NT>
__global__ __launch_bounds__(256) void filt(const v2i64* __restrict__ kv, int64_t n_vec, int64_t r0, int64_t r1,
                                            int64_t tinc, unsigned long long* cnt) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t full = n_vec / (T * U);
    uint32_t c = 0;
    for (int64_t it = 0; it < full; ++it) {
        const int64_t v0 = it * T * U + tid;
        v2i64 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = NT ? __builtin_nontemporal_load(kv + v0 + u * T) : kv[v0 + u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            c += scramble(r0, r1, x[u][0]) <= tinc;
            c += scramble(r0, r1, x[u][1]) <= tinc;
        }
    }
    if (c) atomicAdd(cnt, c);
}

template <int U, int NT>
int run(const v2i64* d, int64_t n_vec, unsigned long long* cnt, int grid, const char* name) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((filt<U, NT>), dim3(grid), dim3(256), 0, 0, d, n_vec, 1, 2, INT64_MIN, cnt);
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((filt<U, NT>), dim3(grid), dim3(256), 0, 0, d, n_vec, 1, 2, INT64_MIN, cnt);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double s = ms / reps * 1e-3;
    printf("%-10s U=%d grid %5d  %8.1f us  %6.2f TB/s\n", name, U, grid, s * 1e6, n_vec * 16.0 / s / 1e12);
    return 0;
}

__global__ void fill_random(int64_t* p, int64_t n) {  // splitmix64 of the index (the C4 keys' shape)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = (int64_t)(z ^ (z >> 31));
    }
}

int main(int argc, char** argv) {
    const int64_t n = 500000000;  // C4 per-GPU share: 5e8 int64 keys = 4 GB
    v2i64* d;
    CK(hipMalloc(&d, n * 8));
    // argv[1] == "random": splitmix64 keys (the product's data); default: a constant byte (r02)
    if (argc > 1 && argv[1][0] == 'r') {
        hipLaunchKernelGGL(fill_random, dim3(8192), dim3(256), 0, 0, (int64_t*)d, n);
        CK(hipDeviceSynchronize());
    } else {
        CK(hipMemset(d, 0x5A, n * 8));
    }
    unsigned long long* cnt;
    CK(hipMalloc(&cnt, 8));
    const int64_t nv = n / 2;
    for (int grid : {4096, 8192, 16384}) {
        if (run<4, 1>(d, nv, cnt, grid, "nt")) return 1;
        if (run<8, 1>(d, nv, cnt, grid, "nt")) return 1;
        if (run<8, 0>(d, nv, cnt, grid, "plain")) return 1;
        if (run<16, 1>(d, nv, cnt, grid, "nt")) return 1;
    }
    return 0;
}
