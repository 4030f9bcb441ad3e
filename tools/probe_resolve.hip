// probe_resolve.hip -- where the ~5 us of resolve_publish_kernel go (development probe, not part of
// the library).  One workgroup resolves k = 1024 slots as rsv_elements.hip does: the slot's winner
// index (win[j]) -> its key (a random 8-B read of a 8 GB key buffer) -> slot arrays + the first m keys
// into coherent host memory -> a system-scope release of the flag.  Variants drop one stage at a
// time; "warm" runs the full form right after the same gather, so the key lines are cached.
// Kernel time by hipExtLaunchKernelGGL start/stop events (the kernel alone), median of 200.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_resolve.hip -o tools/probe_resolve
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__device__ __forceinline__ void publish(uint32_t* flag, uint32_t gen) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// V: 0 full; 1 no key gather (the index stands in); 2 device dst instead of host; 3 no publication
template <int V>
__global__ __launch_bounds__(1024) void resolve(const int64_t* __restrict__ keys, uint32_t k,
                                                unsigned long long* __restrict__ win, int64_t* __restrict__ slot_key,
                                                int64_t* __restrict__ slot_idx, int64_t* dst, uint32_t* flag,
                                                uint32_t gen) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        const unsigned long long wi = win[j];
        int64_t v = slot_key[j];
        if (wi) {
            v = V == 1 ? (int64_t)wi : keys[wi];
            slot_key[j] = v;
            slot_idx[j] = (int64_t)wi;
        }
        dst[j] = v;
    }
    if (V != 3) publish(flag, gen);
}

// 256 threads, 4 slots each: every load of a lane issued before any use
__global__ __launch_bounds__(256) void resolve4(const int64_t* __restrict__ keys, uint32_t k,
                                                unsigned long long* __restrict__ win, int64_t* __restrict__ slot_key,
                                                int64_t* __restrict__ slot_idx, int64_t* dst, uint32_t* flag,
                                                uint32_t gen) {
    unsigned long long wi[4];
    int64_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t j = threadIdx.x + r * 256;
        wi[r] = j < k ? win[j] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t j = threadIdx.x + r * 256;
        v[r] = wi[r] ? keys[wi[r]] : (j < k ? slot_key[j] : 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t j = threadIdx.x + r * 256;
        if (j >= k) continue;
        if (wi[r]) {
            slot_key[j] = v[r];
            slot_idx[j] = (int64_t)wi[r];
        }
        dst[j] = v[r];
    }
    publish(flag, gen);
}

__global__ void gather_only(const int64_t* __restrict__ keys, const unsigned long long* __restrict__ win, uint32_t k,
                            int64_t* out) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) out[j] = keys[win[j]];
}

__global__ void reset(unsigned long long* win, const unsigned long long* src, uint32_t k) {
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) win[j] = src[j];
}

int main() {
    const uint64_t n = 1000000000ull;
    const uint32_t k = 1024;
    int64_t *keys, *slot_key, *slot_idx, *ddst, *hdst, *tmp;
    unsigned long long *win, *win_src;
    uint32_t* flag;
    CK(hipMalloc(&keys, n * 8));
    CK(hipMemset(keys, 0x5A, n * 8));
    CK(hipMalloc(&slot_key, k * 8));
    CK(hipMalloc(&slot_idx, k * 8));
    CK(hipMalloc(&ddst, k * 8));
    CK(hipMalloc(&tmp, k * 8));
    CK(hipMalloc(&win, k * 8));
    CK(hipMalloc(&win_src, k * 8));
    CK(hipHostMalloc(&hdst, k * 8, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    int64_t* hdst_dev;
    uint32_t* flag_dev;
    CK(hipHostGetDevicePointer((void**)&hdst_dev, hdst, 0));
    CK(hipHostGetDevicePointer((void**)&flag_dev, flag, 0));
    std::vector<unsigned long long> w(k);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"full", "no_key_gather", "device_dst", "no_publish", "warm_keys", "full_256x4"};
    for (int v = 0; v < 6; ++v) {
        std::vector<float> t;
        for (int rep = 0; rep < 200; ++rep) {
            for (auto& x : w) {  // fresh random winners every time: cold key lines
                s ^= s << 13, s ^= s >> 7, s ^= s << 17;
                x = 1 + s % (n - 1);
            }
            CK(hipMemcpy(win_src, w.data(), k * 8, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(reset, dim3(1), dim3(1024), 0, 0, win, win_src, k);
            if (v == 4) hipLaunchKernelGGL(gather_only, dim3(1), dim3(1024), 0, 0, keys, win, k, tmp);
            const uint32_t gen = rep + 1;
            if (v == 0 || v == 4)
                hipExtLaunchKernelGGL(resolve<0>, dim3(1), dim3(1024), 0, 0, e0, e1, 0, keys, k, win, slot_key, slot_idx,
                                      hdst_dev, flag_dev, gen);
            else if (v == 1)
                hipExtLaunchKernelGGL(resolve<1>, dim3(1), dim3(1024), 0, 0, e0, e1, 0, keys, k, win, slot_key, slot_idx,
                                      hdst_dev, flag_dev, gen);
            else if (v == 5)
                hipExtLaunchKernelGGL(resolve4, dim3(1), dim3(256), 0, 0, e0, e1, 0, keys, k, win, slot_key, slot_idx,
                                      hdst_dev, flag_dev, gen);
            else if (v == 2)
                hipExtLaunchKernelGGL(resolve<2>, dim3(1), dim3(1024), 0, 0, e0, e1, 0, keys, k, win, slot_key, slot_idx,
                                      ddst, flag_dev, gen);
            else
                hipExtLaunchKernelGGL(resolve<3>, dim3(1), dim3(1024), 0, 0, e0, e1, 0, keys, k, win, slot_key, slot_idx,
                                      hdst_dev, flag_dev, gen);
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1000.0f);
        }
        std::sort(t.begin(), t.end());
        printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", names[v], t[t.size() / 2],
               t[t.size() / 10], t[t.size() * 9 / 10]);
    }
    return 0;
}
