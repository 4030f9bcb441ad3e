// probe_latency.hip -- host<->device round-trip costs of the small tail of a sampler step
// (development probe, not part of the library).  hipcc --offload-arch=gfx950 -O3 probe_latency.hip
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ void empty_kernel() {}

__global__ void copy_kernel(const uint64_t* src, uint64_t* dst, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

// write n words to (host) memory, then publish a flag with a system-scope release
__global__ void publish_kernel(const uint64_t* src, uint64_t* dst, int n, uint32_t* flag, uint32_t value) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class F>
double time_us(F f, int reps = 200) {
    for (int i = 0; i < 20; ++i) f();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
    const int k = 1024;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint64_t *d_src, *d_dst, *h_pin, *h_coh;
    uint32_t* flag;
    CK(hipMalloc(&d_src, k * 8));
    CK(hipMalloc(&d_dst, k * 8));
    CK(hipMemset(d_src, 1, k * 8));
    CK(hipHostMalloc(&h_pin, k * 8, hipHostMallocDefault));
    CK(hipHostMalloc(&h_coh, k * 8, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    *flag = 0;

    printf("empty launch + streamSync            %7.2f us\n", time_us([&] {
               empty_kernel<<<1, 64, 0, s>>>();
               (void)hipStreamSynchronize(s);
           }));
    printf("empty launch + event record/sync     %7.2f us\n", time_us([&] {
               empty_kernel<<<1, 64, 0, s>>>();
               (void)hipEventRecord(ev, s);
               (void)hipEventSynchronize(ev);
           }));
    printf("3 launches + streamSync              %7.2f us\n", time_us([&] {
               empty_kernel<<<1, 64, 0, s>>>();
               empty_kernel<<<1, 64, 0, s>>>();
               empty_kernel<<<1, 64, 0, s>>>();
               (void)hipStreamSynchronize(s);
           }));
    printf("memset 8KB + 2 launches + streamSync %7.2f us\n", time_us([&] {
               (void)hipMemsetAsync(d_dst, 0, k * 8, s);
               empty_kernel<<<1, 64, 0, s>>>();
               empty_kernel<<<1, 64, 0, s>>>();
               (void)hipStreamSynchronize(s);
           }));
    printf("kernel + D2H 8KB pinned + streamSync %7.2f us\n", time_us([&] {
               copy_kernel<<<1, 256, 0, s>>>(d_src, d_dst, k);
               (void)hipMemcpyAsync(h_pin, d_dst, k * 8, hipMemcpyDeviceToHost, s);
               (void)hipStreamSynchronize(s);
           }));
    printf("D2H 8KB pinned + streamSync          %7.2f us\n", time_us([&] {
               (void)hipMemcpyAsync(h_pin, d_dst, k * 8, hipMemcpyDeviceToHost, s);
               (void)hipStreamSynchronize(s);
           }));
    uint32_t gen = 0;
    printf("kernel -> coherent host + flag spin  %7.2f us\n", time_us([&] {
               ++gen;
               publish_kernel<<<1, 256, 0, s>>>(d_src, h_coh, k, flag, gen);
               while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen) {
               }
           }));
    printf("kernel -> coherent host + streamSync %7.2f us\n", time_us([&] {
               ++gen;
               publish_kernel<<<1, 256, 0, s>>>(d_src, h_coh, k, flag, gen);
               (void)hipStreamSynchronize(s);
           }));
    printf("2 empty + publish + flag spin        %7.2f us\n", time_us([&] {
               ++gen;
               empty_kernel<<<1, 64, 0, s>>>();
               empty_kernel<<<1, 64, 0, s>>>();
               publish_kernel<<<1, 256, 0, s>>>(d_src, h_coh, k, flag, gen);
               while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != gen) {
               }
           }));
    CK(hipStreamSynchronize(s));
    // correctness of the published copy
    int bad = 0;
    for (int i = 0; i < k; ++i) bad += h_coh[i] != 0x0101010101010101ull;
    printf("published words wrong: %d\n", bad);
    return 0;
}
