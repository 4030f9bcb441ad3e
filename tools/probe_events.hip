// probe_events.hip -- what timing a kernel with HIP events costs the stream it runs on
// (development probe).  A ~130 us all-CU VALU kernel, then a tiny kernel, then a host round trip,
// per step; variants differ only in how the big kernel is timed.
// hipcc --offload-arch=gfx950 -O3 tools/probe_events.hip -o tools/probe_events
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

__global__ void busy_kernel(uint32_t iters, uint32_t* out) {
    uint32_t a = threadIdx.x, b = blockIdx.x;
    for (uint32_t i = 0; i < iters; ++i) {
        a = a * 0x9E3779B9u + b;
        b ^= a >> 7;
    }
    if (a == 0x12345678u && b == 0) out[0] = a;
}
__global__ void tiny_kernel(uint32_t* out) {
    if (threadIdx.x == 1000000) out[0] = 1;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* d;
    CK(hipMalloc(&d, 64));
    const unsigned flagsets[] = {hipEventDefault, hipEventDisableSystemFence, hipEventReleaseToDevice};
    const char* fnames[] = {"default", "DisableSystemFence", "ReleaseToDevice"};
    const uint32_t iters = 900;
    auto run = [&](int mode, unsigned ef, double& step_us, double& k_us) -> int {
        hipEvent_t e0[64], e1[64];
        for (int i = 0; i < 64; ++i) {
            CK(hipEventCreateWithFlags(&e0[i], ef));
            CK(hipEventCreateWithFlags(&e1[i], ef));
        }
        double tot_ms = 0;
        auto one = [&](int i) {
            if (mode == 0) {
                hipLaunchKernelGGL(busy_kernel, dim3(8192), dim3(256), 0, s, iters, d);
            } else if (mode == 1) {
                (void)hipEventRecord(e0[i], s);
                hipLaunchKernelGGL(busy_kernel, dim3(8192), dim3(256), 0, s, iters, d);
                (void)hipEventRecord(e1[i], s);
            } else if (mode == 2) {
                hipExtLaunchKernelGGL(busy_kernel, dim3(8192), dim3(256), 0, s, e0[i], e1[i], 0, iters, d);
            } else {  // start event on the big kernel, stop event = start of the next (tiny) kernel
                hipExtLaunchKernelGGL(busy_kernel, dim3(8192), dim3(256), 0, s, e0[i], nullptr, 0, iters, d);
            }
            if (mode == 3)
                hipExtLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s, e1[i], nullptr, 0, d);
            else
                hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s, d);
            (void)hipStreamSynchronize(s);
        };
        for (int i = 0; i < 64; ++i) one(i);
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 64; ++i) one(i);
        auto t1 = std::chrono::steady_clock::now();
        if (mode) {
            for (int i = 0; i < 64; ++i) {
                float ms;
                CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
                tot_ms += ms;
            }
        }
        step_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / 64;
        k_us = tot_ms * 1e3 / 64;
        for (int i = 0; i < 64; ++i) {
            (void)hipEventDestroy(e0[i]);
            (void)hipEventDestroy(e1[i]);
        }
        return 0;
    };
    const char* mnames[] = {"no events", "hipEventRecord x2", "hipExtLaunch start+stop", "ext start, stop on next"};
    for (int rep = 0; rep < 3; ++rep)
        for (int m = 0; m < 4; ++m)
            for (int f = 0; f < (m ? 3 : 1); ++f) {
                double st, ku;
                if (run(m, flagsets[f], st, ku)) return 1;
                printf("%-26s %-20s step %8.2f us  timed %8.2f us\n", mnames[m], m ? fnames[f] : "-", st, ku);
            }
    return 0;
}
