// rsv_segmented.hip -- K2: S independent Algorithm-R samplers per launch (rsv_sample_segmented), one
// wave per stream; the reference counterpart is S separate Sampler instances (Sampler.scala:196-332).
//
// Work per stream of n elements (draw format R2, rsv_device.h): one level-0 Philox per 16-index block
// of [k, n) and one level-1 Philox per index whose level-0 byte leaves j_i < k possible
// (b_i (i+1) < 256 k).  At C3's shape (4096 elements, k = 64) every block is in the dense region: the
// candidates (~270 per stream, 9/10 of them real hits) crowd the head -- the first block holds ~15 of
// its 16 indices, the last ~0.1.
//
// Per iteration the wave evaluates 64 level-0 blocks (one per lane, Philox with the counter's high
// words wave-uniform), takes each block's candidate mask with a bit-sliced compare b < T (T from the
// block's first index), and appends the candidates -- 16-bit references (ring slot, lane, byte) into
// the block words it stashed in LDS -- to a per-wave FIFO at offsets from ONE wave prefix sum of the
// per-lane counts (5 ballots).  Whenever 64 candidates wait, every lane resolves one: it decodes its
// byte from the stashed block, runs the level-1 Philox and, on a hit, takes an LDS atomicMax on the
// stream's k-slot last-writer table.  (The previous form pushed candidates one per lane per ballot
// round and decoded the byte inside the round: ~1700 wave-instructions per C3 stream, PMC
// SQ_INSTS_VALU; this form ~4x fewer)  The winners' keys are gathered at the end.
//
// k >= 512 (k2::kWGMinK): one WORKGROUP of 8 waves per stream with one shared winner table
// (k2_segmented_wg, rsv_k2.h) -- per-wave tables would leave a CU one or two workgroups, and beyond
// k = 4416 not fit at all.  The table is u32 when the streams span < 2^32 elements (the host reads
// offsets[0] and offsets[S] once), in LDS while it fits beside the waves' rings (k <= ~29.5k), else
// the workgroup's slice of a per-device global scratch that is zeroed once and left zero by every
// launch -- no allocation or fill per call.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "rsv_internal.h"
#include "rsv_k2.h"

namespace rsv {

using namespace k2;

namespace {
#define RSV_HIP_RET(expr)                      \
    do {                                       \
        const hipError_t _e = (expr);          \
        if (_e != hipSuccess) return _e;       \
    } while (0)

// The workgroup form's global tables (k too large for LDS): one scratch per device, zeroed ONCE when
// allocated and left zero by every launch (its gather swaps each entry back to 0), reused by the next
// launch on the same stream, or on any stream once the last launch's event has completed; a launch
// that finds it busy on another stream takes a private zeroed block instead.
struct GtScratch {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
};
std::mutex g_gt_mu;
GtScratch g_gt[64];

hipError_t gt_acquire(int dev, size_t bytes, hipStream_t st, void** out, bool* priv) {
    GtScratch& c = g_gt[dev & 63];
    *priv = false;
    const bool idle = !c.p || c.st == st || !c.done || hipEventQuery(c.done) == hipSuccess;
    if (c.p && idle && bytes <= c.bytes) {
        *out = c.p;
        return hipSuccess;
    }
    if (!idle) {  // another stream's launch may still use it
        *priv = true;
        hipError_t e = hipMallocAsync(out, bytes, st);
        return e == hipSuccess ? hipMemsetAsync(*out, 0, bytes, st) : e;
    }
    if (c.p) {  // idle but too small: replaced (its last user finished or is this stream)
        hipError_t e = hipStreamSynchronize(st);
        if (e == hipSuccess) e = hipFree(c.p);
        c.p = nullptr;
        c.bytes = 0;
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipMalloc(&c.p, bytes);
    if (e != hipSuccess) return e;
    c.bytes = bytes;
    *out = c.p;
    return hipMemsetAsync(c.p, 0, bytes, st);
}

void gt_release(int dev, hipStream_t st, bool priv, void* p) {
    if (priv) {
        (void)hipFreeAsync(p, st);
        return;
    }
    GtScratch& c = g_gt[dev & 63];
    if (!c.done && hipEventCreateWithFlags(&c.done, hipEventDisableTiming) != hipSuccess) c.done = nullptr;
    if (c.done) (void)hipEventRecord(c.done, st);
    c.st = st;
}

template <typename KeyT, typename TabT>
hipError_t launch_wg(const KeyT* keys, const int64_t* offsets, int64_t S, uint32_t k, const DrawParams& dp,
                     KeyT* out, int64_t* counts, hipStream_t st, uint32_t fifo_cap) {
    const uint32_t k0 = (uint32_t)dp.seed, k1 = (uint32_t)(dp.seed >> 32);
    const size_t lds = k2::lds_bytes_wg(k, sizeof(TabT), false);
    if (lds <= k2::kLdsMax) {
        // as many workgroups as the CUs hold at once, twice over (streams are taken grid-stride)
        const uint64_t per_cu = std::max<uint64_t>(1, k2::kLdsMax / lds);
        const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)S, 256ull * per_cu * 2);
        hipLaunchKernelGGL((k2_segmented_wg<KeyT, TabT, false>), dim3(grid), dim3(64 * kWavesWG), lds, st, keys,
                           offsets, S, k, k0, k1, dp.stream, out, counts, fifo_cap, (TabT*)nullptr);
        return hipGetLastError();
    }
    int dev = 0;
    RSV_HIP_RET(hipGetDevice(&dev));
    const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)S, 512);
    const size_t bytes = (size_t)grid * k * sizeof(TabT);
    std::lock_guard<std::mutex> lk(g_gt_mu);
    void* gt = nullptr;
    bool priv = false;
    RSV_HIP_RET(gt_acquire(dev, bytes, st, &gt, &priv));
    hipLaunchKernelGGL((k2_segmented_wg<KeyT, TabT, true>), dim3(grid), dim3(64 * kWavesWG),
                       k2::lds_bytes_wg(k, sizeof(TabT), true), st, keys, offsets, S, k, k0, k1, dp.stream, out,
                       counts, fifo_cap, (TabT*)gt);
    const hipError_t e = hipGetLastError();
    gt_release(dev, st, priv, gt);
    return e;
}
}  // namespace

hipError_t launch_segmented(const void* keys, int key_width, const int64_t* offsets, int64_t S, uint32_t k,
                            const DrawParams& dp, void* out, int64_t* counts, hipStream_t st) {
    if (S <= 0) return hipSuccess;
    // RSV_K2_FIFO_CAP (tests, read once per process): a lower bulk-append limit, so the ballot-
    // round overflow path runs
    static const uint32_t fifo_cap = [] {
        const char* e = std::getenv("RSV_K2_FIFO_CAP");
        return e ? (uint32_t)std::atoi(e) : k2::kQCap;
    }();
    if (k >= k2::kWGMinK) {  // one workgroup per stream
        // every index fits 32 bits when the streams together span < 2^32 elements: u32 tables
        int64_t ends[2] = {0, 0};
        RSV_HIP_RET(hipMemcpyAsync(&ends[0], offsets, 8, hipMemcpyDeviceToHost, st));
        RSV_HIP_RET(hipMemcpyAsync(&ends[1], offsets + S, 8, hipMemcpyDeviceToHost, st));
        RSV_HIP_RET(hipStreamSynchronize(st));
        const bool t32 = ends[1] - ends[0] < ((int64_t)1 << 32);
        if (key_width == 8)
            return t32 ? launch_wg<int64_t, uint32_t>((const int64_t*)keys, offsets, S, k, dp, (int64_t*)out, counts, st, fifo_cap)
                       : launch_wg<int64_t, unsigned long long>((const int64_t*)keys, offsets, S, k, dp, (int64_t*)out,
                                                                counts, st, fifo_cap);
        return t32 ? launch_wg<int32_t, uint32_t>((const int32_t*)keys, offsets, S, k, dp, (int32_t*)out, counts, st, fifo_cap)
                   : launch_wg<int32_t, unsigned long long>((const int32_t*)keys, offsets, S, k, dp, (int32_t*)out,
                                                            counts, st, fifo_cap);
    }
    const size_t lds = k2::lds_bytes(k);
    const uint32_t k0 = (uint32_t)dp.seed, k1 = (uint32_t)(dp.seed >> 32);
    // up to 128 four-wave workgroups per CU over the launch (C3: 8 streams per wave): tools/micro_k2 G
    // (r03ai) 1.78 ms at 4096 workgroups, 1.71 at 16384, 1.65 at 32768, 1.66-1.68 at 65536, 1.84 at
    // one stream per wave (262144: every workgroup rebuilds the threshold table)
    const uint64_t blocks = ((uint64_t)S + kWaves - 1) / kWaves;
    const unsigned grid = (unsigned)std::min<uint64_t>(blocks, 256ull * 128);
    if (key_width == 8)
        hipLaunchKernelGGL(k2_segmented<int64_t>, dim3(grid), dim3(64 * kWaves), lds, st, (const int64_t*)keys,
                           offsets, S, k, k0, k1, dp.stream, (int64_t*)out, counts, fifo_cap);
    else
        hipLaunchKernelGGL(k2_segmented<int32_t>, dim3(grid), dim3(64 * kWaves), lds, st, (const int32_t*)keys,
                           offsets, S, k, k0, k1, dp.stream, (int32_t*)out, counts, fifo_cap);
    return hipGetLastError();
}

}  // namespace rsv
