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
#include <algorithm>
#include <cstdlib>

#include "rsv_internal.h"
#include "rsv_k2.h"

namespace rsv {

using namespace k2;

namespace {
// global winner tables (k > 4416): scratch of k * 8 bytes per wave, at most this much per launch
constexpr size_t kGtabBudget = 1ull << 30;
}  // namespace

hipError_t launch_segmented(const void* keys, int key_width, const int64_t* offsets, int64_t S, uint32_t k,
                            const DrawParams& dp, void* out, int64_t* counts, hipStream_t st) {
    if (S <= 0) return hipSuccess;
    const uint64_t blocks = ((uint64_t)S + kWaves - 1) / kWaves;
    if (k2::lds_bytes(k) > k2::kLdsMax) {
        // large k: the same kernel with each wave's k-slot table in global scratch (zeroed once;
        // every stream leaves its slice zero again).  Grid: up to 16 workgroups per CU, fewer when
        // their tables would pass kGtabBudget (k = 65536: 512 workgroups, 1 GiB)
        const size_t per_wg = (size_t)kWaves * k * 8;
        const uint64_t cap = std::max<uint64_t>(1, kGtabBudget / per_wg);
        const unsigned grid = (unsigned)std::min<uint64_t>(std::min<uint64_t>(blocks, cap), 256ull * 16);
        const size_t bytes = (size_t)grid * per_wg;
        unsigned long long* gtab = nullptr;
        hipError_t e = hipMallocAsync((void**)&gtab, bytes, st);
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(gtab, 0, bytes, st);
        const uint32_t k0 = (uint32_t)dp.seed, k1 = (uint32_t)(dp.seed >> 32);
        const size_t lds = k2::lds_bytes(k, 0, true);
        if (e == hipSuccess) {
            if (key_width == 8)
                hipLaunchKernelGGL((k2_segmented<int64_t, 0, true>), dim3(grid), dim3(64 * kWaves), lds, st,
                                   (const int64_t*)keys, offsets, S, k, k0, k1, dp.stream, (int64_t*)out, counts,
                                   k2::kQCap, gtab);
            else
                hipLaunchKernelGGL((k2_segmented<int32_t, 0, true>), dim3(grid), dim3(64 * kWaves), lds, st,
                                   (const int32_t*)keys, offsets, S, k, k0, k1, dp.stream, (int32_t*)out, counts,
                                   k2::kQCap, gtab);
            e = hipGetLastError();
        }
        const hipError_t e2 = hipFreeAsync(gtab, st);
        return e != hipSuccess ? e : e2;
    }
    const size_t lds = k2::lds_bytes(k);
    const uint32_t k0 = (uint32_t)dp.seed, k1 = (uint32_t)(dp.seed >> 32);
    // up to 128 four-wave workgroups per CU over the launch (C3: 8 streams per wave): tools/micro_k2 G
    // (r03ai) 1.78 ms at 4096 workgroups, 1.71 at 16384, 1.65 at 32768, 1.66-1.68 at 65536, 1.84 at
    // one stream per wave (262144: every workgroup rebuilds the threshold table)
    const unsigned grid = (unsigned)std::min<uint64_t>(blocks, 256ull * 128);
    // RSV_K2_FIFO_CAP (tests, read once per process): a lower bulk-append limit, so the ballot-
    // round overflow path runs
    static const uint32_t fifo_cap = [] {
        const char* e = std::getenv("RSV_K2_FIFO_CAP");
        return e ? (uint32_t)std::atoi(e) : k2::kQCap;
    }();
    if (key_width == 8)
        hipLaunchKernelGGL(k2_segmented<int64_t>, dim3(grid), dim3(64 * kWaves), lds, st, (const int64_t*)keys,
                           offsets, S, k, k0, k1, dp.stream, (int64_t*)out, counts, fifo_cap);
    else
        hipLaunchKernelGGL(k2_segmented<int32_t>, dim3(grid), dim3(64 * kWaves), lds, st, (const int32_t*)keys,
                           offsets, S, k, k0, k1, dp.stream, (int32_t*)out, counts, fifo_cap);
    return hipGetLastError();
}

}  // namespace rsv
