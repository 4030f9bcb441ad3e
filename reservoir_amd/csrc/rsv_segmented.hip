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

size_t segmented_lds_bytes(uint32_t k) { return k2::lds_bytes(k); }

hipError_t launch_segmented_v1(const void* keys, int key_width, const int64_t* offsets, int64_t S, uint32_t k,
                               const DrawParams& dp, void* out, int64_t* counts, hipStream_t st);

hipError_t launch_segmented(const void* keys, int key_width, const int64_t* offsets, int64_t S, uint32_t k,
                            const DrawParams& dp, void* out, int64_t* counts, hipStream_t st) {
    if (S <= 0) return hipSuccess;
    // RSV_K2=1 keeps the round-1 kernel (A/B measurements); it also serves tables too big for
    // four waves' LDS here
    static const int form = [] {
        const char* e = std::getenv("RSV_K2");
        return e ? std::atoi(e) : 0;
    }();
    const size_t lds = segmented_lds_bytes(k);
    if (form == 1 || lds > 160 * 1024) return launch_segmented_v1(keys, key_width, offsets, S, k, dp, out, counts, st);
    const uint32_t k0 = (uint32_t)dp.seed, k1 = (uint32_t)(dp.seed >> 32);
    const uint64_t blocks = ((uint64_t)S + kWaves - 1) / kWaves;
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
